"""FETCH_SIZE calibration summary (measurement tool): reads the rocprofv3
--pmc FETCH_SIZE (and WRITE_SIZE) passes of tools/fetch_calib and writes
profiles/<tag>_fetch_calib.json -- per access width, the counter against the
bytes the kernel provably read (each byte of a 1 GiB buffer once).

    python tools/fetch_calib.py <tag>      (reads gpurun_out/fetch_calib_<tag>/)
"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    tag = sys.argv[1]
    src = os.path.join(ROOT, "gpurun_out", "fetch_calib_" + tag)
    bytes_ = 1 << 30
    rows = {}
    for f in glob.glob(os.path.join(src, "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for r in csv.DictReader(fh):
                name = r.get("Kernel_Name", "")
                if "read_all" not in name:
                    continue
                w = "4B" if "read_all<float>" in name else ("8B" if "read_all<double>" in name else "16B")
                rows.setdefault(w, {})[r["Counter_Name"]] = float(r["Counter_Value"])
    out = {"bytes_read_per_kernel": bytes_, "widths": {}}
    for w, c in sorted(rows.items()):
        fk = c.get("FETCH_SIZE")
        out["widths"][w] = {"FETCH_SIZE_KiB": fk, "FETCH_SIZE_bytes": fk * 1024 if fk else None,
                            "ratio_raw": fk * 1024 / bytes_ if fk else None,
                            "ratio_x2": 2 * fk * 1024 / bytes_ if fk else None}
    out["note"] = ("read_all<T> reads every byte of a 1 GiB buffer once (8 x 4 MB of L2: every line misses); "
                   "ratio_x2 = 2 x FETCH_SIZE x 1024 / bytes read, the correction tools/pmc_summary.py applies")
    with open(os.path.join(ROOT, "profiles", tag + "_fetch_calib.json"), "w") as fh:
        json.dump(out, fh, indent=1)
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
