"""Markdown rows of the end-of-round table from committed profiles:
    python tools/round_table.py <tag>
reads profiles/<tag>_<robot>_bench.json, _pmc.json and _valu.json for the five
BASELINE robots and prints one row per config plus the FR3 line's extras."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ROBOTS = [("fr3", "FR3 B = 65 536 (the metric)"), ("ur5e", "UR5e B = 65 536 (config 3)"),
          ("husky_fr3", "Husky-FR3 B = 16 384 (config 4)"), ("xls_fr3", "XLS-FR3 B = 65 536 per GPU (config 5 shard)"),
          ("caster_fr3", "Caster-FR3 B = 65 536")]
SIMDS, CLOCK = 1024, 2.4e9


def load(tag, robot, kind):
    with open(os.path.join(ROOT, "profiles", "%s_%s_%s.json" % (tag, robot, kind))) as fh:
        return json.load(fh)


def main():
    tag = sys.argv[1]
    for robot, label in ROBOTS:
        d, v = load(tag, robot, "bench"), load(tag, robot, "valu")
        c = d.get("cpu_baseline") or {}
        roof = SIMDS * CLOCK / v["valu_issue_cycles_per_solve"]
        ns = d["non_solved"]
        print("| %s | %.2f M | %.2f | %d / %d | %s | %.1f k / %.2f k | %.1f M (%.2f) |" % (
            label, d["value"] / 1e6, d["ms_per_step"], *d["admm_iters_p99_max"],
            ns if robot != "husky_fr3" else "%d (PrimalInfeasible)" % ns, c.get("value", 0) / 1e3,
            (c.get("single_thread") or {}).get("value", 0) / 1e3, roof / 1e6, d["value"] / roof))
    d, p = load(tag, "fr3", "bench"), load(tag, "fr3", "pmc")
    print("build", d["build_id"], "batch_4096", d.get("batch_4096", {}).get("value"), "latency_b1",
          {k: d["latency_b1"][k] for k in ("p50_us", "p99_us", "max_us")}, "latency_cycle",
          {k: d["latency_cycle"][k] for k in ("p50_us", "p99_us", "max_us")}, "reference_settings",
          d["reference_settings"]["value"], d["reference_settings"]["non_solved"])
    ro = d["roofline"]
    print("hbm achieved %.2f GB/s frac %.2e; fp64 alg %.2f TF frac %.4f; traffic %.0f MB/step %.0f B/solve"
          % (ro["achieved"], ro["frac"], ro["fp64_algorithmic"]["achieved_tflops"], ro["fp64_algorithmic"]["frac"],
             p["hbm_bytes_per_step"] / 1e6, p["hbm_bytes_per_instance"]))
    print("rocprof avg ns", p["main_dispatch_avg_ns"], "bench sums ms", ro["task_kernel_ms_sum"], ro["qp_kernel_ms_sum"])


if __name__ == "__main__":
    main()
