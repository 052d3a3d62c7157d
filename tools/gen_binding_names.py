"""Writes tests/golden/bindings_names.json: every Python class and method name
the reference's Boost.Python module registers (src/bindings.cpp:219-447),
read from the reference source in the build container (API surface only)."""
import json
import os
import re

REF = "/root/reference/src/bindings.cpp"
OUT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden", "bindings_names.json")


def parse(path):
    names, cls = {}, None
    for line in open(path):
        m = re.search(r'class_<[^>]*(?:<[^>]*>[^>]*)*>\s*\(\s*"(\w+)"', line)
        if m:
            cls = m.group(1)
            names.setdefault(cls, [])
            continue
        m = re.search(r'\.def\(\s*"(\w+)"', line)
        if m and cls:
            if m.group(1) not in names[cls]:
                names[cls].append(m.group(1))
        m = re.search(r'\.(?:def_readwrite|add_property)\(\s*"(\w+)"', line)
        if m and cls and m.group(1) not in names[cls]:
            names[cls].append(m.group(1))
    return names


if __name__ == "__main__":
    names = parse(REF)
    with open(OUT, "w") as fh:
        json.dump(names, fh, indent=1, sort_keys=True)
    print(sum(len(v) for v in names.values()), "names in", len(names), "classes ->", OUT)
