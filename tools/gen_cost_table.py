"""Extract the reference's distance table (pastar/Cost.cpp:12-262) as data.

Run once in the build container (the reference is absent on the GPU box); the
output `tests/golden/cost_table.json` is a fixture: every (row, col, value)
assignment the reference's Cost constructor performs, as a sparse map keyed
by the two residue characters. Unassigned entries are zero (Cost.cpp:10).
"""
import json, re, sys, pathlib

src = pathlib.Path(sys.argv[1] if len(sys.argv) > 1 else
                   "/root/reference/pastar/Cost.cpp").read_text()
names = {"DASH": "-"}
cells = {}
for line in src.splitlines():
    line = line.strip()
    if not line.startswith("pam250["):
        continue
    val = int(re.search(r"=\s*(-?\d+)\s*;", line).group(1))
    for a, b in re.findall(r"pam250\[(\w+)\]\[(\w+)\]", line):
        ra, rb = names.get(a, a), names.get(b, b)
        cells[ra + rb] = val
out = pathlib.Path(__file__).resolve().parents[1] / "tests/golden/cost_table.json"
out.write_text(json.dumps({"source": "pastar/Cost.cpp:12-262", "cells": cells},
                          indent=0, sort_keys=True) + "\n")
print(len(cells), "cells ->", out)
