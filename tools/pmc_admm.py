"""Per-kernel SQ counters of rocprofv3 --pmc passes (csv), summed over the launches of each kernel,
with per-wave ratios: python tools/pmc_admm.py OUT1/..._counter_collection.csv [more.csv ...]"""
import collections
import csv
import json
import re
import sys

acc = collections.defaultdict(lambda: collections.defaultdict(float))
for path in sys.argv[1:]:
    for r in csv.DictReader(open(path)):
        m = re.search(r"\b(k_[A-Za-z0-9_]+)", r["Kernel_Name"])
        name = m.group(1) if m else r["Kernel_Name"][:40]
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
        acc[name]["_rows"] += 1
out = {}
for k, d in acc.items():
    w = d.get("SQ_WAVES", 0) or 1
    cyc = d.get("SQ_WAVE_CYCLES", 0) or 1
    e = {c: v for c, v in d.items() if not c.startswith("_")}
    e["per_wave"] = {c: v / w for c, v in d.items() if c.startswith("SQ_INSTS") or c.startswith("SQ_WAVE_CYCLES")}
    e["frac_of_wave_cycles"] = {c: v / cyc for c, v in d.items() if c.startswith(("SQ_WAIT", "SQ_ACTIVE"))}
    out[k] = e
print(json.dumps(out, indent=1))
