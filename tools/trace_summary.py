"""Per-kernel launch count / average / median duration from a rocprofv3 --kernel-trace CSV
(kernel symbols shortened, templates folded onto the timing ids of include/indy7_mpc.h).

    python tools/trace_summary.py RUN_kernel_trace.csv [--batch B --N N] > profiles/rNN_kernel_trace_summary.json

With --batch, only launches of that batch size count (grid B*64 for the per-problem kernels, B/4*64
for k_admm_iter,
ceil(B*N/10)*64 for k_linearize): bench.py also runs B = 1 and host-to-host solves.
"""
import collections
import csv
import json
import re
import statistics
import sys


def kernel_name(full):
    """Short kernel name from the demangled symbol (also for kernels in an anonymous namespace,
    e.g. `void (anonymous namespace)::i7m::k_linearize<true>(...)`)."""
    m = re.search(r"\b(k_[A-Za-z0-9_]+)", full)
    return m.group(1) if m else full.split("(")[0].split("<")[0].split("::")[-1]

CANON = {"k_riccati_mfma": "k_riccati"}


def main(path, batch=None, N=32):
    d = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        name = kernel_name(r["Kernel_Name"])
        name = CANON.get(name, name)
        if batch is not None and name.startswith("k_"):
            grid = int(r.get("Grid_Size_X", r.get("Grid_Size", 0)) or 0)
            want = (-(-batch * N // 10) * 64 if name == "k_linearize"
                    else -(-batch // 4) * 64 if name == "k_admm_iter"  # (four problems per wave)
                    else batch * 64)
            if grid != want:
                continue
        d[name].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    out = {k: {"launches": len(v), "avg_us": statistics.mean(v), "median_us": statistics.median(v)} for k, v in d.items()}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    import argparse
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("--batch", type=int)
    ap.add_argument("--N", type=int, default=32)
    a = ap.parse_args()
    main(a.trace, a.batch, a.N)
