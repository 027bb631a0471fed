"""Fold one rocprofv3 SQ-counter pass into per-kernel wave-state fractions.

    rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
        SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_LDS SQ_WAVES -- python tools/profile_kernels.py
    python tools/sq_summary.py OUT/sq_counter_collection.csv --batch 4096 --N 32

Per kernel (launches of the timed batch size only), summed over launches: fractions of wave
cycles spent issuing (ACTIVE_INST_ANY), parked on s_waitcnt (WAIT_ANY), waiting for an issue
slot (WAIT_INST_ANY), issuing VALU; VALU and LDS instructions per wave.  The wave-cycle counters
are per wave, so with w waves resident per SIMD the SIMD-level issue share is ~w x issuing_frac.
"""
import argparse
import collections
import csv
import json
import re


def kernel_name(full):
    """Short kernel name from the demangled symbol (also for kernels in an anonymous namespace,
    e.g. `void (anonymous namespace)::i7m::k_linearize<true>(...)`)."""
    m = re.search(r"\b(k_[A-Za-z0-9_]+)", full)
    return m.group(1) if m else full.split("(")[0].split("<")[0].split("::")[-1]

CANON = {"k_riccati_mfma": "k_riccati"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=32)
    a = ap.parse_args()
    acc = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open(a.csv)):
        name = kernel_name(r["Kernel_Name"])
        name = CANON.get(name, name)
        grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        want = -(-a.batch * a.N // 10) * 64 if name == "k_linearize" else a.batch * 64
        if name.startswith("k_") and abs(grid - want) > 256:
            continue
        acc[name][r["Counter_Name"]] += float(r["Counter_Value"])
    out = {}
    for k, c in acc.items():
        wc = c.get("SQ_WAVE_CYCLES", 0.0) or 1.0
        wv = c.get("SQ_WAVES", 0.0) or 1.0
        out[k] = {"issuing_frac": c.get("SQ_ACTIVE_INST_ANY", 0) / wc, "waitcnt_frac": c.get("SQ_WAIT_ANY", 0) / wc,
                  "issue_stall_frac": c.get("SQ_WAIT_INST_ANY", 0) / wc,
                  "valu_active_frac": c.get("SQ_ACTIVE_INST_VALU", 0) / wc,
                  "valu_insts_per_wave": c.get("SQ_INSTS_VALU", 0) / wv, "lds_insts_per_wave": c.get("SQ_INSTS_LDS", 0) / wv}
    print(json.dumps({"batch": a.batch, "N": a.N, "kernels": out}, indent=1))


if __name__ == "__main__":
    main()
