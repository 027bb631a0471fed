"""Fold rocprofv3 PMC passes (FETCH_SIZE, WRITE_SIZE; separate runs) into
profiles/pmc_traffic.json: HBM bytes per launch of each kernel, corrected as
/opt/skills/guides/MI355X_MICROARCH.md §HBM prescribes (FETCH_SIZE and WRITE_SIZE are in KiB;
gfx950 FETCH_SIZE reads 1/2 of a wide coalesced read -> x2).

    python tools/pmc_traffic.py FETCH_CSV WRITE_CSV --batch 4096 --N 32 [--out profiles/pmc_traffic.json]
Launches of the timed batch size only (grid size identifies them); median over launches of the
first SQP iteration (all problems active) is reported.  --admm-stagger: k_admm_iter's launches of
ADMM mode's two staggered ranges (batch / 2 problems each, both SQP iterations), MEAN over every
such launch — the per-launch average bench.py's event pass reports beside it — under the key
k_admm_iter:B<batch/2>:N<N>:stagger.
"""
import argparse
import collections
import csv
import json
import os
import re
import statistics


def kernel_name(full):
    """Short kernel name from the demangled symbol (also for kernels in an anonymous namespace,
    e.g. `void (anonymous namespace)::i7m::k_linearize<true>(...)`)."""
    m = re.search(r"\b(k_[A-Za-z0-9_]+)", full)
    return m.group(1) if m else full.split("(")[0].split("<")[0].split("::")[-1]


# kernel symbol -> the timing id bench.py reports (include/indy7_mpc.h I7M_K_*)
CANON = {"k_riccati_mfma": "k_riccati"}


def per_kernel(path, counter):
    vals = collections.defaultdict(list)
    for r in csv.DictReader(open(path)):
        if r.get("Counter_Name") != counter:
            continue
        name = kernel_name(r["Kernel_Name"])
        name = CANON.get(name, name)
        grid = int(r.get("Grid_Size", r.get("Grid_Size_X", 0)) or 0)
        vals[(name, grid)].append(float(r["Counter_Value"]))
    return vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("fetch")
    ap.add_argument("write")
    ap.add_argument("--batch", type=int, default=4096)
    ap.add_argument("--N", type=int, default=32)
    ap.add_argument("--out", default=os.path.join(os.path.dirname(__file__), "..", "profiles", "pmc_traffic.json"))
    ap.add_argument("--admm-stagger", action="store_true")
    a = ap.parse_args()
    f = per_kernel(a.fetch, "FETCH_SIZE")
    w = per_kernel(a.write, "WRITE_SIZE")
    grids = {"k_linearize": -(-a.batch * a.N // 10) * 64, "k_riccati": a.batch * 64, "k_linesearch": a.batch * 64,
             "k_ipm_fused": a.batch * 64, "k_sqp_fused": a.batch * 64, "k_admm_iter": -(-a.batch // 4) * 64,
             "k_admm_scale": a.batch * 64, "k_admm_factor": a.batch * 64}
    try:
        d = json.load(open(a.out))
    except (OSError, ValueError):
        d = {}
    for k, g in grids.items():
        gg = [key for key in f if key[0] == k and abs(key[1] - g) <= 256]
        if not gg:
            continue
        fv = f[gg[0]]
        wv = w.get(gg[0], [0.0])
        # launches alternate iteration 1 / iteration 2 of each solve: take iteration-1 launches
        f1, w1 = fv[0::2], wv[0::2]
        fetch_b = 2.0 * 1024.0 * statistics.median(f1)
        write_b = 1024.0 * statistics.median(w1)
        d[f"{k}:B{a.batch}:N{a.N}"] = {"hbm_bytes_per_launch": fetch_b + write_b, "fetch_bytes_corrected": fetch_b,
                                       "write_bytes": write_b, "fetch_kib_raw_median": statistics.median(f1),
                                       "launches": len(fv)}
    if a.admm_stagger:
        hb = a.batch // 2
        g = -(-hb // 4) * 64
        gg = [key for key in f if key[0] == "k_admm_iter" and key[1] == g]
        if gg:
            fv, wv = f[gg[0]], w.get(gg[0], [0.0])
            fetch_b = 2.0 * 1024.0 * statistics.mean(fv)
            write_b = 1024.0 * statistics.mean(wv)
            d[f"k_admm_iter:B{hb}:N{a.N}:stagger"] = {
                "hbm_bytes_per_launch": fetch_b + write_b, "fetch_bytes_corrected": fetch_b, "write_bytes": write_b,
                "fetch_kib_raw_mean": statistics.mean(fv), "launches": len(fv),
                "fetch_kib_raw_per_launch": fv, "write_kib_per_launch": wv,
                "note": "mean over every launch of the staggered ranges (both SQP iterations)"}
    os.makedirs(os.path.dirname(a.out), exist_ok=True)
    json.dump(d, open(a.out, "w"), indent=1)
    print(json.dumps(d, indent=1))


if __name__ == "__main__":
    main()
