"""Compact per-kernel resource table (VGPRs, SGPRs, spills, scratch, LDS, occupancy) of the
library's translation units, from hipcc's -Rpass-analysis=kernel-resource-usage remarks.

    python tools/resource_usage.py [filter-substring ...] [--diag] [--unit=lin_tu]
"""
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import __graft_entry__ as ge  # noqa: E402

KEYS = ("VGPRs", "AGPRs", "TotalSGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize [bytes/lane]", "LDS Size [bytes/block]",
        "Occupancy [waves/SIMD]")


def demangle(names):
    try:
        out = subprocess.run(["c++filt"], input="\n".join(names), capture_output=True, text=True, check=True).stdout
        return out.splitlines()
    except (OSError, subprocess.CalledProcessError):
        return names


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    defines = ["-DI7M_DIAG"] if "--diag" in sys.argv else []
    unit = next((a.split("=", 1)[1] for a in sys.argv[1:] if a.startswith("--unit=")), "")
    extra_flags = next((a.split("=", 1)[1].split() for a in sys.argv[1:] if a.startswith("--flags=")), [])
    rows = []
    with tempfile.TemporaryDirectory() as td:
        for i, (src, extra) in enumerate(ge.LIB_UNITS):
            if unit not in os.path.basename(src):
                continue
            cmd = [ge.HIPCC, f"--offload-arch={ge.ARCH}", "-O3", "-std=c++17", "-fPIC", *extra, *defines, *extra_flags,
                   "-I" + os.path.join(ROOT, "include"), "-c", src, "-o", os.path.join(td, f"u{i}.o"),
                   "-Rpass-analysis=kernel-resource-usage"]
            err = subprocess.run(cmd, capture_output=True, text=True).stderr
            cur = None
            for line in err.splitlines():
                m = re.search(r"remark: ([^:]+): (.*?) \[-Rpass", line)
                if not m:
                    continue
                k, v = m.group(1).strip(), m.group(2)
                if k == "Function Name":
                    cur = {"name": v}
                    rows.append(cur)
                elif cur is not None and k in KEYS:
                    cur[k] = v
    names = demangle([r["name"] for r in rows])
    print(f"{'kernel':70s} {'VGPR':>5s} {'AGPR':>5s} {'SGPR':>5s} {'Vspill':>6s} {'Sspill':>6s} {'scr':>5s} {'LDS':>6s} {'occ':>4s}")
    for r, n in zip(rows, names):
        n = re.sub(r"\(.*", "", n.replace("(anonymous namespace)::", ""))
        if args and not any(a in n for a in args):
            continue
        print(f"{n[:70]:70s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} {r.get('TotalSGPRs', '?'):>5s} "
              f"{r.get('VGPRs Spill', '?'):>6s} {r.get('SGPRs Spill', '?'):>6s} {r.get('ScratchSize [bytes/lane]', '?'):>5s} "
              f"{r.get('LDS Size [bytes/block]', '?'):>6s} {r.get('Occupancy [waves/SIMD]', '?'):>4s}")


if __name__ == "__main__":
    main()
