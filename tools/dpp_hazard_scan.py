"""Static scan of the built library's gfx950 code for the DPP hazard of
`tools/probes/rowsplit_probe.hip` (`profiles/r06zi_dpp_shrinking_bank_mask_probe.json`): a DPP
fma whose row or bank mask leaves lanes out, accumulating into a register the VALU wrote within the
two wait states before it — the masked-out lanes then get back the accumulator as it was before
that write.  The kernels' dot products keep a chain's fma's four instructions apart; this scan
checks that no build puts two closer (inline asm gets no hazard nops from the compiler).

    python tools/dpp_hazard_scan.py [lib.so]        -> JSON: DPP fma's seen, hazards found
"""
from __future__ import annotations

import json
import os
import re
import subprocess
import sys
import tempfile

LLVM = "/opt/rocm/lib/llvm/bin"
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
_REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)")


def _regs(op: str):
    m = _REG.fullmatch(op.strip())
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def _code_objects(lib: str, td: str):
    # the bundles are written next to the input: extract from a copy in the scratch directory
    import shutil
    cp = os.path.join(td, os.path.basename(lib))
    shutil.copyfile(lib, cp)
    subprocess.run([os.path.join(LLVM, "llvm-objdump"), "--offloading", cp], cwd=td, check=True,
                   capture_output=True)
    return sorted(os.path.join(td, f) for f in os.listdir(td) if "gfx950" in f)


def scan_text(asm: str):
    """Over objdump output: the DPP fma's with a partial mask, their hazards as (function, line),
    and DPP reads of a source the VALU wrote within two wait states (the compiler's own guard)."""
    seen, hazards, src_hazards, func = 0, [], [], "?"
    recent = []  # (wait states since, registers written) of the last VALU writes
    for line in asm.splitlines():
        s = line.split("//")[0].strip()
        if s.endswith(">:"):
            func, recent = s[s.find("<") + 1:-2], []
            continue
        if not s or s.endswith(":"):
            continue
        w = s.split(None, 1)
        op, args = w[0], (w[1] if len(w) > 1 else "")
        if op == "s_nop":
            n = int(args.split()[0], 0) + 1
            recent = [(d + n, r) for d, r in recent]
            continue
        ops = [a for a in args.split(",")]
        if "_dpp" in op and len(ops) > 1 and any(d < 2 and (r & _regs(ops[1].split()[0])) for d, r in recent):
            src_hazards.append((func, s))  # the documented one: a DPP source the VALU just wrote
        if op.startswith("v_fmac_f64_dpp") or (op.startswith("v_fmac_") and "_dpp" in op):
            masks = dict(re.findall(r"(row_mask|bank_mask):(0x[0-9a-f]+)", args))
            partial = masks.get("row_mask", "0xf") != "0xf" or masks.get("bank_mask", "0xf") != "0xf"
            dst = _regs(ops[0].split()[0]) if ops else set()
            if partial:
                seen += 1
                if any(d < 2 and (r & dst) for d, r in recent):
                    hazards.append((func, s))
        recent = [(d + 1, r) for d, r in recent if d + 1 < 2]
        if op.startswith("v_") and ops:
            r = _regs(ops[0].split()[0])
            if r:
                recent.append((0, r))
    return seen, hazards, src_hazards


def scan(lib: str):
    with tempfile.TemporaryDirectory() as td:
        seen, hazards, src = 0, [], []
        for co in _code_objects(lib, td):
            asm = subprocess.run([os.path.join(LLVM, "llvm-objdump"), "-d", "--mcpu=gfx950", co],
                                 check=True, capture_output=True, text=True).stdout
            s, h, hs = scan_text(asm)
            seen, hazards, src = seen + s, hazards + h, src + hs
    return {"lib": os.path.relpath(lib, ROOT), "partial_mask_dpp_fma": seen, "hazards": len(hazards),
            "first": hazards[:5], "dpp_source_hazards": len(src), "first_source": src[:5]}


if __name__ == "__main__":
    lib = sys.argv[1] if len(sys.argv) > 1 else os.path.join(ROOT, "indy7_mpc_amd", "lib", "libindy7mpc.so")
    r = scan(lib)
    print(json.dumps(r))
    sys.exit(1 if r["hazards"] else 0)
