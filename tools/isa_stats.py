"""Instruction statistics of one kernel in a hipcc -S (device-only) assembly file: total
instructions, and counts of waits, LDS, barriers, scratch, MFMA, fp64 VALU, global memory.

    hipcc --offload-arch=gfx950 -O3 --offload-device-only -S ... -o x.s
    python tools/isa_stats.py x.s SUBSTRING_OF_MANGLED_NAME [...]
"""
import collections
import re
import sys


def kernel_bodies(text):
    for m in re.finditer(r"^(_Z\S+):\s*(;.*)?$", text, re.M):
        end = text.find("s_endpgm", m.end())
        yield m.group(1), text[m.end():end]


def stats(body):
    ops = collections.Counter()
    for line in body.splitlines():
        t = line.strip()
        if not t or t.startswith((".", ";")) or t.endswith(":"):
            continue
        ops[t.split()[0]] += 1
    groups = {
        "insts": sum(ops.values()),
        "s_waitcnt": sum(v for k, v in ops.items() if k.startswith("s_waitcnt")),
        "ds": sum(v for k, v in ops.items() if k.startswith("ds_")),
        "s_barrier": ops.get("s_barrier", 0),
        "scratch": sum(v for k, v in ops.items() if "scratch" in k or k.startswith("buffer_")),
        "mfma": sum(v for k, v in ops.items() if "mfma" in k),
        "valu_f64": sum(v for k, v in ops.items() if k.startswith("v_") and "f64" in k),
        "global": sum(v for k, v in ops.items() if k.startswith("global_")),
        "readlane": sum(v for k, v in ops.items() if "readlane" in k or "writelane" in k),
    }
    return groups


def main():
    path, pats = sys.argv[1], sys.argv[2:]
    text = open(path).read()
    for name, body in kernel_bodies(text):
        if all(p in name for p in pats):
            print(name[:90], stats(body))


if __name__ == "__main__":
    main()
