"""The vector-memory skeleton of one kernel in a hipcc -S (device-only) assembly file: its
s_waitcnt vmcnt(n) as Wn, LDS DMA wave-instructions as L (runs as L*k), other buffer/global
loads as ld, stores as ST, labels and branches in order, to check the sweep's counted waits
against the stores and DMA the compiler actually emitted between them (k_admm_iter).

    hipcc --offload-arch=gfx950 -O3 -std=c++17 --offload-device-only -S -Iinclude \
        indy7_mpc_amd/csrc/i7m_api.hip -o /tmp/api.s
    python tools/vm_waits.py /tmp/api.s _ZN3i7m11k_admm_iterILb0EEEvNS_8AdmmArgsE
"""
import re
import sys


def skeleton(text, name):
    i = text.find("\n" + name + ":")
    if i < 0:
        raise SystemExit("no kernel " + name)
    body = text[i:text.find("s_endpgm", i)]
    seq = []
    for line in body.splitlines():
        t = line.split(";")[0].strip()
        if not t:
            continue
        if t.startswith("s_waitcnt") and "vmcnt" in t:
            seq.append("W" + re.search(r"vmcnt\((\d+)\)", t).group(1))
        elif t.startswith(("buffer_store", "global_store")):
            seq.append("ST")
        elif t.startswith("buffer_load") and t.endswith(" lds"):
            seq.append("L")
        elif t.startswith(("buffer_load", "global_load")):
            seq.append("ld")
        elif re.match(r"^\.LBB\S+:", t):
            seq.append(t.split(":")[0].split("_")[-1] + ":")
        elif t.startswith(("s_cbranch", "s_branch")):
            seq.append("->" + t.split()[1].split("_")[-1])
    out = " ".join(seq)
    return re.sub(r"L( L)+", lambda m: "L*%d" % m.group(0).count("L"), out)


if __name__ == "__main__":
    text = open(sys.argv[1]).read()
    for name in sys.argv[2:]:
        print(name)
        print(skeleton(text, name))
