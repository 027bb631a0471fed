"""The built library's code has no partial-mask DPP fma within two wait states of the VALU write of
its accumulator (the hazard of tools/probes/rowsplit_probe.hip: masked-out lanes get the stale
accumulator back).  Static: disassembles the in-tree library, no GPU."""
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import dpp_hazard_scan as dhs  # noqa: E402

LIB = os.path.join(ROOT, "indy7_mpc_amd", "lib", "libindy7mpc.so")


def test_scan_flags_back_to_back_shrinking_masks():
    asm = """
<k>:
	v_fmac_f64_dpp v[12:13], v[2:3], v[4:5] row_newbcast:0 row_mask:0xf bank_mask:0xf
	v_fmac_f64_dpp v[12:13], v[2:3], v[6:7] row_newbcast:4 row_mask:0xf bank_mask:0xe
	s_nop 1
	v_fmac_f64_dpp v[12:13], v[2:3], v[8:9] row_newbcast:8 row_mask:0xf bank_mask:0xc
	v_fmac_f64_dpp v[14:15], v[2:3], v[8:9] row_newbcast:8 row_mask:0xf bank_mask:0xc
	v_add_f64 v[16:17], v[0:1], v[0:1]
	v_fmac_f64_dpp v[16:17], v[2:3], v[8:9] row_newbcast:8 row_mask:0x3 bank_mask:0xf
	v_mov_b32 v20, v0
	v_mov_b32_dpp v21, v20 row_shr:1 row_mask:0xf bank_mask:0xf
"""
    seen, hazards, src = dhs.scan_text(asm)
    assert [h[1].split()[0] for h in src] == ["v_mov_b32_dpp"]
    assert seen == 4
    # the second (right after a write of v[12:13]) and the last (right after v_add wrote v[16:17])
    assert [h[1].split()[1] for h in hazards] == ["v[12:13],", "v[16:17],"]


@pytest.mark.skipif(not os.path.exists(LIB), reason="library not built (__graft_entry__.build())")
@pytest.mark.skipif(not os.path.exists(os.path.join(dhs.LLVM, "llvm-objdump")), reason="no llvm-objdump")
def test_release_library_has_no_dpp_mask_hazard():
    r = dhs.scan(LIB)
    assert r["partial_mask_dpp_fma"] > 0, r  # the scan sees the sweeps' triangular products
    assert r["hazards"] == 0, r
    assert r["dpp_source_hazards"] == 0, r
