"""CPU: the C-ABI library builds for gfx950, loads, exports every symbol include/indy7_mpc.h
declares, its structs match the ctypes mirror, and it fails loudly without a GPU
(no CPU fallback)."""
import ctypes as C
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "indy7_mpc.h")


def _declared():
    txt = open(HEADER).read()
    return sorted(set(re.findall(r"^\s*(?:const\s+char\*|int|void)\s+(i7m_\w+)\s*\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib():
    from indy7_mpc_amd import _lib
    import __graft_entry__ as ge

    ge.build_lib()
    return _lib.load()


def test_every_declared_symbol_is_exported(lib):
    from indy7_mpc_amd import _lib

    names = _declared()
    assert len(names) >= 20
    for n in names:
        assert hasattr(lib, n), n
    bound = {s[0] for s in _lib.SIGNATURES}
    assert set(names) == bound, set(names) ^ bound


def test_so_is_gfx950_code_object(lib):
    from indy7_mpc_amd import _lib

    data = open(_lib.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in data or b"gfx950" in data
    assert b"k_riccati" in data and b"k_linearize" in data and b"k_linesearch" in data


def test_struct_layout_matches_header(tmp_path):
    from indy7_mpc_amd import _lib

    src = tmp_path / "s.c"
    src.write_text('#include "indy7_mpc.h"\n#include <stdio.h>\n#include <stddef.h>\n'
                   'int main(){printf("%zu %zu %zu %zu\\n",sizeof(i7m_config),offsetof(i7m_config,model),'
                   'sizeof(i7m_model),sizeof(i7m_problem_stats));return 0;}\n')
    exe = tmp_path / "s"
    subprocess.run(["gcc", "-I" + os.path.dirname(HEADER), str(src), "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()]
    assert got == [C.sizeof(_lib.i7m_config), _lib.i7m_config.model.offset, C.sizeof(_lib.i7m_model),
                   C.sizeof(_lib.i7m_problem_stats)]


def test_config_default(lib):
    from indy7_mpc_amd import _lib

    cfg = _lib.i7m_config()
    assert lib.i7m_config_default(C.byref(cfg)) == 0
    assert (cfg.N, cfg.dt, cfg.dQ_cost, cfg.R_cost, cfg.QN_cost, cfg.eps, cfg.mu, cfg.step_tol, cfg.max_sqp_iters) == \
        (32, 0.01, 0.01, 1e-5, 100.0, 1.0, 10.0, 1e-3, 2)  # src/osqp_solver.py:7, src/osqp_sqp.py:50,77,90


def test_invalid_arguments_are_rejected(lib):
    from indy7_mpc_amd import _lib

    cfg = _lib.i7m_config()
    lib.i7m_config_default(C.byref(cfg))
    h = C.c_void_p()
    cfg.N = 65
    assert lib.i7m_create(C.byref(cfg), C.byref(h)) == -1
    assert b"N must be" in lib.i7m_last_error()
    assert lib.i7m_solve(None, 1, None, None, None, 3, None, None) == -1


def test_precision_field_refuses_fp32(lib):
    """i7m_config.precision (SURVEY.md 8b's ABI sketch): I7M_PREC_F64 is the default and the only
    arithmetic built; I7M_PREC_F32 (GATO's float, gato_controller.py:54-62) and unknown values are
    refused by i7m_create before any device work, with a message naming the reason."""
    from indy7_mpc_amd import _lib

    cfg = _lib.i7m_config()
    lib.i7m_config_default(C.byref(cfg))
    assert cfg.precision == _lib.PREC_F64
    h = C.c_void_p()
    cfg.precision = _lib.PREC_F32
    assert lib.i7m_create(C.byref(cfg), C.byref(h)) == -1
    assert b"I7M_PREC_F32 is not built" in lib.i7m_last_error()
    cfg.precision = 7
    assert lib.i7m_create(C.byref(cfg), C.byref(h)) == -1
    assert b"unknown precision" in lib.i7m_last_error()


def test_no_cpu_fallback_without_gpu(lib, model):
    """With no GPU (this container) creating a handle raises — nothing silently runs on CPU."""
    from indy7_mpc_amd import _lib

    if _lib.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(_lib.I7MError):
        _lib.Handle(model, N=16)
    from indy7_mpc_amd.osqp_solver import OSQPSolver

    with pytest.raises(_lib.I7MError):
        OSQPSolver(model, N=16)


def test_version_is_stamped_with_the_source_tree(lib):
    """i7m_version() carries the sha256 prefix of the sources it was built from
    (__graft_entry__.src_hash): the loaded binary matches this tree, and it is the release
    build (no I7M_DIAG ablation kernels)."""
    from indy7_mpc_amd import _lib
    import __graft_entry__ as ge

    v = _lib.version()
    assert v.endswith("src " + ge.src_hash()), (v, ge.src_hash())
    assert "release" in v


def test_abi_version_matches_header_and_binding(lib, tmp_path):
    """i7m_abi_version() == the header's I7M_ABI_VERSION == the revision the ctypes binding
    follows (i7m_aba / i7m_rk4 / i7m_set_external_wrench changed signature under the
    same names in 0.2, so a caller can only tell the revisions apart by asking)."""
    from indy7_mpc_amd import _lib

    m = re.search(r"#define\s+I7M_ABI_VERSION\s+(\d+)", open(HEADER).read())
    assert m and int(m.group(1)) == lib.i7m_abi_version() == _lib.ABI_VERSION
