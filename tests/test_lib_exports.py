"""The C-ABI library loads on CPU and exports every symbol include/phgpu.h declares
(no compute calls without a GPU)."""
import ctypes
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "include", "phgpu.h")
LIB = os.path.join(ROOT, "mpi-sppy-1_amd", "mpisppy_amd", "libphgpu.so")


def declared_symbols():
    txt = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int|int64_t)\s+(phgpu_\w+)\s*\(", txt, re.M)))


@pytest.fixture(scope="module")
def lib():
    if not os.path.exists(LIB):
        import __graft_entry__ as g
        g.build(verbose=False)
    return ctypes.CDLL(LIB)


def test_header_declares_the_abi():
    syms = declared_symbols()
    for s in ["phgpu_create", "phgpu_set_scenarios", "phgpu_set_ph_state", "phgpu_solve",
              "phgpu_ph_reduce", "phgpu_ph_update", "phgpu_destroy", "phgpu_last_error"]:
        assert s in syms


def test_library_exports_every_declared_symbol(lib):
    for s in declared_symbols():
        assert hasattr(lib, s), s
    from mpisppy_amd import _lib
    assert sorted(_lib.EXPORTS) == declared_symbols()


def test_nm_shows_extern_c(lib):
    out = subprocess.run(["nm", "-D", "--defined-only", LIB], capture_output=True, text=True).stdout
    for s in declared_symbols():
        assert re.search(rf"\bT {s}$", out, re.M), s


def test_host_only_calls(lib):
    """Calls that touch no device: default options, last_error, null-handle errors."""
    from mpisppy_amd import _lib
    o = _lib.default_options(eps_abs=1e-13)
    assert o.eps_rel == 1e-9 and o.omega_clamp == 1e4 and o.check_every == 64 and o.max_iter == 100000
    L = _lib.load()
    assert L.phgpu_destroy(None) == 0
    assert L.phgpu_set_ph_state(None, None, None, None, 0, 0) != 0
    assert "null handle" in _lib.last_error()
    assert L.phgpu_workspace_bytes(None) == -1
    with pytest.raises(KeyError):
        _lib.default_options(nonsense=1)
    # the library keeps PDLP's restart constants; farmer's recommended PH-solve options
    # (examples/farmer.py, used by bench.py) are valid phgpu_options fields
    assert o.beta_sufficient == 0.2 and o.beta_necessary == 0.8 and o.beta_artificial == 0.36
    from mpisppy_amd.examples import farmer
    of = _lib.default_options(**farmer.PDHG_ITERK_OPTIONS)
    assert of.beta_sufficient == farmer.PDHG_ITERK_OPTIONS["beta_sufficient"]


def test_product_path_has_no_cpu_fallback():
    """The product package never imports the oracle and the engine refuses to run
    without a GPU."""
    pkg = os.path.join(ROOT, "mpi-sppy-1_amd", "mpisppy_amd")
    for dp, _, fs in os.walk(pkg):
        for f in fs:
            if f.endswith(".py"):
                src = open(os.path.join(dp, f)).read()
                assert "import oracle" not in src and "from oracle" not in src, f
    import torch
    if not torch.cuda.is_available():
        from mpisppy_amd.engine import PHEngine
        from mpisppy_amd.examples import farmer
        from mpisppy_amd import _lib
        b = farmer.batch_creator(farmer.scenario_names_creator(3))
        with pytest.raises(_lib.PhgpuError):
            PHEngine(b)
