"""The register path's two queue modes give bit-identical solves.

Record mode (longest-first queue, scenario-major records) only changes which lanes run a
scenario and when: every scenario still runs the same instruction sequence on the same
data, so x, objective, bound, status and iteration counts must match scenario order
exactly, solve after solve (Iter0 LP and warm-started PH QPs, whose warm start lives in
the records in one mode and in the [k][S] arrays in the other).  Sizes: 20,000 farmer
scenarios (L = 4, more scenarios than resident groups, so record mode is the default)."""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _run(mode, S, iters):
    from mpisppy_amd.engine import PHEngine
    from mpisppy_amd.examples import farmer
    from mpisppy_amd import _lib
    os.environ["PHGPU_REG_REC"] = str(mode)
    try:
        b = farmer.batch_creator(farmer.scenario_names_creator(S), crops_multiplier=1, num_scens=S)
        e = PHEngine(b, device="cuda:0")
        e.want_duals = True
        out = []
        e.solve(_lib.default_options(eps_rel=1e-10), warm=False)
        assert e.kernel_info()["rec"] == mode
        out.append({k: e.host(k).copy() for k in ("x", "y", "obj", "bound", "status", "iters")})
        e.set_rho(1.0)
        e.set_terms(1, 1)
        for _ in range(iters):
            e.compute_xbar()
            e.update(True)
            e.solve(_lib.default_options(), warm=True)
            out.append({k: e.host(k).copy() for k in ("x", "y", "obj", "bound", "status", "iters")})
        e.close()
        return out
    finally:
        del os.environ["PHGPU_REG_REC"]


def test_record_mode_matches_scenario_order(gpu, register_path):
    S = 20000
    a = _run(0, S, 3)
    b = _run(1, S, 3)
    for k, (ra, rb) in enumerate(zip(a, b)):
        for name in ra:
            assert np.array_equal(ra[name], rb[name]), (k, name, np.abs(ra[name] - rb[name]).max())
    assert (a[-1]["status"] == 0).all()
