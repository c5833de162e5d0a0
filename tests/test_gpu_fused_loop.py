"""The fused PH loop (phgpu_ph_loop): PHBase.iterk_loop of one rank in one
cooperative launch -- x̄ -> W -> conv -> (conv < convthresh: stop) -> solve per iteration,
x̄ and conv by grid-wide steps, every scenario in registers across the iterations.

  * config 3 as bench.py runs it, 5 PH iterations from Iter0 against farmer_scale.json
    (x̄ / conv of every iteration, sampled W, E[obj]; north_star tolerances);
  * against the step-by-step loop (the speculative solve with the folded step) on the same
    scenarios: the same break iteration and x̄ / W / x / conv within 1e-8 relative (the
    warm start comes from registers instead of the scaled warm state: last-bit differences
    the interior point's stopping points amplify over the iterations);
  * a solve that hands scenarios to the PDHG fallback ends the launch (end 2) and the loop
    goes on step by step: the same iterates as the step-by-step loop with the same fallback;
  * states the launch does not take (more workgroups than fit at once, several ranks,
    extensions) run step by step (engine.ph_loop returns None, nothing launched).

The config-3 run to convergence (break at the oracle's iteration +-1, the conv trajectory
within 1e-6) is test_gpu_convergence.py's fused case.
"""
import json
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
SCALE = json.load(open(os.path.join(HERE, "golden", "farmer_scale.json")))
ABS = 1e-5
OBJ_REL = 1e-5


def _farmer(S, iters, thresh, fused, **extra):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": iters, "defaultPHrho": 1.0, "convthresh": thresh,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": farmer.batch_creator, "fused_ph_loop": fused,
            "iterk_solver_options": dict(farmer.PDHG_ITERK_OPTIONS)}
    opts.update(extra)
    return PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
              scenario_creator_kwargs={"crops_multiplier": 1, "num_scens": S})


def _state(ph):
    e = ph.engine
    return {"iter": ph._PHIter, "conv": ph.conv, "W": e.W.cpu().numpy().copy(), "xbar": e.xbar.cpu().numpy().copy(),
            "node_buf": e.node_buf.cpu().numpy().copy(), "x": e.x.cpu().numpy().copy(),
            "status": e.host("status").copy(), "calls": dict(e.calls), "loops": list(getattr(ph, "fused_loops", [])),
            "declined": getattr(e, "ph_loop_declined", None)}


def test_fused_loop_config3_five_iterations_vs_fixture(gpu):
    g = SCALE["farmer65536_cm1"]
    ph = _farmer(65536, 5, -1.0, True)
    ph.PH_Prep()
    tb = ph.Iter0()
    assert abs(tb - g["trivial_bound"]) <= OBJ_REL * abs(g["trivial_bound"])
    ph.iterk_loop()
    e = ph.engine
    assert e.calls["ph_loop"] == 1, (e.calls, getattr(e, "ph_loop_declined", None))
    r = ph.fused_loops[-1]
    assert r["steps"] == 5 and r["end"] == 0, r
    conv = np.array(r["conv"])
    assert np.abs(conv - np.array(g["conv"])).max() <= ABS, (conv, g["conv"])
    assert abs(ph.conv - g["conv"][4]) <= ABS
    xb = ph.xbar_by_node()["ROOT"][:3]
    assert np.abs(xb - np.array(g["xbar"][4])).max() <= ABS, xb
    W = ph.W_array()[np.array(g["sample"])]
    assert np.abs(W - np.array(g["W"])).max() <= ABS
    eobj = ph.Eobjective()
    assert abs(eobj - g["Eobj"]) <= OBJ_REL * abs(g["Eobj"]), (eobj, g["Eobj"])
    assert (e.host("status") == 0).all()
    # the launch's IPM iterations are what the step-by-step solves would count (7.5 per
    # scenario and PH iteration at this configuration)
    assert 5 * 65536 * 4 <= r["ipm_iters"] <= 5 * 65536 * 20, r["ipm_iters"]


@pytest.mark.parametrize("S", [40000, 65536])
def test_fused_loop_matches_step_by_step(gpu, S):
    out = {}
    for fused in (False, True):
        ph = _farmer(S, 400, 3e-2, fused)
        ph.ph_main(finalize=False)
        assert ph.converged
        out[fused] = _state(ph)
        ph.engine.close()
    a, b = out[True], out[False]
    assert a["calls"]["ph_loop"] == 1 and b["calls"]["ph_loop"] == 0
    assert a["loops"][0]["end"] == 1 and a["loops"][0]["steps"] == a["iter"]
    assert a["iter"] == b["iter"], (a["iter"], b["iter"])
    assert abs(a["conv"] - b["conv"]) <= 1e-8 * abs(b["conv"]), (a["conv"], b["conv"])
    for k in ("W", "xbar", "node_buf", "x"):
        scale = max(1.0, float(np.abs(b[k]).max()))
        assert np.abs(a[k] - b[k]).max() <= 1e-8 * scale, (k, np.abs(a[k] - b[k]).max())
    assert (a["status"] == 0).all()


def test_fused_loop_hands_over_to_the_fallback(gpu):
    """(65,536 scenarios: a share the one-lane module runs; smaller shares take lane groups,
    which the fused loop does not.)  PHGPU_IPM_MAXIT=6: scenarios that need more interior-point iterations go to the PDHG
    fallback; the fused launch stops at the first such solve (end 2) and the loop finishes
    step by step -- the same PH iterates as the step-by-step loop under the same cap."""
    keep = os.environ.get("PHGPU_IPM_MAXIT")
    os.environ["PHGPU_IPM_MAXIT"] = "6"
    try:
        out = {}
        for fused in (False, True):
            ph = _farmer(65536, 8, -1.0, fused)
            ph.ph_main(finalize=False)
            out[fused] = _state(ph)
            ph.engine.close()
    finally:
        if keep is None:
            os.environ.pop("PHGPU_IPM_MAXIT", None)
        else:
            os.environ["PHGPU_IPM_MAXIT"] = keep
    a, b = out[True], out[False]
    assert a["calls"]["ph_loop"] == 1 and a["loops"][0]["end"] == 2, (a["calls"], a["loops"], a["declined"])
    assert a["loops"][0]["steps"] < 8
    assert a["iter"] == b["iter"] == 8
    # the handed-over scenarios are solved by the PDHG fallback to its eps_rel from the
    # loop's warm start in one case and the step-by-step warm state in the other: the
    # iterates agree to the first-order solver's tolerance (measured 1.5e-6 of max|W|), not
    # to the last bits
    assert abs(a["conv"] - b["conv"]) <= 1e-5 * abs(b["conv"]), (a["conv"], b["conv"])
    for k in ("W", "xbar", "x"):
        scale = max(1.0, float(np.abs(b[k]).max()))
        assert np.abs(a[k] - b[k]).max() <= 1e-5 * scale, (k, np.abs(a[k] - b[k]).max())


def test_fused_loop_not_taken_where_it_does_not_apply(gpu):
    """70,000 scenarios: 274 workgroups of the one-lane module do not fit the GPU at once
    (one per CU): the loop runs step by step, nothing launched by phgpu_ph_loop."""
    ph = _farmer(70000, 3, -1.0, True)
    ph.ph_main(finalize=False)
    e = ph.engine
    assert e.calls["ph_loop"] == 0 and not getattr(ph, "fused_loops", []), e.calls
    assert e.calls["ph_step_defer"] >= 2, e.calls
    assert (e.host("status") == 0).all()
