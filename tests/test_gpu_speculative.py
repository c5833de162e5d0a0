"""The speculative solve of PHBase.iterk_loop changes nothing the reference loop would not.

iterk_loop launches iteration k+1's solve before the host reads conv (the solve depends
only on W and x̄, final after Update_W), and keeps it only when the loop goes on
(phbase.py:909-957 order: x̄ -> W -> conv -> break? -> solve).  The launch goes through
phgpu_solve_deferred: its outputs land in a spare set and its warm-start state in the
library's second slot, made current only by phgpu_commit.  So a run with the speculative
solve and one without give bit-identical x̄, W, conv and iteration counts, and a solve
after the convergence break warm-starts from the last committed iterate in both --
checked here bit for bit on the register path in scenario order and in record mode, on
the global-memory kernel, and on the multistage aircond tree (with the one-rank step run as
its own launch, PHGPU_FUSE_STEP=0).

With one rank, path 6 and a two-stage tree the speculative loop also folds the x̄ / W /
conv step into the solve launch (phgpu_ph_step_defer): its sums run in
another grid partition, so that run is checked against the unfolded one to 1e-12 (x̄, W, x)
and for the same PH iteration count.
"""
import os

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _farmer(S, spec, thresh, kernel=0, cm=1):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    so = {"kernel": kernel} if kernel else {}
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 2000, "defaultPHrho": 1.0, "convthresh": thresh,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": farmer.batch_creator, "speculative_solve": spec, "fused_ph_loop": False,
            "iter0_solver_options": dict(so), "iterk_solver_options": dict(so)}
    return PH(opts, farmer.scenario_names_creator(S), farmer.scenario_creator,
              scenario_creator_kwargs={"crops_multiplier": cm, "num_scens": S})


def _aircond(spec, thresh):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import aircond
    from mpisppy_amd.sputils import create_nodenames_from_branching_factors
    bf = [4, 3, 2]
    kw = {"branching_factors": bf, "Capacity": 200, "QuadShortCoeff": 0.3, "BeginInventory": 50, "mu_dev": 0,
          "sigma_dev": 40, "start_seed": 0}
    opts = {"solver_name": "mi355x_pdhg", "PHIterLimit": 2000, "defaultPHrho": 1.0, "convthresh": thresh,
            "verbose": False, "display_progress": False, "toc": False, "device": "cuda:0",
            "batch_creator": aircond.batch_creator, "speculative_solve": spec, "fused_ph_loop": False}
    return PH(opts, aircond.scenario_names_creator(24), aircond.scenario_creator, scenario_creator_kwargs=kw,
              all_nodenames=create_nodenames_from_branching_factors(bf))


def _run(make, spec):
    ph = make(spec)
    ph.ph_main(finalize=False)
    assert ph.converged
    assert ph._speculate(False) == spec
    e = ph.engine
    out = {"iter": ph._PHIter, "conv": ph.conv, "W": e.W.cpu().numpy().copy(),
           "xbar": e.xbar.cpu().numpy().copy(), "node_buf": e.node_buf.cpu().numpy().copy(),
           "x": e.x.cpu().numpy().copy()}
    # one more solve after the break: warm-started from the last committed solve
    ph.solve_loop(solver_options=ph.iterk_solver_options, gripe=True)
    out["x_after"] = e.x.cpu().numpy().copy()
    out["iters_after"] = e.iters.cpu().numpy().copy()
    out["kernel"] = e.kernel_info()
    out["ipm"] = e.ipm_info()
    return out


CASES = {
    "farmer3": lambda spec: _farmer(3, spec, 1e-3),
    "farmer4096_record_mode": lambda spec: _farmer(4096, spec, 3e-2),
    "farmer4096_ipm": lambda spec: _farmer(4096, spec, 3e-2),
    "farmer256_global_kernel": lambda spec: _farmer(256, spec, 3e-2, kernel=1),
    # config 2's pattern (cm = 10): the subtree interior point, which never folds the step
    "farmer128_cm10_subtree": lambda spec: _farmer(128, spec, 3e-2, cm=10),
    "aircond432": lambda spec: _aircond(spec, 1e-4),
}


@pytest.mark.parametrize("case", sorted(CASES))
def test_speculative_solve_is_invisible(gpu, case):
    keep = os.environ.get("PHGPU_REG_REC")
    keep_ipm = os.environ.get("PHGPU_IPM")
    keep_fuse = os.environ.get("PHGPU_FUSE_STEP")
    os.environ["PHGPU_FUSE_STEP"] = "0"
    if case == "farmer4096_record_mode":
        os.environ["PHGPU_REG_REC"] = "1"
        os.environ["PHGPU_IPM"] = "0"
    try:
        a = _run(CASES[case], True)
        b = _run(CASES[case], False)
    finally:
        for k, v in (("PHGPU_REG_REC", keep), ("PHGPU_IPM", keep_ipm), ("PHGPU_FUSE_STEP", keep_fuse)):
            if v is None:
                os.environ.pop(k, None)
            else:
                os.environ[k] = v
    if case == "farmer4096_record_mode":
        assert a["kernel"]["rec"] == 1, a["kernel"]
    if case == "farmer4096_ipm":
        assert a["kernel"]["path"] == 6, a["kernel"]
    if case == "farmer128_cm10_subtree":
        assert a["kernel"]["path"] == 6 and a["ipm"]["kernel"] == 4 and a["ipm"]["folded_steps"] == 0, a
    assert a["iter"] == b["iter"] and a["conv"] == b["conv"], (a["iter"], b["iter"], a["conv"], b["conv"])
    for k in ("W", "xbar", "node_buf", "x", "x_after", "iters_after"):
        assert np.array_equal(a[k], b[k]), (case, k, np.abs(a[k] - b[k]).max())


@pytest.mark.parametrize("S", [4096, 40000])
def test_folded_step_matches_the_step_launch(gpu, S):
    """The speculative loop with the PH step folded into the path-6 solve launch (lane
    groups at 4,096 scenarios, one lane at 40,000) against the same loop with the step as
    its own launch: the same PH iteration count to conv < 3e-2, the folded path actually
    taken, and x̄ / W / x / conv within 1e-8 relative: the x̄ sums run in another grid
    partition (bits differ at 1e-16), and over a hundred PH iterations the interior point's
    own stopping points amplify that to ~1e-10 (40,000 scenarios: conv 3e-10 relative)."""
    keep = os.environ.get("PHGPU_FUSE_STEP")
    try:
        os.environ["PHGPU_FUSE_STEP"] = "0"
        b = _run(lambda spec: _farmer(S, spec, 3e-2), True)
        # (the lane groups at 4,096 scenarios fold only when asked: PHGPU_FUSE_STEP=1)
        if S == 4096:
            os.environ["PHGPU_FUSE_STEP"] = "1"
        else:
            os.environ.pop("PHGPU_FUSE_STEP", None)
        ph = _farmer(S, True, 3e-2)
        ph.ph_main(finalize=False)
        assert ph.converged
        e = ph.engine
        folded = e.ipm_info()["folded_steps"]
        a = {"iter": ph._PHIter, "conv": ph.conv, "W": e.W.cpu().numpy().copy(), "xbar": e.xbar.cpu().numpy().copy(),
             "node_buf": e.node_buf.cpu().numpy().copy(), "x": e.x.cpu().numpy().copy()}
    finally:
        if keep is None:
            os.environ.pop("PHGPU_FUSE_STEP", None)
        else:
            os.environ["PHGPU_FUSE_STEP"] = keep
    assert e.kernel_info()["path"] == 6
    assert folded >= a["iter"] - 2, (folded, a["iter"])
    assert a["iter"] == b["iter"], (a["iter"], b["iter"])
    assert abs(a["conv"] - b["conv"]) <= 1e-8 * abs(b["conv"]), (a["conv"], b["conv"])
    for k in ("W", "xbar", "node_buf", "x"):
        scale = max(1.0, float(np.abs(b[k]).max()))
        assert np.abs(a[k] - b[k]).max() <= 1e-8 * scale, (k, np.abs(a[k] - b[k]).max())


def test_subtree_kernel_never_folds_the_step(gpu):
    """PHGPU_FUSE_STEP=1 asks the library to fold the one-rank PH step into lane-group
    launches too; the workgroup kernels (config 2's subtree interior point) carry no folded
    step, so the step must still run as its own launch there: same iterations and bits as
    the unforced run, folded_steps 0."""
    keep = os.environ.get("PHGPU_FUSE_STEP")
    try:
        os.environ.pop("PHGPU_FUSE_STEP", None)
        b = _run(lambda spec: _farmer(128, spec, 3e-2, cm=10), True)
        os.environ["PHGPU_FUSE_STEP"] = "1"
        a = _run(lambda spec: _farmer(128, spec, 3e-2, cm=10), True)
    finally:
        if keep is None:
            os.environ.pop("PHGPU_FUSE_STEP", None)
        else:
            os.environ["PHGPU_FUSE_STEP"] = keep
    assert a["ipm"]["kernel"] == 4 and a["ipm"]["folded_steps"] == 0, a["ipm"]
    assert a["iter"] == b["iter"] and a["conv"] == b["conv"]
    for k in ("W", "xbar", "x"):
        assert np.array_equal(a[k], b[k]), k
