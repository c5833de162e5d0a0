"""bench.py's self-check (its JSON line's ``checks``, exit status 3 on a mismatch), run on
the CPU: the warmup of a fixture workload is compared with the oracle fixture on every
rank, so a driver N > 1 run that computes a wrong x̄, W or conv (phbase.py:83-87,
339-343) fails loudly instead of printing a throughput.

The observations are produced by the exact vectorised oracle (oracle/farmer_vec.py) on
config 2 (farmer 1,024 scenarios, cm = 10), split over two "ranks" the way
sputils.py:803-810 slices them: at the fixture's rho every check holds; a perturbed rho
(1.02) -- a stand-in for any wrong reduction -- fails conv, x̄, W and E[obj]."""
import json
import os
import sys

import numpy as np
import pytest

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from oracle.farmer_vec import FarmerVecPH  # noqa: E402


def _observe(rho, warmup=5, world=2):
    g = bench.load_check_fixture("farmer", 1024, 10)
    ph = FarmerVecPH([f"scen{i}" for i in range(1024)], 10, rho=rho)
    tb = ph.iter0()
    ph.iterk_loop(warmup)
    conv = [h["conv"] for h in ph.history]
    per_rank = []
    for r in range(world):
        lo, hi = r * 1024 // world, (r + 1) * 1024 // world
        obs = {"trivial_bound": tb, "conv": conv, "warmup": warmup, "xbar_last": ph.history[-1]["xbar"],
               "w_rows": {s: ph.W[s] for s in range(lo, hi)}, "eobj": ph.Eobjective()}
        d = bench.parity_checks(g, obs, 1.0)
        d["conv_seen"] = conv
        per_rank.append(d)
    return bench.combine_checks(per_rank, world, "gloo")


@pytest.fixture(scope="module")
def fixture_ok():
    return bench.load_check_fixture("farmer", 1024, 10) is not None


def test_fixture_lookup():
    assert bench.load_check_fixture("farmer", 65536, 1)["ph_iters"] == 5
    assert bench.load_check_fixture("farmer", 4096, 1) is None
    assert bench.load_check_fixture("aircond", 65536, None, bf=[32, 32, 64]) is not None
    assert bench.load_check_fixture("aircond", 65536, None, bf=[64, 32, 32]) is None


def test_checks_pass_at_the_fixture_rho(fixture_ok):
    c = _observe(1.0)
    assert c["all_ok"], c
    assert c["ranks_seen"] == 2 and c["ranks_seen_ok"] and c["W_rows_checked"] == 128
    for k in ("trivial_bound_ok", "conv_ok", "xbar_ok", "W_ok", "eobj_ok"):
        assert c[k] is True, (k, c)


def test_checks_fail_on_a_perturbed_rho(fixture_ok):
    c = _observe(1.02)
    assert not c["all_ok"], c
    assert c["trivial_bound_ok"] is True          # Iter0 does not see rho
    assert c["conv_ok"] is False and c["xbar_ok"] is False and c["W_ok"] is False, c


def test_short_warmup_checks_what_it_reaches():
    """Fewer warmup iterations than the fixture pins: conv of those iterations only."""
    c = _observe(1.0, warmup=3)
    assert c["all_ok"] and c["conv_ok"] is True and c["xbar_ok"] is None and c["W_ok"] is None, c


def test_ranks_disagreeing_on_conv_fail():
    g = bench.load_check_fixture("farmer", 1024, 10)
    obs = {"trivial_bound": g["trivial_bound"], "conv": g["conv"], "warmup": 5, "xbar_last": g["xbar"][4],
           "w_rows": {s: g["W"][j] for j, s in enumerate(g["sample"])}, "eobj": g["Eobj"]}
    a = bench.parity_checks(g, obs, 1.0)
    b = dict(a)
    a["conv_seen"] = list(g["conv"])
    b["conv_seen"] = list(g["conv"][:4]) + [g["conv"][4] * (1 + 1e-15)]
    assert bench.combine_checks([a, dict(a)], 2, "nccl")["all_ok"]
    c = bench.combine_checks([a, b], 2, "nccl")
    assert not c["ranks_agree_on_conv"] and not c["all_ok"]
    # a rank missing from the gather
    assert not bench.combine_checks([a], 2, "nccl")["all_ok"]


def test_json_line_carries_checks_key():
    """The JSON line is built with the checks dict (serialisable as is)."""
    c = _observe(1.0, warmup=5)
    json.dumps(c)
