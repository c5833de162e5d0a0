"""Generate the committed golden fixtures from the CPU oracle (tests/golden/*.json).

Run:  python tests/golden/make_golden.py
Provenance: the oracle restates the reference (see oracle/__init__.py); its farmer
trajectory reproduces the reference's own fixtures ref_w_file.csv / ref_xbar_file.csv
(copied verbatim from mpisppy/tests/examples/w_test_data/, used by
mpisppy/tests/test_w_writer.py:85-117) to <= 3e-7, checked in tests/test_oracle_golden.py.
"""
import json
import os
import sys
import warnings

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, ROOT)
warnings.simplefilter("ignore")

from oracle.models import farmer_scenario, farmer_yields, aircond_scenario  # noqa: E402
from oracle.ph import OraclePH  # noqa: E402


def farmer_run(names, cm, rho, iters, thresh, num_scens=None):
    scens = [farmer_scenario(n, cm, num_scens=num_scens) for n in names]
    crops_sorted = sorted(farmer_yields(names[0], cm)[0])
    Ys = [farmer_yields(n, cm)[1] for n in names]
    ph = OraclePH(scens, rho, solver="farmer", farmer_info=(crops_sorted, Ys, cm))
    tb = ph.iter0()
    x0 = ph.x.copy()
    obj0 = ph.obj.copy()
    ph.iterk_loop(iters, thresh)
    return ph, tb, x0, obj0


def main():
    out = {}
    # farmer 3 scenarios, rho = 1 (test_w_writer.py setup): trajectory to conv < 1e-4
    names = [f"scen{i}" for i in range(3)]
    ph, tb, x0, obj0 = farmer_run(names, 1, 1.0, 200, 1e-4, num_scens=3)
    out["farmer3_rho1"] = {
        "names": names, "crops_multiplier": 1, "rho": 1.0,
        "nonant_names": ["DevotedAcreage[CORN0]", "DevotedAcreage[SUGAR_BEETS0]", "DevotedAcreage[WHEAT0]"],
        "trivial_bound": tb, "iter0_x": x0.tolist(), "iter0_obj": obj0.tolist(),
        "conv_1e-4_iter": ph.converged_at, "Eobj_at_conv": ph.Eobjective(),
        "traj": [{"iter": h["iter"], "conv": h["conv"], "xbar": h["xbar"][0].tolist(),
                  "W": h["W"].tolist()} for h in ph.history],
    }
    ph3, _, _, _ = farmer_run(names, 1, 1.0, 400, 1e-3, num_scens=3)
    out["farmer3_rho1"]["conv_1e-3_iter"] = ph3.converged_at
    # farmer Scenario1..30 trivial bound (test_aph.py:230-253)
    names30 = [f"Scenario{i + 1}" for i in range(30)]
    scens = [farmer_scenario(n, 1) for n in names30]
    out["farmer30_trivial_bound"] = OraclePH(scens, 1.0).iter0()
    # farmer cm=10, 16 scenarios, 5 PH iterations (parity at the cfg-2 problem size).
    # scen0..2 are skipped: with cm > 1 their crop copies have identical yields, so the
    # Iter0 LP optimum is not unique and any LP solver may return any optimal vertex.
    names16 = [f"scen{i}" for i in range(3, 19)]
    ph16, tb16, x016, _ = farmer_run(names16, 10, 1.0, 5, 1e-12, num_scens=16)
    out["farmer16_cm10_rho1"] = {"names": names16, "trivial_bound": tb16, "iter0_x": x016.tolist(),
                                 "W5": ph16.W.tolist(), "xbar5": ph16.xbar[0].tolist(),
                                 "Eobj5": ph16.Eobjective()}
    # aircond bf 4 3 2 with straight_tests.py:36 parameters, rho = 1
    kw = dict(Capacity=200, QuadShortCoeff=0.3, BeginInventory=50, mu_dev=0, sigma_dev=40, start_seed=0)
    bf = [4, 3, 2]
    an = [f"scen{i}" for i in range(24)]
    sc = [aircond_scenario(n, bf, **kw) for n in an]
    pha = OraclePH(sc, 1.0)
    atb = pha.iter0()
    ax0 = pha.x.copy()
    pha.iterk_loop(300, 1e-4)
    out["aircond432_rho1"] = {
        "names": an, "branching_factors": bf, "kwargs": kw, "trivial_bound": atb,
        "iter0_x": ax0.tolist(), "conv_1e-4_iter": pha.converged_at,
        "traj5": [{"iter": h["iter"], "conv": h["conv"], "W": h["W"].tolist(),
                   "xbar": h["xbar"].tolist()} for h in pha.history[:5]],
        "node_xbar_final": {k: v.tolist() for k, v in pha.node_xbar.items()},
    }
    with open(os.path.join(HERE, "golden.json"), "w") as f:
        json.dump(out, f, indent=1)
    print("farmer3 conv iters", ph.converged_at, ph3.converged_at, "tb", tb,
          "tb30", out["farmer30_trivial_bound"], "aircond conv", pha.converged_at, "tb", atb)


if __name__ == "__main__":
    main()
