"""Fixture for config 5 (UC LP relaxation): HiGHS optimum of the LP relaxation of
Scenario1..8 (mpisppy_amd/examples/uc.py restating paperruns/larger_uc/ReferenceModel_OK.py
on the packed RootNode.dat + Node1..8.dat wind data) and the model's sizes.

Parity UNPINNED: the reference ships no UC results (its driver needs egret and gurobi),
so these numbers pin our restatement against an exact LP solver, not against the
reference.  Regenerate: python tests/golden/make_golden_uc.py
"""
import json
import os
import sys
from collections import Counter

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
sys.path.insert(0, ROOT)

from mpisppy_amd.examples import uc  # noqa: E402
from oracle import uc as ouc  # noqa: E402


def main():
    names = uc.scenario_names_creator(8)
    b = uc.batch_creator(names, num_scens=1000)
    mdl = b.template
    out = {"names": names, "num_scens": 1000, "n": b.n, "m": b.m, "nnz": b.nnz, "nn": b.nn,
           "model_rows": mdl.m, "model_nnz": sum(len(r[0]) for r in mdl.rows),
           "var_families": dict(Counter(v.name.split("[")[0] for v in mdl.vars)),
           "row_families": dict(Counter(r[3].split("[")[0] for r in mdl.rows)),
           "lp_obj": [], "lp_sum_unit_on": []}
    for s in range(len(names)):
        x, obj, st = ouc.solve_lp(b, s)
        assert st == 0
        out["lp_obj"].append(obj)
        out["lp_sum_unit_on"].append(float(x[b.nonant_col].sum()))
        print(names[s], obj, flush=True)
    rho = uc.rho_vector(mdl)
    out["rho_first"] = [float(v) for v in rho[:50]]
    out["rho_sum"] = float(rho.sum())
    json.dump(out, open(os.path.join(HERE, "uc.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
