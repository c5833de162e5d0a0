"""Diagnostic (TEST INFRASTRUCTURE, not collected): config 4 (aircond 65,536) PH to conv <
1e-2 as test_config4_aircond65536_iterations_to_convergence, with iterk eps_rel from argv;
prints the break iteration, x̄ / W errors against aircond_conv.json and the worst W samples.

    python tests/diag_config4.py [eps_rel]
"""
import json
import os
import sys
import time

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(HERE, "..", "mpi-sppy-1_amd"))
sys.path.insert(0, HERE)


def main():
    from test_gpu_config4 import _aircond_ph, CONV_FILE
    g = json.load(open(CONV_FILE))
    extra = {}
    if len(sys.argv) > 1:
        extra["iterk_solver_options"] = {"eps_rel": float(sys.argv[1])}
    want = g["break_iteration"]
    ph = _aircond_ph(g["branching_factors"], want + 10, g["conv_thresh"], **extra)
    t0 = time.perf_counter()
    ph.ph_main()
    print("ph_main %.2f s, iter %d (want %d), ipm %s" % (time.perf_counter() - t0, ph._PHIter, want, ph.engine.ipm_info()))
    key = str(ph._PHIter)
    if key in g["xbar_last"]:
        nx = ph.xbar_by_node()
        got = np.array([nx[nd][:2] for nd in g["node_names"]])
        print("xbar err %.3e" % np.abs(got - np.array(g["xbar_last"][key])).max())
    if ph._PHIter == want:
        smp = np.array(g["W_sample"])
        W = ph.W_array()[smp]
        ref = np.array(g["W_break"])
        err = np.abs(W - ref)
        worst = np.argsort(-err.max(1))[:6]
        print("W err max %.3e mean %.3e" % (err.max(), err.mean()))
        for k in worst:
            print("   sample %d scen %d err %.3e W %s ref %s" % (k, smp[k], err[k].max(), np.round(W[k], 6), np.round(ref[k], 6)))


if __name__ == "__main__":
    main()
