"""W and x-bar CSV files (mirrors mpisppy/utils/wxbarutils.py:42-395).

The file formats are the reference's, so files written by one side read on the other:

  W, one file            scenario_name,variable_name,value   (wxbarutils.py:69-81)
  W, one file per scen   <dir>/<scenario_name>_weights.csv with variable_name,value
  x-bar                  variable_name,value   (nonants of the first local scenario)

Rows starting with '#' are comments; a variable name may contain commas (it is what
lies between the first and the last comma).  Values are written with ``str(float)``,
as the reference does.  Variable names are the batch's ``nonant_names`` (the Pyomo
``var.name`` of each nonant in the flat node-list order, scenario_tree.py:39).

Values move between the files and the engine's device arrays through host copies:
``PHB.W_array()`` / ``engine.set_W`` and ``engine.host("xbar")`` / ``engine.set_xbar``.
"""
import os

import numpy as np


def nonant_names(PHB):
    b = PHB.batch
    return list(b.nonant_names) if b.nonant_names else [f"nonant[{k}]" for k in range(b.nn)]


# ------------------------------------------------------------------ W
def write_W_to_file(PHB, fname, sep_files=False):
    """wxbarutils.py:42-81: one file (rank 0 appends every rank's rows, in rank order)
    or one ``<sname>_weights.csv`` per local scenario under the directory ``fname``."""
    names = nonant_names(PHB)
    W = PHB.W_array()
    if sep_files:
        for s, sname in enumerate(PHB.local_scenario_names):
            with open(os.path.join(fname, sname + "_weights.csv"), "w") as f:
                for k, vname in enumerate(names):
                    f.write(",".join([vname, str(float(W[s, k]))]) + "\n")
        return
    rows = [(sname, names[k], float(W[s, k]))
            for s, sname in enumerate(PHB.local_scenario_names) for k in range(len(names))]
    gathered = PHB.mpicomm.gather_object(rows, root=0)
    if PHB.cylinder_rank == 0:
        with open(fname, "a") as f:
            for part in gathered:
                for (sname, vname, val) in part:
                    f.write(",".join([sname, vname, str(val)]) + "\n")


def set_W_from_file(fname, PHB, rank, sep_files=False, disable_check=False):
    """wxbarutils.py:87-129: read W for the local scenarios, check it (unless
    disabled) and load it into the engine."""
    local = list(PHB.local_scenario_names)
    if sep_files:
        w_val_dict = {sname: _parse_W_csv_single(os.path.join(fname, sname + "_weights.csv"))
                      for sname in local}
    else:
        w_val_dict = _parse_W_csv(fname, local, PHB.all_scenario_names, rank)
    if not disable_check:
        _check_W(w_val_dict, PHB, rank)
    index = {vname: k for k, vname in enumerate(nonant_names(PHB))}
    W = np.array(PHB.W_array(), dtype=np.float64, copy=True)
    for s, sname in enumerate(local):
        for vname, val in w_val_dict[sname].items():
            W[s, index[vname]] = val            # KeyError on an unknown name, as mp[...] (:120-129)
    PHB.engine.set_W(W)


def _parse_W_csv_single(fname):
    """wxbarutils.py:131-151: variable_name,value rows of one scenario."""
    if not os.path.exists(fname):
        raise RuntimeError(f"Could not find file {fname}")
    results = {}
    with open(fname, "r") as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.split(",")
            results[",".join(parts[:-1])] = float(parts[-1])
    return results


def _parse_W_csv(fname, scenario_names_local, scenario_names_global, rank):
    """wxbarutils.py:153-217: scenario_name,variable_name,value rows; unknown scenarios
    are ignored (with a warning on rank 0), a missing local scenario raises."""
    glob = set(scenario_names_global)
    loc = set(scenario_names_local)
    results = {}
    with open(fname, "r") as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.split(",")
            sname = parts[0]
            vname = ",".join(parts[1:-1])
            wval = float(parts[-1])
            if sname not in glob:
                if rank == 0:
                    print("WARNING: Ignoring unknown scenario name", sname)
                continue
            if sname not in loc:
                continue
            results.setdefault(sname, {})[vname] = wval
    missing = [nm for nm in scenario_names_local if nm not in results]
    if missing:
        raise RuntimeError("rank " + str(rank) + " could not find the following "
                           "scenarios in the provided weight file: " + ", ".join(missing))
    return results


def _check_W(w_val_dict, PHB, rank):
    """wxbarutils.py:219-267: missing variables raise, extra ones are dropped with a
    message, and sum_s p_s W_s must vanish per variable (|.| <= 1e-7).  The dual
    feasibility sums are gathered on every rank, so all ranks raise together (the
    reference raises on rank 0 only)."""
    vn_model = set(nonant_names(PHB))
    for sname in PHB.local_scenario_names:
        provided = set(w_val_dict[sname].keys())
        diff = vn_model.difference(provided)
        if diff:
            raise RuntimeError(sname + " is missing the following variables: " + ", ".join(sorted(diff)))
        diff = provided.difference(vn_model)
        if diff:
            print("Removing unknown variables:", ", ".join(sorted(diff)))
            for vname in diff:
                w_val_dict[sname].pop(vname, None)
    probs = np.asarray(PHB.batch.prob, dtype=np.float64)
    checks = {vname: sum(float(probs[s]) * w_val_dict[sname][vname]
                         for s, sname in enumerate(PHB.local_scenario_names))
              for vname in vn_model}
    gathered = PHB.mpicomm.allgather_object(checks)
    for vname in sorted(vn_model):
        dual = sum(c[vname] for c in gathered)
        if abs(dual) > 1e-7:
            raise RuntimeError("Provided weights do not satisfy dual feasibility: "
                               "\\sum_{scenarios} prob(s) * w(s) != 0. Error on variable " + vname)


# ------------------------------------------------------------------ x-bar
def write_xbar_to_file(PHB, fname):
    """wxbarutils.py:271-291: rank 0 appends the x-bar of its first local scenario."""
    if PHB.cylinder_rank != 0:
        return
    xbar = PHB.engine.host("xbar")[0]
    with open(fname, "a") as f:
        for k, vname in enumerate(nonant_names(PHB)):
            f.write(",".join([vname, str(float(xbar[k]))]) + "\n")


def set_xbar_from_file(fname, PHB):
    """wxbarutils.py:293-315: every local scenario's x-bar from variable_name,value rows
    (x-bar^2 is not kept by this engine: nothing on the hot path reads it)."""
    xbar_val_dict = _parse_xbar_csv(fname)
    if PHB.cylinder_rank == 0:
        _check_xbar(xbar_val_dict, PHB)
    names = nonant_names(PHB)
    missing = [vname for vname in names if vname not in xbar_val_dict]
    if missing:
        raise RuntimeError("Could not find the following required variable values in the provided "
                           "input file: " + ", ".join(missing))
    row = np.array([xbar_val_dict[vname] for vname in names], dtype=np.float64)
    PHB.engine.set_xbar(np.tile(row, (len(PHB.local_scenario_names), 1)))


def _parse_xbar_csv(fname):
    """wxbarutils.py:317-351."""
    results = {}
    with open(fname, "r") as f:
        for line in f:
            if line.startswith("#"):
                continue
            parts = line.split(",")
            results[",".join(parts[:-1])] = float(parts[-1])
    return results


def _check_xbar(xbar_val_dict, PHB):
    """wxbarutils.py:353-370."""
    var_names = set(nonant_names(PHB))
    provided = set(xbar_val_dict.keys())
    set1 = var_names.difference(provided)
    if set1:
        raise RuntimeError("Could not find the following required variable values in the provided "
                           "input file: " + ", ".join(sorted(set1)))
    set2 = provided.difference(var_names)
    if set2:
        print("Ignoring the following variables values provided in the input file: " +
              ", ".join(sorted(set2)))


def ROOT_xbar_npy_serializer(PHB, fname):
    """wxbarutils.py:373-383: the ROOT node's x-bar as a numpy text file."""
    b = PHB.batch
    xbar = PHB.engine.host("xbar")[0]
    root = [float(xbar[k]) for k in range(b.nn) if b.nonant_depth[k] == 0]
    np.savetxt(fname, root)
