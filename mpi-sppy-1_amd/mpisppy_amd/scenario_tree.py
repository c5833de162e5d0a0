"""Scenario tree nodes (mirrors mpisppy/scenario_tree.py:11-96).

A node carries the nonanticipative variables of one stage.  As in the reference,
indexed variables (here: lists / dicts of ``Var``) are expanded in **sorted key
order** (scenario_tree.py:39) -- that order is the flat nonant order used by W, x̄,
the W cache and the GPU nonant map.
"""
from .model import Var


def build_vardatalist(varlist):
    """scenario_tree.py:11-42 for this engine's Var containers.

    * a ``Var``                      -> [var]
    * a ``dict`` key -> Var (indexed) -> vars in sorted(key) order
    * a list / tuple of the above     -> concatenation, in list order
    """
    if varlist is None:
        raise RuntimeError("varlist is None in scenario_tree.build_vardatalist")
    if isinstance(varlist, (Var, dict)):
        varlist = [varlist]
    out = []
    for v in varlist:
        if isinstance(v, dict):
            out.extend(v[k] for k in sorted(v.keys()))
        elif isinstance(v, Var):
            out.append(v)
        else:
            raise TypeError(f"cannot expand nonant entry {v!r}")
    return out


class ScenarioNode:
    """scenario_tree.py:44-96: name, cond_prob, stage, cost expression, nonant vars."""

    def __init__(self, name, cond_prob, stage, cost_expression, nonant_list, scen_model,
                 nonant_ef_suppl_list=None, parent_name=None):
        self.name = name
        self.cond_prob = cond_prob
        self.stage = stage
        self.cost_expression = cost_expression
        self.nonant_list = nonant_list
        self.nonant_ef_suppl_list = nonant_ef_suppl_list
        self.parent_name = parent_name
        if name != "ROOT" and parent_name is None:
            # the reference derives it from the name (scenario_tree.py:72-76)
            self.parent_name = name.rsplit("_", 1)[0]
        self.nonant_vardata_list = build_vardatalist(nonant_list)
        self.uncond_prob = None
