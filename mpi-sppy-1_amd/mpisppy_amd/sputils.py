"""Scenario-tree and naming utilities (mirrors mpisppy/utils/sputils.py).

Only what the PH hot path needs: ``extract_num`` (sputils.py:481-490), the balanced
tree helpers (``node_idx`` 494-519, ``_nodenum_before_stage`` 654-657,
``create_nodenames_from_branching_factors`` 934-959), ``attach_root_node``
(844-860) and the rank partition of ``_ScenTree.scen_names_to_ranks`` (774-840).
"""
import re
import numpy as np

from .scenario_tree import ScenarioNode


def extract_num(string):
    """Longest run of digits at the right end of ``string`` (sputils.py:481-490)."""
    return int(re.compile(r"(\d+)$").search(string).group(1))


def _nodenum_before_stage(t, branching_factors):
    return int(sum(np.prod(branching_factors[0:i]) for i in range(t)))


def node_idx(node_path, branching_factors):
    if node_path == []:
        return 0
    stage_id = 0
    for t in range(len(node_path)):
        stage_id = node_path[t] + branching_factors[t] * stage_id
    return _nodenum_before_stage(len(node_path), branching_factors) + stage_id


def create_nodenames_from_branching_factors(BFS):
    stage_nodes = ["ROOT"]
    nodenames = ["ROOT"]
    if len(BFS) == 1:
        return nodenames
    for bf in BFS:
        old = stage_nodes
        stage_nodes = []
        for k in range(len(old)):
            stage_nodes += ["%s_%i" % (old[k], b) for b in range(bf)]
        nodenames += stage_nodes
    return nodenames


def attach_root_node(model, firstobj, varlist, nonant_ef_suppl_list=None):
    """sputils.py:844-860: a two-stage scenario has the single node ROOT."""
    model._mpisppy_node_list = [
        ScenarioNode("ROOT", 1.0, 1, firstobj, varlist, model,
                     nonant_ef_suppl_list=nonant_ef_suppl_list)
    ]


def rank_slices(num_scens, n_proc):
    """Contiguous scenario slices per rank, sputils.py:798-810 (n_proc == 1 special
    case 798-801; ``range(int(i*avg), int((i+1)*avg))`` otherwise)."""
    if n_proc == 1:
        return [list(range(num_scens))]
    avg = num_scens / n_proc
    return [list(range(int(i * avg), int((i + 1) * avg))) for i in range(n_proc)]


def option_string_to_dict(ostr):
    """sputils.option_string_to_dict: 'a=1 b' -> {'a': 1.0, 'b': None}."""
    def convert_value_string_to_number(s):
        try:
            return int(s)
        except ValueError:
            try:
                return float(s)
            except ValueError:
                return s
    solver_options = dict()
    if ostr is None or ostr == "":
        return solver_options
    for this_option_string in ostr.split():
        this_option_pieces = this_option_string.strip().split("=")
        if len(this_option_pieces) == 2:
            solver_options[this_option_pieces[0]] = convert_value_string_to_number(this_option_pieces[1])
        elif len(this_option_pieces) == 1:
            solver_options[this_option_pieces[0]] = None
        else:
            raise RuntimeError("Illegally formed subsolve directive option=%s detected" % this_option_string)
    return solver_options


class TreeNode:
    """Non-leaf / leaf node of the scenario tree with the contiguous range of scenario
    indices below it (the scenfirst / scenlast / kids / is_leaf of sputils._TreeNode,
    sputils.py:672-726)."""

    def __init__(self, name, stage, scenfirst, scenlast):
        self.name = name
        self.stage = stage
        self.scenfirst = scenfirst
        self.scenlast = scenlast
        self.kids = []

    @property
    def is_leaf(self):
        return not self.kids


def scenario_tree(all_nodenames, num_scens):
    """{name: TreeNode} for every node of all_nodenames (sputils._ScenTree, 743-772).

    Two-stage (all_nodenames None or ['ROOT']): ROOT spans all scenarios and has no kids.
    Multistage: leaves are the nodes without a child '<name>_0'; every leaf is one
    scenario and a node's scenarios are its descendant leaves, in name order."""
    if all_nodenames is None or list(all_nodenames) == ["ROOT"]:
        return {"ROOT": TreeNode("ROOT", 1, 0, num_scens - 1)}
    names = set(all_nodenames)

    def children(nd):
        out = []
        i = 0
        while f"{nd}_{i}" in names:
            out.append(f"{nd}_{i}")
            i += 1
        return out

    nodes = {}

    def build(nd, stage, first):
        kids = children(nd)
        if not kids:
            nodes[nd] = TreeNode(nd, stage, first, first)
            return first + 1
        nxt = first
        for k in kids:
            nxt = build(k, stage + 1, nxt)
        node = TreeNode(nd, stage, first, nxt - 1)
        node.kids = [nodes[k] for k in kids]
        nodes[nd] = node
        return nxt

    last = build("ROOT", 1, 0)
    if last != num_scens:
        raise RuntimeError(f"The all_nodenames argument gives {last} leaves for {num_scens} scenarios")
    ordered = {}

    def preorder(t):          # _ScenTree.nonleaves order: node, then its subtrees
        ordered[t.name] = t
        for k in t.kids:
            preorder(k)
    preorder(nodes["ROOT"])
    return ordered
