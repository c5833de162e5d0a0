"""Per-scenario extension hooks pre_solve / post_solve (spopt.py:146-147, 220-221;
extensions/extension.py:18-45): they bracket the batched solve, once per local scenario per
solve_loop, post_solve with the scenario's solution loaded and a results object in the
Pyomo shape (termination condition, Lower_bound / Upper_bound; 'infeasible' / 'unbounded'
with an empty solution for a certified failure).

CPU: which hooks an extension overrides (the loop keeps its speculative solve unless a hook
that needs the reference's order is defined).  GPU: farmer (per-scenario models) and the
batch creator (ScenarioViews) through PH, the hooks' view of each solve against the
engine's outputs, and the PH results unchanged by them."""
import numpy as np
import pytest

from mpisppy_amd.extensions.extension import Extension, MultiExtension, overrides


class Recorder(Extension):
    def __init__(self, opt):
        super().__init__(opt)
        self.log = []

    def pre_solve(self, subproblem):
        self.log.append(("pre", subproblem.name))

    def post_solve(self, subproblem, results):
        self.log.append(("post", subproblem.name, results))
        return results


class EndOnly(Extension):
    def enditer(self):
        pass


def test_overrides():
    assert overrides(Recorder(None), "pre_solve") and overrides(Recorder(None), "post_solve")
    assert not overrides(Recorder(None), "miditer")
    assert not overrides(EndOnly(None), "pre_solve") and overrides(EndOnly(None), "enditer")
    assert not overrides(None, "pre_solve")
    m = MultiExtension(None, [EndOnly])
    assert not overrides(m, "post_solve")
    m = MultiExtension(None, [EndOnly, Recorder])
    assert overrides(m, "post_solve")

    class Duck:  # a duck-typed extension object (not an Extension subclass)
        def pre_solve(self, s):
            pass
    assert overrides(Duck(), "pre_solve") and not overrides(Duck(), "post_solve")


def _opts(**kw):
    o = {"solver_name": "mi355x_pdhg", "PHIterLimit": 3, "defaultPHrho": 1.0, "convthresh": -1.0,
         "verbose": False, "display_progress": False, "toc": False}
    o.update(kw)
    return o


def test_speculation_follows_the_hooks():
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    import types

    def mk(ext):
        ph = PH(_opts(), farmer.scenario_names_creator(3), farmer.scenario_creator,
                scenario_creator_kwargs={"num_scens": 3}, extensions=ext)
        ph.engine = types.SimpleNamespace(shared=False)  # (no device here)
        return ph
    assert mk(EndOnly)._speculate(True)
    assert not mk(Recorder)._speculate(True)


@pytest.mark.gpu
def test_hooks_bracket_every_solve_with_models(gpu):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    ph = PH(_opts(device="cuda:0"), farmer.scenario_names_creator(3), farmer.scenario_creator,
            scenario_creator_kwargs={"num_scens": 3}, extensions=Recorder)
    conv, eobj, tb = ph.ph_main()
    log = ph.extobject.log
    names = ["scen0", "scen1", "scen2"]
    # Iter0 + 3 PH iterations, each: 3 pre then 3 post in scenario order
    assert len(log) == 4 * 6
    for k in range(4):
        blk = log[6 * k:6 * k + 6]
        assert [e[:2] for e in blk] == [("pre", n) for n in names] + [("post", n) for n in names]
    # the last solve's results against the engine, and the solution loaded into the models
    x = ph.engine.host("x")
    obj, bd = ph.engine.host("obj"), ph.engine.host("bound")
    for k, (_, n, res) in enumerate(log[-3:]):
        assert res.solver.termination_condition == "optimal" and res.status == 0 and res.solution
        assert res.Problem[0].Upper_bound == pytest.approx(obj[k], rel=1e-12)
        assert res.Problem[0].Lower_bound == pytest.approx(bd[k], rel=1e-12)
        assert res.Problem[0].Lower_bound <= res.Problem[0].Upper_bound + 1e-6 * abs(obj[k])
        mdl = ph.local_scenarios[n]
        np.testing.assert_array_equal([v._value for v in mdl.vars], x[k])
    # the hooks observe only: same PH results as without them (unspeculated loop order)
    ref = PH(_opts(device="cuda:0", speculative_solve=False), farmer.scenario_names_creator(3),
             farmer.scenario_creator, scenario_creator_kwargs={"num_scens": 3})
    c2, e2, t2 = ref.ph_main()
    assert (conv, eobj, tb) == (c2, e2, t2)
    np.testing.assert_array_equal(ph.W_array(), ref.W_array())


@pytest.mark.gpu
def test_hooks_on_a_batch_creator(gpu):
    from mpisppy_amd.opt.ph import PH
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.spopt import ScenarioView
    ph = PH(_opts(device="cuda:0", PHIterLimit=1, batch_creator=farmer.batch_creator),
            farmer.scenario_names_creator(64), farmer.scenario_creator,
            scenario_creator_kwargs={"num_scens": 64}, extensions=Recorder)
    ph.ph_main()
    log = ph.extobject.log
    assert len(log) == 2 * 128
    post = [e for e in log[-64:]]
    assert all(e[0] == "post" and e[2].solver.termination_condition == "optimal" for e in post)
    assert [e[1] for e in post] == ph.local_scenario_names
    v = ScenarioView(ph, 5, ph.local_scenario_names[5])
    np.testing.assert_array_equal(v.x, ph.engine.host("x")[5])


def test_results_object_for_failed_and_optimal_solves():
    """a certified infeasible / unbounded scenario gets a results object with that
    termination condition and an empty solution (spopt.py:165-221), not None; the solution
    set is callable like Pyomo's (results.solution(0))."""
    from mpisppy_amd import _lib
    from mpisppy_amd.spopt import ScenarioResults
    r = ScenarioResults(_lib.PRIMAL_INFEASIBLE, float("inf"), float("inf"), 600)
    assert r.solver.termination_condition == "infeasible" and len(r.solution) == 0 and not r.solution
    r = ScenarioResults(_lib.DUAL_INFEASIBLE, -float("inf"), -float("inf"), 600)
    assert r.solver.termination_condition == "unbounded" and r.solver.status == "warning"
    r = ScenarioResults(_lib.OPTIMAL, 3.0, 2.5, 7, sense=-1)
    assert r.solution(0) is r and r.solution[0] is r
    assert (r.Problem[0].Lower_bound, r.Problem[0].Upper_bound) == (3.0, 2.5)
