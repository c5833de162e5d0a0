"""Extension hooks of the PH loop (mirrors mpisppy/extensions/extension.py:12-170).

The hook points and their place in the loop are the reference's (phbase.py Iter0 /
iterk_loop / post_loops; spopt.py solve_loop).  The per-scenario ``pre_solve`` /
``post_solve`` bracket the one batched device solve that replaces the reference's
``solve_one`` calls (spopt.py:146-147, 220-221): every local scenario's ``pre_solve`` runs
before the launch, every ``post_solve`` after it, with the scenario's solution loaded and a
results object per scenario (``spopt.ScenarioResults``; None for an infeasible or unbounded
one, as the reference passes).  A hook that edits a scenario's model does not change the
batched solve (its data are on the device); ``overrides`` tells which hooks an extension
defines, so the others cost nothing.
"""


class Extension:
    """Base class: every hook is a no-op; ``self.opt`` is the SPOpt/PHBase object."""

    def __init__(self, spopt_object):
        self.opt = spopt_object

    def pre_solve(self, subproblem):
        pass

    def post_solve(self, subproblem, results):
        return results

    def pre_solve_loop(self):
        pass

    def post_solve_loop(self):
        pass

    def pre_iter0(self):
        pass

    def post_iter0(self):
        pass

    def post_iter0_after_sync(self):
        pass

    def miditer(self):
        pass

    def enditer(self):
        pass

    def enditer_after_sync(self):
        pass

    def post_everything(self):
        pass


_HOOKS = ("pre_solve_loop", "post_solve_loop", "pre_iter0", "post_iter0", "post_iter0_after_sync",
          "miditer", "enditer", "enditer_after_sync", "post_everything")


class MultiExtension(Extension):
    """Several extensions as one (extension.py:113-170): constructed in list order,
    each hook fans out in that order; ``extdict`` maps class name -> instance."""

    def __init__(self, ph, ext_classes):
        super().__init__(ph)
        self.extdict = {cls.__name__: cls(ph) for cls in ext_classes}

    def pre_solve(self, subproblem):
        for e in self.extdict.values():
            e.pre_solve(subproblem)

    def post_solve(self, subproblem, results):
        for e in self.extdict.values():
            results = e.post_solve(subproblem, results)
        return results


def _fan_out(name):
    def hook(self):
        for e in self.extdict.values():
            getattr(e, name)()
    hook.__name__ = name
    return hook


for _h in _HOOKS:
    setattr(MultiExtension, _h, _fan_out(_h))


def overrides(ext, name):
    """True if ``ext`` defines hook ``name`` beyond the base class's no-op (for a
    MultiExtension: if any member does).  The PH loop skips, or keeps its speculative
    solve around, hooks that do nothing."""
    if ext is None:
        return False
    if isinstance(ext, MultiExtension):
        return any(overrides(e, name) for e in ext.extdict.values())
    f = getattr(type(ext), name, None)
    if f is None:
        return callable(getattr(ext, name, None))
    return f is not getattr(Extension, name, None)
