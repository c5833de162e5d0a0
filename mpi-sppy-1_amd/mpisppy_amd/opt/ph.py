"""PH (mirrors mpisppy/opt/ph.py:18-71)."""
from ..phbase import PHBase


class PH(PHBase):
    """PH. See PHBase for the list of args."""

    def ph_main(self, finalize=True):
        """PH_Prep -> Iter0 -> iterk_loop -> post_loops; returns (conv, Eobj, trivial_bound)
        exactly as opt/ph.py:25-71 (Eobj is None when finalize is False)."""
        self.PH_Prep()
        trivial_bound = self.Iter0()
        if self.options.get("asynchronousPH", False):
            raise RuntimeError("asynchronousPH is deprecated; use APH")
        self.iterk_loop()
        Eobj = self.post_loops(self.extensions) if finalize else None
        return self.conv, Eobj, trivial_bound
