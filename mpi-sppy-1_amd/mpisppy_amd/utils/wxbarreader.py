"""WXBarReader extension: start PH from W and/or x-bar read from CSV files
(mirrors mpisppy/utils/wxbarreader.py:36-97).

Options (the hub's PH options dict):
    "init_W_fname"           file (or directory with "init_separate_W_files") of W
    "init_Xbar_fname"        file of x-bar
    "init_separate_W_files"  read <scenario>_weights.csv files from init_W_fname

At PH iteration 1, after x-bar / W have been updated and before the solve (miditer),
the file values overwrite the engine's device W / x-bar and the W / prox terms are
switched on (wxbarreader.py:80-90).  A missing file raises RuntimeError where the
reference prints and calls quit() (wxbarreader.py:46-61).
"""
import os

from ..extensions.extension import Extension
from . import wxbarutils


class WXBarReader(Extension):
    def __init__(self, ph):
        super().__init__(ph)
        opts = ph.options
        sep_files = bool(opts.get("init_separate_W_files", False))
        w_fname = opts.get("init_W_fname")
        x_fname = opts.get("init_Xbar_fname")
        if w_fname is not None and not os.path.exists(w_fname):
            raise RuntimeError(("Cannot find path " if sep_files else "Cannot find file ") + str(w_fname))
        if x_fname is not None and not os.path.exists(x_fname):
            raise RuntimeError("Cannot find file " + str(x_fname))
        if x_fname is None and w_fname is None and ph.cylinder_rank == 0:
            print("Warning: no input files provided to WXBarReader. "
                  "W and Xbar will be initialized to their default values.")
        self.PHB = ph
        self.cylinder_rank = ph.cylinder_rank
        self.w_fname = w_fname
        self.x_fname = x_fname
        self.sep_files = sep_files

    # wxbarreader.py:80-90
    def miditer(self):
        if self.PHB._PHIter == 1:
            if self.w_fname:
                wxbarutils.set_W_from_file(self.w_fname, self.PHB, self.cylinder_rank, sep_files=self.sep_files)
                self.PHB._reenable_W()
            if self.x_fname:
                wxbarutils.set_xbar_from_file(self.x_fname, self.PHB)
                self.PHB._reenable_prox()
