"""WXBarWriter extension: save W and/or x-bar to CSV files at the end of the run
(mirrors mpisppy/utils/wxbarwriter.py:36-101).

Options (the hub's PH options dict, as in the reference):
    "W_fname"          file (or directory when "separate_W_files" is True) for W
    "Xbar_fname"       file for x-bar
    "separate_W_files" one <scenario>_weights.csv per scenario under W_fname
Files are appended to, as in the reference; the format is wxbarutils'.
"""
import os

from ..extensions.extension import Extension
from . import wxbarutils


class WXBarWriter(Extension):
    def __init__(self, ph):
        super().__init__(ph)
        opts = ph.options
        w_fname = opts.get("W_fname")
        x_fname = opts.get("Xbar_fname")
        sep_files = bool(opts.get("separate_W_files", False))
        rank = ph.cylinder_rank
        if x_fname is None and w_fname is None and rank == 0:
            print("Warning: no output files provided to WXBarWriter. No values will be saved.")
        if w_fname and not sep_files and os.path.exists(w_fname) and rank == 0:
            print(f"Warning: specified W_fname ({w_fname}) already exists. Results will be appended to this file.")
        elif w_fname and sep_files and not os.path.exists(w_fname):
            if rank == 0:
                print(f"Warning: path {w_fname} does not exist. Creating...")
            os.makedirs(w_fname, exist_ok=True)
        if x_fname and os.path.exists(x_fname) and rank == 0:
            print(f"Warning: specified Xbar_fname ({x_fname}) already exists. Results will be appended to this file.")
        self.PHB = ph
        self.cylinder_rank = rank
        self.w_fname = w_fname
        self.x_fname = x_fname
        self.sep_files = sep_files

    # wxbarwriter.py:91-101
    def post_everything(self):
        if self.w_fname:
            wxbarutils.write_W_to_file(self.PHB, self.w_fname, sep_files=self.sep_files)
        if self.x_fname:
            wxbarutils.write_xbar_to_file(self.PHB, self.x_fname)
