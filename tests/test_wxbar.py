"""W / x-bar CSV compatibility (mpisppy/utils/wxbarutils.py,
wxbarwriter.py, wxbarreader.py; test model: mpisppy/tests/test_w_writer.py:85-117).

CPU tests: the parsers and writers against the reference's own fixture files
(tests/golden/ref_w_file.csv / ref_xbar_file.csv, copied from
mpisppy/tests/examples/w_test_data) through a host stand-in for the PH object.
GPU tests: WXBarWriter / WXBarReader on a farmer PH hub, as test_w_writer does."""
import csv
import os
from types import SimpleNamespace

import numpy as np
import pytest

from mpisppy_amd.comm import Comm
from mpisppy_amd.utils import wxbarutils

HERE = os.path.dirname(os.path.abspath(__file__))
W_FILE = os.path.join(HERE, "golden", "ref_w_file.csv")
XBAR_FILE = os.path.join(HERE, "golden", "ref_xbar_file.csv")
NAMES = ["DevotedAcreage[CORN0]", "DevotedAcreage[SUGAR_BEETS0]", "DevotedAcreage[WHEAT0]"]
SCENS = ["scen0", "scen1", "scen2"]


class _Engine:
    def __init__(self, S, nn):
        self.W = np.zeros((S, nn))
        self.xbar = np.zeros((S, nn))

    def set_W(self, W):
        self.W = np.array(W, dtype=float)

    def set_xbar(self, xbar):
        self.xbar = np.array(xbar, dtype=float)

    def host(self, name):
        return getattr(self, name)


def _phb(local=SCENS, allnames=SCENS, names=NAMES):
    b = SimpleNamespace(nonant_names=list(names), nn=len(names), prob=np.full(len(local), 1.0 / len(allnames)),
                        nonant_depth=np.zeros(len(names), dtype=int))
    e = _Engine(len(local), len(names))
    return SimpleNamespace(batch=b, engine=e, local_scenario_names=list(local), all_scenario_names=list(allnames),
                           mpicomm=Comm(), cylinder_rank=0, W_array=lambda: e.W)


def test_parse_reference_w_file():
    """The reference fixture (the same 9 rows appended 8 times) parses to the values
    test_w_writer.py:107-109 asserts."""
    w = wxbarutils._parse_W_csv(W_FILE, SCENS, SCENS, 0)
    assert w["scen0"]["DevotedAcreage[SUGAR_BEETS0]"] == 70.84705093609978
    assert w["scen1"]["DevotedAcreage[CORN0]"] == -41.104251445950844
    ph = _phb()
    wxbarutils.set_W_from_file(W_FILE, ph, 0)
    assert ph.engine.W[0, 1] == 70.84705093609978 and ph.engine.W[1, 0] == -41.104251445950844


def test_parse_reference_xbar_file():
    ph = _phb()
    wxbarutils.set_xbar_from_file(XBAR_FILE, ph)
    assert ph.engine.xbar[0, 1] == 274.2239371483933   # test_w_writer.py:115
    assert ph.engine.xbar[1, 0] == 96.88717449844287    # test_w_writer.py:117
    assert np.all(ph.engine.xbar == ph.engine.xbar[0])


def test_w_round_trip_and_rows(tmp_path):
    ph = _phb()
    rng = np.random.default_rng(0)
    W = rng.normal(size=(3, 3))
    W -= W.mean(0)
    ph.engine.W = W
    f = tmp_path / "w.csv"
    wxbarutils.write_W_to_file(ph, str(f))
    rows = list(csv.reader(open(f)))
    assert [r[:2] for r in rows] == [[s, v] for s in SCENS for v in NAMES]
    assert float(rows[1][2]) == W[0, 1]
    ph2 = _phb()
    wxbarutils.set_W_from_file(str(f), ph2, 0)
    assert np.array_equal(ph2.engine.W, W)                   # str(float) round-trips exactly
    # separate files
    d = tmp_path / "wdir"
    d.mkdir()
    wxbarutils.write_W_to_file(ph, str(d), sep_files=True)
    assert sorted(os.listdir(d)) == [s + "_weights.csv" for s in SCENS]
    ph3 = _phb()
    wxbarutils.set_W_from_file(str(d), ph3, 0, sep_files=True)
    assert np.array_equal(ph3.engine.W, W)


def test_xbar_round_trip(tmp_path):
    ph = _phb()
    ph.engine.xbar = np.tile([96.5, 274.25, 128.0], (3, 1))
    f = tmp_path / "x.csv"
    wxbarutils.write_xbar_to_file(ph, str(f))
    assert [r[0] for r in csv.reader(open(f))] == NAMES
    ph2 = _phb()
    wxbarutils.set_xbar_from_file(str(f), ph2)
    assert np.array_equal(ph2.engine.xbar, ph.engine.xbar)


def test_comments_commas_and_rank_slices(tmp_path):
    """'#' rows are skipped, variable names may contain commas, a rank reads only its
    own scenarios and ignores unknown ones."""
    names = ["x[1,a]", "y"]
    f = tmp_path / "w.csv"
    f.write_text("# header\nscen0,x[1,a],1.5\nscen0,y,-2.0\nscen1,x[1,a],-1.5\nscen1,y,2.0\nbogus,y,3\n")
    ph = _phb(local=["scen1"], allnames=["scen0", "scen1"], names=names)
    wxbarutils.set_W_from_file(str(f), ph, 0, disable_check=True)
    assert ph.engine.W.tolist() == [[-1.5, 2.0]]


def test_errors(tmp_path):
    f = tmp_path / "w.csv"
    f.write_text("scen0,DevotedAcreage[CORN0],1.0\n")
    with pytest.raises(RuntimeError, match="could not find the following scenarios"):
        wxbarutils.set_W_from_file(str(f), _phb(), 0)
    rows = "".join(f"{s},{v},1.0\n" for s in SCENS for v in NAMES[:2])
    f.write_text(rows)
    with pytest.raises(RuntimeError, match="is missing the following variables"):
        wxbarutils.set_W_from_file(str(f), _phb(), 0)
    rows = "".join(f"{s},{v},1.0\n" for s in SCENS for v in NAMES)
    f.write_text(rows)
    with pytest.raises(RuntimeError, match="dual feasibility"):
        wxbarutils.set_W_from_file(str(f), _phb(), 0)
    g = tmp_path / "x.csv"
    g.write_text("DevotedAcreage[CORN0],1\n")
    with pytest.raises(RuntimeError, match="Could not find the following required variable"):
        wxbarutils.set_xbar_from_file(str(g), _phb())


def test_extension_adder_builds_multiextension():
    from mpisppy_amd.utils import cfg_vanilla as vanilla
    from mpisppy_amd.extensions.extension import MultiExtension
    from mpisppy_amd.utils.wxbarreader import WXBarReader
    from mpisppy_amd.utils.wxbarwriter import WXBarWriter
    hub = {"opt_kwargs": {"options": {}, "extensions": None, "extension_kwargs": None}}
    cfg = SimpleNamespace(init_W_fname="a.csv", init_Xbar_fname=None, W_fname="b.csv", Xbar_fname="c.csv")
    vanilla.add_wxbar_read_write(hub, cfg)
    assert hub["opt_kwargs"]["extensions"] is MultiExtension
    assert hub["opt_kwargs"]["extension_kwargs"]["ext_classes"] == [WXBarReader, WXBarWriter]
    assert hub["opt_kwargs"]["options"]["W_fname"] == "b.csv"


# ---------------------------------------------------------------- GPU (test_w_writer.py)
def _farmer_hub(tmp_path, ext, max_iter, **opts):
    from mpisppy_amd.examples import farmer
    from mpisppy_amd.spin_the_wheel import WheelSpinner
    from mpisppy_amd.utils import cfg_vanilla as vanilla
    cfg = SimpleNamespace(solver_name="mi355x_pdhg", default_rho=1.0, max_iterations=max_iter, device="cuda:0",
                          toc=False)
    names = farmer.scenario_names_creator(3)
    hub = vanilla.ph_hub(cfg, farmer.scenario_creator, None, names, scenario_creator_kwargs={"num_scens": 3},
                         ph_extensions=ext)
    hub["opt_kwargs"]["options"].update(opts)
    ws = WheelSpinner(hub, [])
    ws.spin()
    return ws.spcomm.opt


@pytest.mark.gpu
def test_wwriter_xbarwriter(gpu, tmp_path):
    """test_w_writer.py:85-101: W and x-bar after 5 PH iterations (places=5)."""
    from mpisppy_amd.utils.wxbarwriter import WXBarWriter
    wf, xf = str(tmp_path / "w.csv"), str(tmp_path / "x.csv")
    _farmer_hub(tmp_path, WXBarWriter, 5, W_fname=wf, Xbar_fname=xf)
    rows = list(csv.reader(open(wf)))
    assert abs(float(rows[1][2]) - 70.84705093609978) < 1e-5
    assert abs(float(rows[3][2]) - (-41.104251445950844)) < 1e-5
    ref = {(r[0], r[1]): float(r[2]) for r in csv.reader(open(W_FILE))}
    for r in rows:
        assert abs(float(r[2]) - ref[(r[0], r[1])]) < 1e-5
    xrows = list(csv.reader(open(xf)))
    assert abs(float(xrows[1][1]) - 274.2239371483933) < 1e-5
    xref = {r[0]: float(r[1]) for r in csv.reader(open(XBAR_FILE))}
    for r in xrows:
        assert abs(float(r[1]) - xref[r[0]]) < 1e-5


@pytest.mark.gpu
def test_wreader_xbarreader(gpu, tmp_path):
    """test_w_writer.py:103-117: with PHIterLimit 1 the hub ends holding the file values."""
    from mpisppy_amd.utils.wxbarreader import WXBarReader
    ph = _farmer_hub(tmp_path, WXBarReader, 1, init_W_fname=W_FILE, init_Xbar_fname=XBAR_FILE)
    W = ph.W_array()
    xbar = ph.engine.host("xbar")
    assert W[0, 1] == 70.84705093609978
    assert W[1, 0] == -41.104251445950844
    assert xbar[0, 1] == 274.2239371483933
    assert xbar[1, 0] == 96.88717449844287
    assert not ph.W_disabled and not ph.prox_disabled
