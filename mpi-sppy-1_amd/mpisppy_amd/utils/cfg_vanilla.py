"""Cylinder dict builders (mirrors mpisppy/utils/cfg_vanilla.py:41-495 for the cylinders
this engine serves: ph_hub, lagrangian_spoke, xhatshuffle_spoke; extension_adder and
add_wxbar_read_write for the hub's extensions).

``cfg`` is any object with the reference's config attribute names (solver_name,
default_rho, max_iterations, rel_gap, ...); missing attributes take the reference's
defaults.  The returned dicts feed ``WheelSpinner(hub_dict, list_of_spoke_dict)``.
"""
import copy

from ..cylinders.hub import PHHub
from ..cylinders.lagrangian_bounder import LagrangianOuterBound
from ..cylinders.xhatshufflelooper_bounder import XhatShuffleInnerBound
from ..extensions.extension import MultiExtension
from ..opt.ph import PH
from ..phbase import PHBase
from .xhat_eval import Xhat_Eval
from .wxbarreader import WXBarReader
from .wxbarwriter import WXBarWriter


def _get(cfg, name, default=None):
    v = getattr(cfg, name, default)
    return default if v is None else v


# cfg_vanilla.py:41-62
def shared_options(cfg):
    shoptions = {
        "solver_name": _get(cfg, "solver_name", "mi355x_pdhg"),
        "defaultPHrho": _get(cfg, "default_rho", 1.0),
        "convthresh": 0,
        "PHIterLimit": _get(cfg, "max_iterations", 1),
        "verbose": _get(cfg, "verbose", False),
        "display_progress": _get(cfg, "display_progress", False),
        "display_convergence_detail": _get(cfg, "display_convergence_detail", False),
        "iter0_solver_options": dict(_get(cfg, "iter0_solver_options", {})),
        "iterk_solver_options": dict(_get(cfg, "iterk_solver_options", {})),
        "tee-rank0-solves": _get(cfg, "tee_rank0_solves", False),
        "trace_prefix": getattr(cfg, "trace_prefix", None),
        "device": getattr(cfg, "device", None),
        "toc": _get(cfg, "toc", True),
    }
    if getattr(cfg, "batch_creator", None) is not None:
        shoptions["batch_creator"] = cfg.batch_creator
    return shoptions


# cfg_vanilla.py:77-125
def ph_hub(cfg, scenario_creator, scenario_denouement, all_scenario_names, scenario_creator_kwargs=None,
           ph_extensions=None, extension_kwargs=None, ph_converger=None, rho_setter=None,
           variable_probability=None, all_nodenames=None):
    options = copy.deepcopy(shared_options(cfg))
    options["convthresh"] = _get(cfg, "intra_hub_conv_thresh", 1e-10)
    options["bundles_per_rank"] = _get(cfg, "bundles_per_rank", 0)
    return {
        "hub_class": PHHub,
        "hub_kwargs": {"options": {"rel_gap": getattr(cfg, "rel_gap", None),
                                   "abs_gap": getattr(cfg, "abs_gap", None),
                                   "max_stalled_iters": getattr(cfg, "max_stalled_iters", None)}},
        "opt_class": PH,
        "opt_kwargs": {
            "options": options,
            "all_scenario_names": all_scenario_names,
            "scenario_creator": scenario_creator,
            "scenario_creator_kwargs": scenario_creator_kwargs,
            "scenario_denouement": scenario_denouement,
            "rho_setter": rho_setter,
            "variable_probability": variable_probability,
            "extensions": ph_extensions,
            "extension_kwargs": extension_kwargs,
            "ph_converger": ph_converger,
            "all_nodenames": all_nodenames,
        },
    }


# cfg_vanilla.py:320-353
def lagrangian_spoke(cfg, scenario_creator, scenario_denouement, all_scenario_names,
                     scenario_creator_kwargs=None, rho_setter=None, all_nodenames=None):
    return {
        "spoke_class": LagrangianOuterBound,
        "opt_class": PHBase,
        "opt_kwargs": {
            "options": copy.deepcopy(shared_options(cfg)),
            "all_scenario_names": all_scenario_names,
            "scenario_creator": scenario_creator,
            "scenario_creator_kwargs": scenario_creator_kwargs,
            "scenario_denouement": scenario_denouement,
            "rho_setter": rho_setter,
            "all_nodenames": all_nodenames,
        },
    }


# cfg_vanilla.py:457-492
def xhatshuffle_spoke(cfg, scenario_creator, scenario_denouement, all_scenario_names, all_nodenames=None,
                      scenario_creator_kwargs=None):
    shoptions = shared_options(cfg)
    xhat_options = copy.deepcopy(shoptions)
    xhat_options["bundles_per_rank"] = 0
    xhat_options["xhat_looper_options"] = {
        "xhat_solver_options": shoptions["iterk_solver_options"],
        "dump_prefix": "delme",
        "csvname": "looper.csv",
        "tries_per_sync": _get(cfg, "xhat_tries_per_sync", 1),
    }
    if getattr(cfg, "add_reversed_shuffle", None) is not None:
        xhat_options["xhat_looper_options"]["reverse"] = cfg.add_reversed_shuffle
    if getattr(cfg, "xhatshuffle_iter_step", None) is not None:
        xhat_options["xhat_looper_options"]["iter_step"] = cfg.xhatshuffle_iter_step
    return {
        "spoke_class": XhatShuffleInnerBound,
        "opt_class": Xhat_Eval,
        "opt_kwargs": {
            "options": xhat_options,
            "all_scenario_names": all_scenario_names,
            "scenario_creator": scenario_creator,
            "scenario_creator_kwargs": scenario_creator_kwargs,
            "scenario_denouement": scenario_denouement,
            "all_nodenames": all_nodenames,
        },
    }


# cfg_vanilla.py:164-181
def extension_adder(hub_dict, ext_class):
    ok = hub_dict["opt_kwargs"]
    if ok.get("extensions") is None:
        ok["extensions"] = ext_class
    elif ok["extensions"] == MultiExtension:
        if ok.get("extension_kwargs") is None:
            ok["extension_kwargs"] = {"ext_classes": []}
        if ext_class not in ok["extension_kwargs"]["ext_classes"]:
            ok["extension_kwargs"]["ext_classes"].append(ext_class)
    elif ok["extensions"] != ext_class:
        ok["extension_kwargs"] = {"ext_classes": [ok["extensions"], ext_class]}
        ok["extensions"] = MultiExtension
    return hub_dict


# cfg_vanilla.py:202-224 (options stay loose in the hub's options dict, as there)
def add_wxbar_read_write(hub_dict, cfg):
    if getattr(cfg, "init_W_fname", None) is not None or getattr(cfg, "init_Xbar_fname", None) is not None:
        hub_dict = extension_adder(hub_dict, WXBarReader)
        hub_dict["opt_kwargs"]["options"].update({
            "init_W_fname": getattr(cfg, "init_W_fname", None),
            "init_Xbar_fname": getattr(cfg, "init_Xbar_fname", None),
            "init_separate_W_files": bool(getattr(cfg, "init_separate_W_files", False)),
        })
    if getattr(cfg, "W_fname", None) is not None or getattr(cfg, "Xbar_fname", None) is not None:
        hub_dict = extension_adder(hub_dict, WXBarWriter)
        hub_dict["opt_kwargs"]["options"].update({
            "W_fname": getattr(cfg, "W_fname", None),
            "Xbar_fname": getattr(cfg, "Xbar_fname", None),
            "separate_W_files": bool(getattr(cfg, "separate_W_files", False)),
        })
    return hub_dict
