"""Write the generated path-6 source for a farmer / aircond batch and compile it offline
to gfx950 assembly (TOOL ONLY): the hipRTC module's code, for reading its loop.

    python tools/ipm_isa.py S lanes out_prefix [--model aircond] [--cm CM]
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
sys.path.insert(0, ROOT)

ap = argparse.ArgumentParser()
ap.add_argument("S", type=int)
ap.add_argument("lanes", type=int)
ap.add_argument("out")
ap.add_argument("--model", default="farmer")
ap.add_argument("--cm", type=int, default=1)
ap.add_argument("--maxilp", action="store_true")
ap.add_argument("-D", action="append", default=[])
ap.add_argument("--wpe", type=int, default=0, help="lane-group kernel: waves per SIMD budget (ML_WPE)")
a = ap.parse_args()
import mpisppy_amd._lib as L  # noqa: E402
if a.model == "farmer":
    from mpisppy_amd.examples import farmer
    b = farmer.batch_creator(farmer.scenario_names_creator(a.S), crops_multiplier=a.cm, num_scens=a.S)
else:
    import numpy as np
    from mpisppy_amd.examples import aircond
    from bench import AIRCOND_KW
    bf = [4, 32, 64] if a.S == 8192 else [32, 32, 64]
    b = aircond.batch_creator(aircond.scenario_names_creator(int(np.prod(bf))), branching_factors=bf, **AIRCOND_KW)
src, _ = L.ipm_source(b, a.lanes)
if a.wpe:
    a.D.append(f"ML_WPE={a.wpe}")
    if "ML_WPE" not in src:  # a library built before the knob: patch the kernel header
        src = src.replace("extern \"C\" __global__ void __launch_bounds__(256) k_solve_ipm_ml",
                          "extern \"C\" __global__ void __launch_bounds__(256) "
                          "__attribute__((amdgpu_waves_per_eu(ML_WPE, ML_WPE))) k_solve_ipm_ml")
defs = "".join(f"#define {d.split('=')[0]} {d.split('=', 1)[1] if '=' in d else 1}\n" for d in a.D)
open(a.out + ".hip", "w").write("#include <hip/hip_runtime.h>\n" + defs + src)
cmd = ["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "--cuda-device-only", "-S", "-o",
       a.out + ".s", a.out + ".hip"]
if a.maxilp:
    cmd[4:4] = ["-mllvm", "-amdgpu-sched-strategy=max-ilp"]
subprocess.run(cmd, check=True)
txt = open(a.out + ".s").read()
for key in ("vgpr_count", "agpr_count", "sgpr_count", "private_segment_fixed_size", "group_segment_fixed_size"):
    import re
    print(key, re.findall(rf"\.{key}:\s+(\d+)", txt)[:3])
