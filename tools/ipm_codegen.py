"""Generate the path-6 (interior point) source for farmer / aircond batches with the
library's own generator (phgpu_ipm_source, no GPU), compile it offline for gfx950 and
print the kernel's register / scratch use.  Usage: python tools/ipm_codegen.py [out_dir]"""
import os
import re
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "mpi-sppy-1_amd"))
sys.path.insert(0, ROOT)


def batches():
    from mpisppy_amd.examples import farmer, aircond
    from bench import AIRCOND_KW
    yield "farmer", farmer.batch_creator(farmer.scenario_names_creator(64))
    yield "aircond", aircond.batch_creator(aircond.scenario_names_creator(64), branching_factors=[4, 4, 4],
                                           **AIRCOND_KW)


def compile_report(src, path):
    with open(path, "w") as f:
        f.write("#include <hip/hip_runtime.h>\n" + src)
    r = subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-c", "--cuda-device-only",
                        "-Rpass-analysis=kernel-resource-usage", "-o", path + ".o", path],
                       capture_output=True, text=True)
    if r.returncode:
        raise RuntimeError(r.stderr[-4000:])
    out = {}
    fn = None
    for line in r.stderr.splitlines():
        m = re.search(r"Function Name: (\w+)", line)
        if m:
            fn = m.group(1)
            out[fn] = {}
        m = re.search(r"remark:\s+([A-Za-z][^:]*?): (\d+)", line)
        if m and fn:
            out[fn][m.group(1).strip()] = int(m.group(2))
    return out


def main():
    import mpisppy_amd._lib as L
    od = sys.argv[1] if len(sys.argv) > 1 else "/tmp"
    tmpl = open(os.path.join(ROOT, "mpi-sppy-1_amd", "csrc", "jit_ipm.hip.in")).read()
    for name, b in batches():
        src, (mr, nf, _, _) = L.ipm_source(b)
        # the IPM part only, with the template as it is on disk (no library rebuild needed)
        src = src[src.index("#define IPM_GAM"):src.index("// jit_ipm.hip.in --")] + tmpl
        rep = compile_report(src, os.path.join(od, f"ipm_{name}.hip"))
        print(name, f"n={b.n} m={b.m} nnz={b.nnz} rows={mr} factor={nf}")
        for fn, d in rep.items():
            if fn != "k_solve_ipm":
                continue
            print("  ", fn, {k: v for k, v in d.items() if k in ("VGPRs", "AGPRs", "ScratchSize [bytes/lane]", "VGPRs Spill",
                                                              "SGPRs Spill")})


if __name__ == "__main__":
    main()
