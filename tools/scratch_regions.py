"""Where a kernel's scratch (spill) operations sit: per loop of the disassembly.

    python tools/scratch_regions.py [--co CODE_OBJECT] [KERNEL_SUBSTRING ...]

Without --co it compiles csrc/phgpu.hip for gfx950 (device only, ~75 s) and unbundles the
code object.  For every kernel whose mangled name contains one of the substrings it
prints the scratch size from the code-object notes, then every loop (a backward branch
and the range it closes) with its LDS reads / writes, fp64 VALU operations and
scratch_load / scratch_store count.  The PDHG step loop of k_solve_reg is the innermost
loop with at least two ds_write_b64 and four ds_read_b64 (the x~ / T(y) hand-offs and
their gathers).
"""
import argparse
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"


def build_co(out_dir):
    dev = os.path.join(out_dir, "dev.co")
    co = os.path.join(out_dir, "gfx950.co")
    subprocess.run(["/opt/rocm/bin/hipcc", "--offload-arch=gfx950", "-O3", "-std=c++17", "-I",
                    os.path.join(ROOT, "include"), "--cuda-device-only", "-c", "-o", dev,
                    os.path.join(ROOT, "mpi-sppy-1_amd", "csrc", "phgpu.hip")], check=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--unbundle", "--type=o", f"--input={dev}",
                    "--targets=hipv4-amdgcn-amd-amdhsa--gfx950", f"--output={co}"], check=True)
    return co


def notes(co):
    txt = subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                         text=True).stdout
    cur, rows = {}, {}
    for line in txt.splitlines():
        m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
        if not m:
            continue
        k, v = m.groups()
        if k == "agpr_count" and cur.get("name"):
            rows[cur["name"]] = cur
            cur = {}
        cur[k] = v
    if cur.get("name"):
        rows[cur["name"]] = cur
    return rows


def functions(co):
    txt = subprocess.run([f"{LLVM}/llvm-objdump", "-d", "--no-show-raw-insn", co], check=True,
                         capture_output=True, text=True).stdout
    out, name, body = {}, None, []
    for line in txt.splitlines():
        m = re.match(r"^[0-9a-f]+ <(.+)>:$", line)
        if m:
            if name:
                out[name] = body
            name, body = m.group(1), []
        elif name:
            body.append(line)
    if name:
        out[name] = body
    return out


def loops(body):
    off = []
    for l in body:
        m = re.search(r"//\s*([0-9A-F]{6,}):", l)
        off.append(int(m.group(1), 16) if m else None)
    base = next(o for o in off if o is not None)
    idx = {o - base: i for i, o in enumerate(off) if o is not None}
    res = []
    for i, l in enumerate(body):
        m = re.search(r"(s_cbranch_\w+|s_branch)\s.*\+0x([0-9a-f]+)>", l)
        if m and off[i] is not None:
            t = int(m.group(2), 16)
            if t < off[i] - base and t in idx:
                res.append((idx[t], i))
    return res


def count(lines, pat):
    return sum(1 for x in lines if pat in x)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--co", default=None)
    ap.add_argument("kernels", nargs="*", default=["k_solve_reg"])
    a = ap.parse_args()
    co = a.co or build_co(tempfile.mkdtemp())
    meta = notes(co)
    for name, body in functions(co).items():
        if not any(k in name for k in a.kernels):
            continue
        md = meta.get(name, {})
        print(f"{name}\n  vgpr {md.get('vgpr_count')} scratch {md.get('private_segment_fixed_size')} B, "
              f"{count(body, 'scratch_')} scratch ops in {len(body)} instructions")
        step = None
        for s, e in loops(body):
            seg = body[s:e + 1]
            rd, wr = count(seg, "ds_read_b64"), count(seg, "ds_write_b64")
            if rd >= 4 and wr >= 2 and (step is None or e - s < step[1] - step[0]):
                step = (s, e)
        for s, e in loops(body):
            seg = body[s:e + 1]
            sc = count(seg, "scratch_")
            if e - s < 40 and not sc:
                continue
            tag = "  <- PDHG step loop" if step == (s, e) else ""
            print(f"  loop [{s}, {e}] {e - s:5d} instr: ds_read {count(seg, 'ds_read'):3d} "
                  f"ds_write {count(seg, 'ds_write'):3d} f64 {count(seg, '_f64'):4d} "
                  f"scratch {sc:3d}{tag}")
        if step:
            print(f"  step loop scratch ops: {count(body[step[0]:step[1] + 1], 'scratch_')}")
    return 0


if __name__ == "__main__":
    sys.exit(main())
