"""Per-step dispatch sequence from a rocprofv3 kernel trace (run_kernel_trace.csv): the
dispatches between the last few solve launches with their durations and the idle gaps
before them.  Usage: python tools/step_trace.py run_kernel_trace.csv [steps]"""
import csv
import sys


def main():
    rows = sorted(csv.DictReader(open(sys.argv[1])), key=lambda d: int(d["Start_Timestamp"]))
    steps = int(sys.argv[2]) if len(sys.argv) > 2 else 2
    idx = [i for i, d in enumerate(rows) if d["Kernel_Name"].startswith("k_solve_ipm")
           or d["Kernel_Name"].startswith("k_solve_reg")]
    a, b = idx[-1 - steps], idx[-1]
    t0 = int(rows[a]["Start_Timestamp"])
    prev = None
    busy = gap = 0.0
    for d in rows[a:b]:
        s, e = int(d["Start_Timestamp"]), int(d["End_Timestamp"])
        g = (s - prev) / 1e3 if prev is not None else 0.0
        busy += (e - s) / 1e3
        gap += max(g, 0.0)
        print(f"{(s - t0) / 1e3:9.2f} us  {(e - s) / 1e3:7.2f}  gap {g:6.2f}  {d['Kernel_Name'][:70]}")
        prev = e
    print(f"per step: busy {busy / steps:.1f} us, idle {gap / steps:.1f} us")


if __name__ == "__main__":
    main()
