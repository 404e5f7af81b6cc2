"""Kernel-trace window check: which kernels run between the first and last launch of the final
forward pass (first fc1 GEMM of the last 12 / last head GEMM), from a rocprofv3 --kernel-trace
CSV directory.  Usage: python scripts/trace_window.py <rocprof output dir>"""
import collections
import csv
import glob
import os
import sys


def main(d):
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = list(csv.DictReader(open(f)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    name = lambda r: r["Kernel_Name"]  # noqa: E731
    norm = lambda s: s.replace("true", "T").replace("false", "F").replace(" ", "")  # noqa: E731
    fc1 = [i for i, r in enumerate(rows) if "gemm_bf16_kernel<1," in norm(name(r))]
    head = [i for i, r in enumerate(rows) if "gemm_bf16_kernel<" in norm(name(r)) and ",2,T,1>" in norm(name(r))]
    if len(fc1) < 12 or not head:
        print("kernel names:", sorted({norm(name(r))[:90] for r in rows if "gemm" in name(r)}))
        return
    lo, hi = fc1[-12], head[-1]
    win = rows[lo - 8:hi + 1]
    t0, t1 = int(win[0]["Start_Timestamp"]), int(win[-1]["End_Timestamp"])
    c = collections.Counter(name(r)[:70] for r in win)
    busy = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in win)
    print(f"last pass window: {len(win)} kernels, {(t1 - t0) / 1e6:.2f} ms wall, {busy / 1e6:.2f} ms busy")
    for k, v in c.most_common():
        print(f"  {v:4d}  {k}")


if __name__ == "__main__":
    main(sys.argv[1])
