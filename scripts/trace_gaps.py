"""Gaps between consecutive kernels of a rocprofv3 kernel trace (e.g. the row -> column hand-off of
one rfft2 call inside a graph replay).

  python scripts/trace_gaps.py gpurun_out/fft_trace_r4s05 [name-substring ...]
"""
import collections
import csv
import glob
import os
import statistics
import sys


def main(argv):
    d = argv[1]
    pats = argv[2:]
    f = sorted(glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True))[0]
    rows = sorted(csv.DictReader(open(f)), key=lambda r: int(r["Start_Timestamp"]))
    rows = [r for r in rows if not pats or any(p in r["Kernel_Name"] for p in pats)]
    gaps = collections.defaultdict(list)
    durs = collections.defaultdict(list)
    short = lambda n: n.replace("amd_dft::(anonymous namespace)::", "")[:60]  # noqa: E731
    for a, b in zip(rows, rows[1:]):
        g = (int(b["Start_Timestamp"]) - int(a["End_Timestamp"])) / 1e3
        if 0 <= g < 50:  # same burst (graph replay), not host gaps
            gaps[(short(a["Kernel_Name"]), short(b["Kernel_Name"]))].append(g)
    for r in rows:
        durs[short(r["Kernel_Name"])].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    print("kernel durations (us): median / n")
    for k, v in sorted(durs.items(), key=lambda kv: -len(kv[1])):
        print(f"  {statistics.median(v):8.2f}  n={len(v):5d}  {k}")
    print("gaps between consecutive kernels (us, < 50 us only): median / p10 / n")
    for (a, b), v in sorted(gaps.items(), key=lambda kv: -len(kv[1]))[:12]:
        v = sorted(v)
        print(f"  {statistics.median(v):6.2f} {v[len(v) // 10]:6.2f} n={len(v):5d}  {a}  ->  {b}")


if __name__ == "__main__":
    main(sys.argv)
