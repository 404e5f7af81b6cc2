"""Average rocprofv3 PMC counters per kernel (short names) from one or more -d dirs, plus a
derived table (LDS bank conflicts per LDS instruction, LDS wait share, HBM-side bytes, L2 hit)."""
import collections
import csv
import glob
import re
import sys


def short(name: str) -> str:
    m = re.search(r"fft_fixed_kernel<\(amd_dft::Kind\)(\d), (\w+), (\d+), (\d+)", name)
    if m:
        return f"fixed K{m.group(1)} cols={m.group(2)} TP={m.group(3)} T={m.group(4)}"
    m = re.search(r"fft_pass_kernel<\(amd_dft::Kind\)(\d)", name)
    if m:
        return f"generic K{m.group(1)}"
    return name[:60]


agg = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
keep = ("amd", "fixed", "generic", "fft_rtc", "transpose")
rows = []
for k, v in sorted(agg.items()):
    if not any(s in k for s in keep):
        continue
    m = {c: sum(x) / len(x) for c, x in v.items()}
    print(k)
    print("   ", {c: round(x) for c, x in sorted(m.items())})
    g = m.get
    lds = g("SQ_INSTS_LDS") or 0
    rows.append((k, g("SQ_WAVES"), (g("SQ_WAVE_CYCLES") or 0) / max(g("SQ_WAVES") or 1, 1),
                 (g("SQ_LDS_BANK_CONFLICT") or 0) / max(lds, 1), 100.0 * (g("SQ_WAIT_INST_LDS") or 0) / max(g("SQ_WAVE_CYCLES") or 1, 1),
                 (g("FETCH_SIZE") or 0), (g("WRITE_SIZE") or 0),  # rocprofv3 derives both in KB
                 100.0 * (g("TCC_HIT_sum") or 0) / max((g("TCC_HIT_sum") or 0) + (g("TCC_MISS_sum") or 0), 1)))
print()
print(f"{'kernel':40s} {'waves':>7s} {'cyc/wave':>9s} {'bankconf/lds':>12s} {'ldswait%':>8s} {'fetch KB':>9s} {'write KB':>9s} {'L2hit%':>7s}")
for k, w, cpw, bc, lw, fe, wr, hit in rows:
    print(f"{k:40s} {w or 0:7.0f} {cpw:9.0f} {bc:12.2f} {lw:8.1f} {fe:9.0f} {wr:9.0f} {hit:7.1f}")
