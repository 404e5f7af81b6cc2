"""Average rocprofv3 PMC counters per kernel (short names) from one or more -d dirs."""
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
for k, v in sorted(agg.items()):
    if "amd" not in k and "fixed" not in k and "generic" not in k and "fft_rtc" not in k and "transpose" not in k:
        continue
    print(k)
    print("   ", {c: round(sum(x) / len(x)) for c, x in sorted(v.items())})
