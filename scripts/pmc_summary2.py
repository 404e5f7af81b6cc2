"""Per-kernel PMC averages + derived per-wave numbers from rocprofv3 counter CSVs."""
import collections
import csv
import glob
import re
import sys

sys.path.insert(0, __file__.rsplit("/", 1)[0])
from kernel_summary import short  # noqa: E402

agg = collections.defaultdict(lambda: collections.defaultdict(list))
dur = collections.defaultdict(list)
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    if not any(s in k for s in ("fft_", "afno", "ln_", "patch", "Cijk", "fno", "dftw", "gemm")):
        continue
    a = {c: sum(x) / len(x) for c, x in v.items()}
    w = a.get("SQ_WAVES", 0) or 1
    out = {c: round(x) for c, x in sorted(a.items())}
    der = {
        "cyc/wave": round(4 * a.get("SQ_WAVE_CYCLES", 0) / w),
        "active%": round(100 * a.get("SQ_ACTIVE_INST_ANY", 0) / max(a.get("SQ_WAVE_CYCLES", 1), 1)),
        "wait%": round(100 * a.get("SQ_WAIT_ANY", 0) / max(a.get("SQ_WAVE_CYCLES", 1), 1)),
        "valu/wave": round(a.get("SQ_INSTS_VALU", 0) / w),
        "mfma/wave": round(a.get("SQ_INSTS_MFMA", 0) / w),
        "lds/wave": round(a.get("SQ_INSTS_LDS", 0) / w),
        "vmem_rd/wave": round(a.get("SQ_INSTS_VMEM_RD", 0) / w),
        "vmem_wr/wave": round(a.get("SQ_INSTS_VMEM_WR", 0) / w),
        "bank_conf/lds": round(a.get("SQ_LDS_BANK_CONFLICT", 0) / max(a.get("SQ_INSTS_LDS", 1), 1), 2),
        "L2hit%": round(100 * a.get("TCC_HIT_sum", 0) / max(a.get("TCC_HIT_sum", 0) + a.get("TCC_MISS_sum", 0), 1)),
    }
    print(k)
    print("   derived:", der)
    print("   raw:", out)
