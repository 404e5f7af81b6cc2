"""Per-kernel PMC table from rocprofv3 ``--pmc`` runs (one ``-d`` dir per counter pass).

  python scripts/pmc_table.py DIR [DIR ...]

Counters are averaged over the calls of each kernel (grouped by the demangled name with the
argument list dropped).  Derived columns:
  cyc/wave     SQ_WAVE_CYCLES / SQ_WAVES (quad-cycles x4 -> shader cycles)
  act% wait%   SQ_ACTIVE_INST_ANY / SQ_WAIT_INST_ANY share of wave cycles
  mfma%        SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x CUs)   (MFMA pipe busy, chip-wide)
  valu/w mfma/w lds/w   instructions per wave (SQ_INSTS_VALU includes MFMA)
  bank/lds     SQ_LDS_BANK_CONFLICT per SQ_INSTS_LDS
  ldsw%        SQ_WAIT_INST_LDS share of wave cycles
  fetch/write  FETCH_SIZE / WRITE_SIZE in MB (rocprofv3 derives them in KB; gfx950 FETCH_SIZE
               under-reads wide streams, /opt/skills/guides/MI355X_MICROARCH.md)
  L2hit%       TCC_HIT / (TCC_HIT + TCC_MISS)
"""
from __future__ import annotations

import collections
import csv
import glob
import re
import sys

CUS = 256


def short(name: str) -> str:
    n = re.sub(r"^void ", "", name)
    for junk in ("amd_dft::", "(anonymous namespace)::", "fixed_detail::", "at::native::"):
        n = n.replace(junk, "")
    n = re.sub(r"\(Kind\)", "K", n)
    depth, cut = 0, len(n)
    for i, ch in enumerate(n):  # drop the argument list: the first '(' outside template brackets
        if ch == "<":
            depth += 1
        elif ch == ">":
            depth -= 1
        elif ch == "(" and depth == 0:
            cut = i
            break
    n = n[:cut]
    n = re.sub(r"\btrue\b", "T", n)
    n = re.sub(r"\bfalse\b", "F", n)
    n = n.replace("AfnoShape", "S").replace(", ", ",")
    return n[:70]


def load(dirs):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in dirs:
        for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
            for r in csv.DictReader(open(f)):
                agg[short(r["Kernel_Name"])][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return agg


def main(dirs) -> None:
    agg = load(dirs)
    hdr = (f"{'kernel':70s} {'waves':>7s} {'cyc/wave':>9s} {'act%':>5s} {'wait%':>5s} {'mfma%':>5s} {'valu/w':>7s} "
           f"{'mfma/w':>7s} {'lds/w':>6s} {'bank/lds':>8s} {'ldsw%':>5s} {'fetchMB':>8s} {'writeMB':>8s} {'L2hit%':>6s}")
    print(hdr)
    for k, v in sorted(agg.items()):
        m = {c: sum(x) / len(x) for c, x in v.items()}
        g = lambda c: m.get(c, 0.0)  # noqa: E731
        waves = max(g("SQ_WAVES"), 1.0)
        cyc = g("SQ_WAVE_CYCLES")
        mfma_busy = g("SQ_VALU_MFMA_BUSY_CYCLES")
        gui = g("GRBM_GUI_ACTIVE")
        row = (f"{k:70s} {g('SQ_WAVES'):7.0f} {4 * cyc / waves:9.0f} "
               f"{100 * g('SQ_ACTIVE_INST_ANY') / max(cyc, 1):5.0f} {100 * g('SQ_WAIT_INST_ANY') / max(cyc, 1):5.0f} "
               f"{100 * mfma_busy / max(gui * CUS, 1):5.1f} {g('SQ_INSTS_VALU') / waves:7.0f} "
               f"{g('SQ_INSTS_MFMA') / waves:7.0f} {g('SQ_INSTS_LDS') / waves:6.0f} "
               f"{g('SQ_LDS_BANK_CONFLICT') / max(g('SQ_INSTS_LDS'), 1):8.3f} "
               f"{100 * g('SQ_WAIT_INST_LDS') / max(cyc, 1):5.1f} {g('FETCH_SIZE') / 1024:8.1f} "
               f"{g('WRITE_SIZE') / 1024:8.1f} "
               f"{100 * g('TCC_HIT_sum') / max(g('TCC_HIT_sum') + g('TCC_MISS_sum'), 1):6.1f}")
        print(row)


if __name__ == "__main__":
    main(sys.argv[1:])
