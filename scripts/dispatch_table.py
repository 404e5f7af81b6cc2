"""Per-dispatch table of selected kernels from rocprofv3 output dirs (kernel trace, optional PMC).

  python scripts/dispatch_table.py REGEX DIR [DIR ...]

For every dispatch whose kernel name matches REGEX: duration (us, from the kernel trace) and, when
the dir holds a counter_collection.csv of the same run, the counters of that dispatch plus
  MHz        GRBM_GUI_ACTIVE / duration   (GPU busy cycles over the dispatch window = mean clock)
  cyc/wave   4 * SQ_WAVE_CYCLES / SQ_WAVES
Summary line per dir: median duration, median clock, median cycles per wave.
"""
from __future__ import annotations

import collections
import csv
import glob
import re
import statistics
import sys


def main(pat: str, dirs) -> None:
    rx = re.compile(pat)
    for d in dirs:
        kt = glob.glob(d + "/**/*kernel_trace.csv", recursive=True)
        cc = glob.glob(d + "/**/*counter_collection.csv", recursive=True)
        disp = {}
        for f in kt:
            for r in csv.DictReader(open(f)):
                if rx.search(r["Kernel_Name"]):
                    disp[r["Dispatch_Id"]] = (r["Kernel_Name"][:60], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
        ctr = collections.defaultdict(dict)
        for f in cc:
            for r in csv.DictReader(open(f)):
                if rx.search(r["Kernel_Name"]):
                    ctr[r["Dispatch_Id"]][r["Counter_Name"]] = ctr[r["Dispatch_Id"]].get(r["Counter_Name"], 0.0) + \
                        float(r["Counter_Value"])
        print(f"== {d}: {len(disp)} dispatches (trace), {len(ctr)} with counters")
        durs, mhz, cpw = [], [], []
        for k in sorted(set(disp) | set(ctr), key=lambda s: int(s)):
            name, us = disp.get(k, ("?", float("nan")))
            c = ctr.get(k, {})
            line = f"  {k:>6s} {name:60s} {us:9.1f} us"
            if "GRBM_GUI_ACTIVE" in c and us == us:
                f_ = c["GRBM_GUI_ACTIVE"] / us
                mhz.append(f_)
                line += f"  {f_:7.0f} MHz"
            if c.get("SQ_WAVES"):
                w = 4 * c["SQ_WAVE_CYCLES"] / c["SQ_WAVES"]
                cpw.append(w)
                line += f"  {w:9.0f} cyc/wave"
            print(line)
            if us == us:
                durs.append(us)
        med = lambda v: statistics.median(v) if v else float("nan")  # noqa: E731
        print(f"  median: {med(durs):.1f} us, {med(mhz):.0f} MHz, {med(cpw):.0f} cyc/wave")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2:])
