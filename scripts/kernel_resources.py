"""Per-kernel register / LDS / scratch usage of a built library (from the code objects' AMDGPU metadata notes).

  python scripts/kernel_resources.py [lib] [name-substring ...]
"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "diag"))
from scan_so import LLVM, code_objects  # noqa: E402


def resources(so, pats=()):
    rows = []
    with tempfile.TemporaryDirectory() as tmp:
        for co in code_objects(so, tmp):
            notes = subprocess.run([os.path.join(LLVM, "llvm-readelf"), "--notes", co], check=True, capture_output=True,
                                   text=True).stdout
            for blk in re.split(r"\n  - \.agpr_count", notes)[1:]:
                def field(k):
                    m = re.search(r"\n    \." + k + r":\s+(\S+)", blk)
                    return m.group(1) if m else "?"
                name = field("name")
                if pats and not any(p in name for p in pats):
                    continue
                agpr = re.match(r":\s+(\d+)", blk)
                rows.append((name, field("vgpr_count"), agpr.group(1) if agpr else "?", field("sgpr_count"),
                             field("group_segment_fixed_size"), field("private_segment_fixed_size")))
    return rows


def main():
    so = sys.argv[1] if len(sys.argv) > 1 else os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                            "tensorrt_dft_plugins_amd", "_C.so")
    for name, v, a, s, lds, scr in resources(so, sys.argv[2:]):
        print(f"vgpr {v:>4} agpr {a:>4} sgpr {s:>4} lds {lds:>6} scratch {scr:>4}  {name[:150]}")


if __name__ == "__main__":
    main()
