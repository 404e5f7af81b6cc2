"""Instruction histogram of one kernel in a hipcc -S listing:  isa_hist.py file.s NAME_SUBSTRING [N]"""
import collections
import re
import sys

s = open(sys.argv[1]).read()
names = [n for n in re.findall(r"^(_Z[^:\s]+):", s, re.M) if sys.argv[2] in n]
name = names[0]
body = s[s.index(name + ":"):]
body = body[:body.index(".Lfunc_end")]
ins = [l.split()[0] for l in body.splitlines() if l.startswith("\t") and not l.strip().startswith((".", ";"))]
c = collections.Counter(ins)
print(name[:120], "total", len(ins))
for k, v in c.most_common(int(sys.argv[3]) if len(sys.argv) > 3 else 40):
    print(f"{v:6d} {k}")
