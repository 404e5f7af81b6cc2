"""Static check of compiled kernels: can a wave reach an s_barrier with LDS operations still in
flight?  A barrier orders LDS traffic between waves only if every wave's own DS operations have
completed (s_waitcnt lgkmcnt(0)) before it arrives; a DS read still in flight when the barrier
opens can return data another wave writes after the barrier (write-after-read), and a DS write
still in flight can be missed by a reader.

Dataflow over the assembly's control-flow graph (labels, s_cbranch_*, s_branch, fall-through):
state = DS operations issued and not yet retired by an s_waitcnt lgkmcnt(N) (DS ops retire in
order, so lgkmcnt(N) leaves at most N); the merge takes the maximum over incoming paths.  Reports
every s_barrier reachable with pending DS operations.

Usage: python scripts/diag/barrier_lds_check.py <file.s> [kernel-substring]
"""
import re
import sys


def kernels(txt):
    for m in re.finditer(r"\n(_Z\S+):\s*(?:;.*)?\n", txt):
        name = m.group(1)
        st = m.end()
        en = txt.find(".Lfunc_end", st)
        if en < 0:
            continue
        yield name, txt[st:en]


def parse(body):
    ins = []  # (kind, text)
    for raw in body.split("\n"):
        s = raw.split(";")[0].strip()
        if not s:
            continue
        if re.match(r"^\.LBB\d+_\d+:", s):
            ins.append(("label", s[:-1]))
        elif s.startswith("."):
            continue
        else:
            ins.append(("op", s))
    return ins


def analyse(ins):
    labels = {t: i for i, (k, t) in enumerate(ins) if k == "label"}
    n = len(ins)
    succ = [[] for _ in range(n)]
    for i, (k, t) in enumerate(ins):
        op = t.split()[0] if k == "op" else ""
        if op == "s_branch":
            succ[i].append(labels[t.split()[1]])
        elif op.startswith("s_cbranch"):
            succ[i].append(labels[t.split()[1]])
            if i + 1 < n:
                succ[i].append(i + 1)
        elif op in ("s_endpgm", "s_setpc_b64"):
            pass
        elif i + 1 < n:
            succ[i].append(i + 1)
    state = [-1] * n
    state[0] = 0
    work = [0]
    findings = {}
    while work:
        i = work.pop()
        p = state[i]
        k, t = ins[i]
        if k == "op":
            op = t.split()[0]
            if op.startswith("ds_"):
                p += 1
            elif op == "s_waitcnt":
                m = re.search(r"lgkmcnt\((\d+)\)", t)
                if m:
                    p = min(p, int(m.group(1)))
            elif op == "s_barrier" and p > 0:
                findings[i] = max(findings.get(i, 0), p)
        for j in succ[i]:
            if p > state[j]:
                state[j] = p
                work.append(j)
    return findings


def main():
    txt = open(sys.argv[1]).read()
    sub = sys.argv[2] if len(sys.argv) > 2 else ""
    bad = 0
    for name, body in kernels(txt):
        if sub not in name:
            continue
        ins = parse(body)
        f = analyse(ins)
        nbar = sum(1 for k, t in ins if k == "op" and t.startswith("s_barrier"))
        if f:
            bad += 1
            print(f"{name[:110]}: {len(f)} of {nbar} barriers reachable with DS ops in flight (max {max(f.values())})")
    print(f"{bad} kernel(s) with barrier-crossing LDS operations")
    return 1 if bad else 0


if __name__ == "__main__":
    sys.exit(main())
