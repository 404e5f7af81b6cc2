"""Static scan of gfx950 assembly for the AFNO -O3 corruption pattern (profiles/afno_o3_bisect_r3.txt):
a packed-FP32 VALU op (v_pk_mul/fma/add_f32) whose op_sel takes the HIGH half of a source VGPR pair into the low
lane, where that pair was last written by an LDS load (ds_read*), not by a VALU op.

  hipcc -S --cuda-device-only -O3 --offload-arch=gfx950 ... -o k.s && python scripts/diag/opsel_lds_check.py k.s

Prints, per kernel, the number of such reads (straight-line program order; the last writer of a register is the
textually previous instruction that wrote it, which is exact inside the unrolled pass bodies this targets).
"""
import re
import sys

REG = re.compile(r"v\[(\d+):(\d+)\]|v(\d+)\b")
MOD = r"\b[a-z_]+\d*:\[[^\]]*\]|\b[a-z_]+\d*:-?\w+"


def regs(tok):
    m = REG.fullmatch(tok.strip())
    if not m:
        return []
    if m.group(1):
        return list(range(int(m.group(1)), int(m.group(2)) + 1))
    return [int(m.group(3))]


def scan(path):
    out = {}
    fn = None
    writer = {}
    for line in open(path):
        s = line.strip()
        if re.match(r"^[_A-Za-z][\w.$]*:\s*(;.*)?$", s) and not s.startswith("."):
            fn = s.split(":")[0]
            writer = {}
            out.setdefault(fn, [0, 0])
            continue
        if fn is None or not s or s.startswith((";", ".", "s_")):
            continue
        s = s.split(";")[0].strip()
        op, _, rest = s.partition(" ")
        mods = " ".join(re.findall(MOD, rest))
        rest = re.sub(MOD, "", rest)
        args = [a.strip().split()[0] for a in rest.split(",") if a.strip()]
        if op.startswith("v_pk_") and op.endswith("_f32"):
            m = re.search(r"op_sel:\[([01,]+)\]", mods)
            sel = [int(x) for x in m.group(1).split(",")] if m else []
            srcs = args[1:]
            for i, b in enumerate(sel):
                if b and i < len(srcs):
                    r = regs(srcs[i])
                    if r:
                        out[fn][1] += 1
                        if writer.get(r[-1]) == "lds":
                            out[fn][0] += 1
        if op.startswith(("ds_read", "ds_load")):
            for r in regs(args[0]) if args else []:
                writer[r] = "lds"
        elif op.startswith(("v_", "global_load", "buffer_load", "flat_load")) and args:
            for r in regs(args[0]):
                writer[r] = "valu" if op.startswith("v_") else "vmem"
    return out


if __name__ == "__main__":
    for p in sys.argv[1:]:
        for fn, (lds, tot) in scan(p).items():
            if tot:
                print(f"{p}: {fn[:90]}: op_sel high-half packed reads {tot}, of LDS-loaded pairs {lds}")
