"""A/B of the hand GEMM kernel variants (MI_DFT_GEMM_KERNEL=8w | 2wg, MI_DFT_GEMM_EPI) on the FourCastNet MLP
launches: bit-exactness of the outputs (both variants run the same MFMA sequence per output, so
they must agree exactly) and timing (bench/bench_gemm.py --x3 in a child per variant, since the
variant is read once per process).

Usage: python bench/gemm_variant_ab.py [--rows 518400] [--rounds 3] [--variants 8w+direct,8w,2wg]  (kernel[+direct])
"""
import argparse
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import os, sys, torch
sys.path.insert(0, %(root)r)
import tensorrt_dft_plugins_amd as tdp
tdp.load_plugins()
ops = torch.ops.amd_dft
torch.manual_seed(0)
M = 256 * 90 + 77  # ragged last token tile; > 256 tiles at N = 768 (the persistent grid is active)
C, H = 768, 3072
x = torch.randn(M, C, device="cuda")
w1 = torch.randn(H, C, device="cuda") * 0.02
w2 = torch.randn(C, H, device="cuda") * 0.02
b1 = torch.randn(H, device="cuda") * 0.02
r = torch.randn(M, C, device="cuda")
xs, w1s, w2s = ops.split_bf16(x), ops.split_bf16(w1), ops.split_bf16(w2)
h = ops.linear3(xs, w1s, b1, 1, None, True)
y = ops.linear3(h, w2s, None, 0, r.clone(), False)
y1 = ops.linear3(xs, w1s, b1, 0, None, False)
# the fp32 block's GEMMs (the persistent variants; staged epilogue only): LN-folded fc1, fc2 +
# statistics, fc2 -> split pairs
extra = {}
if os.environ.get("MI_DFT_GEMM_EPI", "staged") != "direct":
    st = ops.ln_stats(x, None, 1e-6)
    c1, c2 = torch.randn(H, device="cuda"), torch.randn(H, device="cuda") * 0.02
    ys, part = ops.linear3_stats(h, w2s, r.clone(), b1[:C])
    extra = {"hl": ops.linear3_ln(xs, w1s, c1, c2, st, 1), "ys": ys, "part": part,
             "yp": ops.linear3(h, w2s, None, 0, r.clone(), True),
             # the bf16 block's forms: LN-folded fc1 + GELU, fc2 + bias + residual
             "hbl": ops.linear_ln(x.bfloat16(), w1.bfloat16(), c1, b1, st, 1),
             "ybr": ops.linear(torch.randn(M, H, device="cuda").bfloat16(), w2.bfloat16(), b1[:C], 0, r.bfloat16())}
xb, w1b, w2b = x.bfloat16(), w1.bfloat16(), w2.bfloat16()
hb = ops.linear(xb, w1b, b1, 1, None)
yb = ops.linear(hb, w2b, None, 0, r.bfloat16())
torch.cuda.synchronize()
out = {"h": h, "y": y, "y1": y1, "hb": hb, "yb": yb, **extra}
torch.save({k: v.cpu() for k, v in out.items()}, sys.argv[1])
print("saved", sys.argv[1], flush=True)
"""


def variant_env(v: str) -> dict:
    """"8w", "8w+direct" (epilogue stored straight from the MFMA layout), "2wg" (an experimental
    build with bench/experimental/gemm2wg.hip linked in)."""
    kern, _, epi = v.partition("+")
    return {"MI_DFT_GEMM_KERNEL": kern, "MI_DFT_GEMM_EPI": epi or "staged"}


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--rows", type=int, default=32 * 16200)
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--variants", default="8w,2wg")
    ap.add_argument("--no-time", action="store_true")
    a = ap.parse_args(argv)
    outdir = os.environ.get("TMPDIR", "/tmp")
    os.makedirs(outdir, exist_ok=True)
    files = {}
    for v in a.variants.split(","):
        env = dict(os.environ, **variant_env(v))
        f = os.path.join(outdir, f"gemm_ab_{v.replace(':', '_').replace('+', '_')}.pt")
        subprocess.run([sys.executable, "-c", CHILD % {"root": ROOT}, f], env=env, check=True, timeout=300)
        files[v] = f
    import torch

    vs = list(files)
    base = torch.load(files[vs[0]], weights_only=True)
    ok = True
    for v in vs[1:]:
        other = torch.load(files[v], weights_only=True)
        for k in base:
            same = torch.equal(base[k], other[k])
            diff = (base[k].float() - other[k].float()).abs().max().item()
            print(f"{vs[0]} vs {v} {k:3s}: bit-identical={same} max|diff|={diff:.3e}", flush=True)
            ok &= same
    if not a.no_time:
        for v in vs:
            print(f"== MI_DFT_GEMM_KERNEL={v}", flush=True)
            env = dict(os.environ, **variant_env(v))
            subprocess.run([sys.executable, os.path.join(ROOT, "bench", "bench_gemm.py"), "--x3", "--rows", str(a.rows),
                            "--rounds", str(a.rounds)], env=env, check=True, timeout=600)
    return 0 if ok else 1


if __name__ == "__main__":
    sys.exit(main())
