"""Hand MFMA GEMM vs hipBLASLt on the FourCastNet embed (1280 -> 768) and head (768 -> 1280)
shapes, M = 32 * 16200 tokens, bf16; plus the patchify / un-patchify / pos-embed add they
would absorb."""
import torch
import torch.nn.functional as F

from bench_fft import time_graph
import tensorrt_dft_plugins_amd as tdp

tdp.load_plugins()
M = 32 * 16200
ops = torch.ops.amd_dft
r = {}
for name, K, N in (("embed", 1280, 768), ("head", 768, 1280)):
    x = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    w = (torch.randn(N, K, device="cuda") * 0.02).to(torch.bfloat16)
    b = torch.randn(N, device="cuda") * 0.02
    r[name + "_amd"] = time_graph(lambda: ops.linear(x, w, b, 0, None), 5)
    r[name + "_blas"] = time_graph(lambda: F.linear(x, w, b.bfloat16()), 5)
img = torch.randn(32, 20, 720, 1440, device="cuda").to(torch.bfloat16)
t = ops.patchify(img, 8)
pos = torch.randn(1, 16200, 768, device="cuda").to(torch.bfloat16)
e = torch.randn(32, 16200, 768, device="cuda").to(torch.bfloat16)
r["patchify"] = time_graph(lambda: ops.patchify(img, 8), 5)
r["unpatchify"] = time_graph(lambda: ops.unpatchify(t, 20, 90, 180, 8), 5)
r["pos_add"] = time_graph(lambda: e + pos, 5)
print({k: round(v, 1) for k, v in r.items()})
wmat = (torch.randn(768, 1280, device="cuda") * 0.02).to(torch.bfloat16)
be = torch.randn(768, device="cuda") * 0.02
pos2 = pos.reshape(16200, 768)
r2 = {"embed_fused_amd": time_graph(lambda: ops.patch_linear(img, wmat, be, pos2, 8), 5)}
wh = (torch.randn(1280, 768, device="cuda") * 0.02).to(torch.bfloat16)
bh = torch.randn(1280, device="cuda") * 0.02
r2["head_fused_amd"] = time_graph(lambda: ops.linear_unpatch(e.reshape(-1, 768), wh, bh, 20, 90, 180, 8), 5)
print({k: round(v, 1) for k, v in r2.items()})
