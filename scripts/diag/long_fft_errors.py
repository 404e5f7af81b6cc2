"""Measured rel-L2 errors of the long-length FFT compositions (four-step / Bluestein) against
fp64 torch.fft, next to the error model used by tests/test_dft_gpu.py."""
import math, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import torch
import tensorrt_dft_plugins_amd as tdp
tdp.load_plugins()
sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))), "tests"))
from test_dft_gpu import long_fft_tol  # noqa: E402
def rel(a, b):
    a, b = torch.view_as_real(a.cpu().to(torch.complex128)) if a.is_complex() else a.double().cpu(), \
           torch.view_as_real(b.to(torch.complex128)) if b.is_complex() else b.double()
    return ((a - b).norm() / b.norm()).item()
for n in (6553, 8192, 8198, 10007, 20000, 65536, 100003):
    torch.manual_seed(n % 97)
    x = torch.randn(2, n, device="cuda")
    e1 = rel(tdp.rfft(x), torch.fft.rfft(x.double().cpu()))
    e2 = rel(tdp.irfft(tdp.rfft(x), n=n), x.cpu())
    z = torch.randn(2, n, dtype=torch.complex64, device="cuda")
    e3 = rel(tdp.fft(z), torch.fft.fft(z.cpu().to(torch.complex128)))
    e4 = rel(tdp.ifft(z), torch.fft.ifft(z.cpu().to(torch.complex128)))
    print(f"n={n:6d} rfft {e1:.2e} irfft(rfft) {e2:.2e} fft {e3:.2e} ifft {e4:.2e} | model tol {long_fft_tol(n):.2e} "
          f"(max/tol {max(e1, e2, e3, e4) / long_fft_tol(n):.2f})", flush=True)
