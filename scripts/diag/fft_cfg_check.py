import os, sys, torch
sys.path.insert(0, os.getcwd())
import tensorrt_dft_plugins_amd as tdp
tdp.load_plugins()
x = torch.randn(1, 720, 1440, device="cuda")
ref = torch.view_as_real(torch.fft.rfft2(x.double().cpu()))
for cfg in ("90,4", "90,3", "45,6", "90,2"):
    os.environ["MI_DFT_FIXED_CFG"] = cfg
    y = tdp.contrib_rfft(x, signal_ndim=2).double().cpu()
    z = tdp.contrib_irfft(tdp.contrib_rfft(x, signal_ndim=2), signal_ndim=2)
    print(cfg, "rfft2 err", ((y - ref).norm() / ref.norm()).item(), "roundtrip err", ((z - x).norm() / x.norm()).item(), flush=True)
