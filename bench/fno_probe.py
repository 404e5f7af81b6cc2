"""Print bench.py's FNO probes (FNO layer and SpectralConv2d alone, bf16 720x1440) as one JSON line,
labelled with the tuning knobs in the environment (tuning-build sweeps: MI_DFT_FNO_UPW / MI_DFT_FNO_WGS)."""
import importlib.util
import json
import os
import sys

root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, root)
spec = importlib.util.spec_from_file_location("benchmain", os.path.join(root, "bench.py"))
bm = importlib.util.module_from_spec(spec)
spec.loader.exec_module(bm)
bm.tdp.load_plugins()
knobs = {k: os.environ[k] for k in ("MI_DFT_LIB", "MI_DFT_FNO_UPW", "MI_DFT_FNO_WGS", "MI_DFT_FIXED_CFG") if k in os.environ}
print(json.dumps({**knobs, **bm.time_fno_block_us()}), flush=True)
