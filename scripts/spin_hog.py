"""Occupies a few CUs from a SEPARATE process (own hardware queues): K streams each looping
single-workgroup spin kernels (torch.cuda._sleep) for `seconds`.  Used with
scripts/interference_probe.py --spinners 0 to see whether co-running long-lived kernels (like
RCCL collective blocks) slow the step's kernels.   python scripts/spin_hog.py K seconds"""
import sys
import time

import torch

k, secs = int(sys.argv[1]), float(sys.argv[2])
streams = [torch.cuda.Stream() for _ in range(k)]
torch.cuda.synchronize()
print("hog ready", flush=True)
t0 = time.time()
while time.time() - t0 < secs:
    for s in streams:
        with torch.cuda.stream(s):
            torch.cuda._sleep(20_000_000)
    torch.cuda.synchronize()
print("hog done", flush=True)
