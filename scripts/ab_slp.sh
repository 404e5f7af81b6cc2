#!/bin/bash
# A/B: default build vs -fno-slp-vectorize on every HIP file, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python bench/bench_afno_spec.py || return 1
  timeout -k 10 200 python bench/bench_fft.py --rounds 3 --iters 20 | python3 -c "import json,sys; d=json.load(sys.stdin); print({k: round(v['graph']['median_us'],2) for k,v in d.items() if isinstance(v, dict) and 'graph' in v})" || return 1
  timeout -k 10 200 python bench/bench_afno_w.py --cfgs auto || return 1
  timeout -k 10 200 python bench/bench_kernels_fno.py 2>&1 | grep -E "B1 .*m32 gelu1|dftw_r2c bf16 B1 C20 m32|fno_mix B1" || return 1
}
echo "=== default"; run > gpurun_out/ab_default.log 2>&1; cat gpurun_out/ab_default.log | grep -v amdgpu.ids
MI_DFT_HIPCC_EXTRA=-fno-slp-vectorize timeout -k 10 400 python -m tensorrt_dft_plugins_amd._build --force -j 16 > gpurun_out/ab_build.log 2>&1 || { tail gpurun_out/ab_build.log; exit 1; }
echo "=== no-slp"; run > gpurun_out/ab_noslp.log 2>&1; cat gpurun_out/ab_noslp.log | grep -v amdgpu.ids
