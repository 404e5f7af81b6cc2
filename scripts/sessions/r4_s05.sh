#!/bin/bash
# Round 4, GPU sessions 5-6: the fc2 statistics / split-pair epilogue rewrites (phase clocks, headline step), the full GPU
# tier, and the non-temporal FFT store A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp
ROOT=$PWD
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}


TAILN=30 step r4s06_gemm_stamps 200 ./variants/bin/gemm_stamps
TAILN=1 step r4s06_bench 400 python -u bench.py --no-fft --extra-steps 0 --steps 10 --warmup 3
TAILN=6 step r4s05_gpu_tier 900 python -u -m pytest tests -q -m gpu --timeout 300 --timeout-method thread -p no:cacheprovider
# rfft2 / irfft2: non-temporal complex stores (variants/ntstore, -DAMD_DFT_FFT_NT_STORE=1) vs default, ABAB, then a kernel
# trace of the graph replays (the gap between the row and the column kernel of one call)
for r in 1 2; do
  TAILN=0 step r4s05_fft_def_$r 200 python -u bench/bench_fft.py --rounds 8 --json gpurun_out/r4s05_fft_def_$r.json
  python3 -c "import json;d=json.load(open('gpurun_out/r4s05_fft_def_$r.json'));print('default', {k:round(d[k]['graph']['median_us'],2) for k in ('amd_rfft2','amd_irfft2')})"
  MI_DFT_LIB=$ROOT/variants/ntstore/_C.so TAILN=0 step r4s05_fft_nt_$r 200 python -u bench/bench_fft.py --rounds 8 --json gpurun_out/r4s05_fft_nt_$r.json
  python3 -c "import json;d=json.load(open('gpurun_out/r4s05_fft_nt_$r.json'));print('ntstore', {k:round(d[k]['graph']['median_us'],2) for k in ('amd_rfft2','amd_irfft2')})"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/fft_trace_r4s05 -o fft -- python3 bench/bench_fft.py --rounds 3 > gpurun_out/r4s05_fft_trace.log 2>&1; echo "fft trace rc=$?"
