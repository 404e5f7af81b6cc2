#!/bin/bash
# rocprofv3 kernel trace of the rfft2/irfft2 benchmark; then a tiling sweep.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python bench/bench_fft.py --rounds 3 --json gpurun_out/fft_bench.json > gpurun_out/fft_bench.log 2>&1 || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fft -o fft -- python3 bench/bench_fft.py --rounds 1 --iters 20 > gpurun_out/prof_fft.log 2>&1 || exit $?
find gpurun_out/prof_fft -name "*kernel_stats.csv" | head -3
for f in $(find gpurun_out/prof_fft -name "*kernel_stats.csv"); do cat $f | cut -c1-250; done
timeout -k 10 300 python bench/tune_fft.py --op rfft2 > gpurun_out/tune_rfft2.log 2>&1 || exit $?
timeout -k 10 300 python bench/tune_fft.py --op irfft2 > gpurun_out/tune_irfft2.log 2>&1 || exit $?
cat gpurun_out/fft_bench.log | python3 -c "import json,sys; d=json.load(sys.stdin); print({k:v['graph']['median_us'] for k,v in d.items() if isinstance(v,dict)})"
cat gpurun_out/tune_rfft2.log gpurun_out/tune_irfft2.log
