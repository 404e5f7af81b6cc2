#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fft3 -o fft -- python3 bench/bench_fft.py --rounds 1 --iters 20 > gpurun_out/prof_fft3.log 2>&1 || exit $?
for f in $(find gpurun_out/prof_fft3 -name "*kernel_stats.csv"); do cut -d, -f1-4 $f | cut -c1-220; done
