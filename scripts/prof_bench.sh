#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench${PROF_TAG:-} -o bench -- python3 bench.py --steps 3 --warmup 1 --no-fft --extra-steps 0 ${BENCH_ARGS:-} > gpurun_out/prof_bench${PROF_TAG:-}.log 2>&1 || exit $?
python3 scripts/kernel_summary.py gpurun_out/prof_bench${PROF_TAG:-}
