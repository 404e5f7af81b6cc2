#!/bin/bash
# quick iteration: gpu tests (subset via $TESTS), bench, kernel profile of the bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp HSA_ENABLE_IPC_MODE_LEGACY=0
TAG=${1:-iter}
timeout -k 10 900 python -m pytest ${TESTS:-tests} -m gpu -q -rf > gpurun_out/${TAG}_tests.log 2>&1; rc=$?
echo "tests rc=$rc"; tail -12 gpurun_out/${TAG}_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 900 python bench.py --steps 8 --warmup 2 --json-out gpurun_out/${TAG}_bench.json > gpurun_out/${TAG}_bench.log 2>&1; rc=$?
echo "bench rc=$rc"; tail -3 gpurun_out/${TAG}_bench.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_prof -o bench -- python3 bench.py --steps 3 --warmup 1 --no-fft > gpurun_out/${TAG}_prof.log 2>&1 || exit $?
python3 scripts/kernel_summary.py gpurun_out/${TAG}_prof
