#!/bin/bash
# Samples GPU clocks / power (rocm-smi, read-only) while bench.py runs a long timed loop.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --steps 400 --warmup 3 --no-fft > gpurun_out/clock_bench.log 2>&1 &
BP=$!
for i in $(seq 1 90); do
  echo "t=$i $(date +%s.%N) $(grep -c captured gpurun_out/clock_bench.log)" >> gpurun_out/clock_samples.txt
  timeout -k 5 10 rocm-smi --showclocks --showpower --showtemp >> gpurun_out/clock_samples.txt 2>&1 || true
  sleep 0.5
done
wait $BP; rc=$?
grep metric gpurun_out/clock_bench.log
exit $rc
