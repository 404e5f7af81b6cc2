#!/bin/bash
# A/B of the persistent GEMM grid and its start stagger (bench/bench_gemm.py --x3 per setting).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in ${GEMM_CFGS:-"MI_DFT_GEMM_PERSIST=0" "MI_DFT_GEMM_PERSIST=1"}; do
  echo "== $cfg"
  env $cfg timeout -k 10 300 python3 -u bench/bench_gemm.py --x3 --rounds 3 2>&1 | grep -v amdgpu.ids | tail -5 || exit 1
done
