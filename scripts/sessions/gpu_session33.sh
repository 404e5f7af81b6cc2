#!/bin/bash
# GPU session 33 (round 3): FNO block (config 3) column-FFT tile A/B via MI_DFT_FIXED_CFG (the forward H transform and
# the mixing-gather inverse both run the 720-point column kernels): default heuristic vs forced (TP, T).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
for rep in 1 2; do
  for cfg in "" "90,2" "90,4" "90,8" "45,4" "45,8"; do
    MI_DFT_FIXED_CFG="$cfg" timeout -k 10 300 python -u bench/bench_fno.py --amd-only --rounds 8 > gpurun_out/s33_fno_${cfg/,/_}_$rep.log 2>&1 || { echo "fno $cfg failed"; exit 1; }
    echo "cfg=${cfg:-default} rep $rep: $(grep '^bf16' gpurun_out/s33_fno_${cfg/,/_}_$rep.log | python3 -c 'import sys,json; l=sys.stdin.read(); j=json.loads(l[l.index("{"):]); print("bf16 graph %.2f us rel %.2e" % (j["amd_graph"]["median_us"], j["rel_l2_vs_fp32_torch"]))')"
  done
done
