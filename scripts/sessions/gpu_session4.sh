#!/bin/bash
# GPU session 4 (round 3): AFNO v_swap_b32 lead (vectorizer-on build with and without v_swap_b32),
# GPU test tier, fp32 headline with the fc2-fused LayerNorm statistics (A/B against the ln_stats pass),
# and a kernel-time profile of the replayed step.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "gpurun_out/$tag.log" | tail -${TAILN:-12}
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping: $tag ended abnormally ($rc)"; exit $rc; fi
  return $rc
}
TAILN=6 step s4_afno_vec1 200 env MI_DFT_LIB=$PWD/build_diag/vec1/_C.so python -u scripts/diag/afno_race_diag.py
TAILN=6 step s4_afno_vec1x 200 env MI_DFT_LIB=$PWD/build_diag/vec1x/_C.so python -u scripts/diag/afno_race_diag.py
TAILN=6 step s4_afno_vec1_again 200 env MI_DFT_LIB=$PWD/build_diag/vec1/_C.so python -u scripts/diag/afno_race_diag.py
TAILN=6 step s4_afno_vec1x_again 200 env MI_DFT_LIB=$PWD/build_diag/vec1x/_C.so python -u scripts/diag/afno_race_diag.py
TAILN=8 step s4_tests 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests
TAILN=3 step s4_bench 600 python -u bench.py --steps 10 --warmup 3
TAILN=3 step s4_bench_nostats 600 env MI_DFT_FC2_STATS=0 python -u bench.py --steps 10 --warmup 3
TAILN=3 step s4_bench2 600 python -u bench.py --steps 10 --warmup 3
TAILN=40 PROF_TAG=_r3a step s4_prof 700 bash scripts/prof_bench.sh
