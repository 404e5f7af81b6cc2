#!/bin/bash
# Round 4, GPU session 15: FNO block breakdown on the current tree -- per-kernel times (rocprofv3 --stats over
# bench_fno) and the FNO tail's phase clocks (timing-only build variants/bin/fno_stamps).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
export HSA_ENABLE_IPC_MODE_LEGACY=0 TMPDIR=/tmp MI_DFT_BOX_BUILD=0
ROOT=$PWD
step() {
  local tag=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$ROOT/gpurun_out/$tag.log" 2>&1; local rc=$?
  echo "== $tag rc=$rc"; grep -v amdgpu.ids "$ROOT/gpurun_out/$tag.log" | grep -v "warning: failed to meet" | tail -${TAILN:-12}
  if [ $rc -ne 0 ]; then echo "stopping: $tag failed ($rc)"; exit $rc; fi
}
TAILN=30 step r4s15_fno_stamps 120 ./variants/bin/fno_stamps
TAILN=4 step r4s15_fno 200 python -u bench/bench_fno.py --amd-only --rounds 5
TAILN=2 step r4s15_fno_prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fno -o fno -- python3 bench/bench_fno.py --amd-only --rounds 2
python3 scripts/kernel_summary.py gpurun_out/prof_fno | head -12
