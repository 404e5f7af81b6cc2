#!/bin/bash
# Round 4, GPU session 22: the packed-VALU statistics epilogue (pinned stored words, paired sweeps): its GPU tests, the fc2
# forms in one process, and the bench line.
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
python -u -c "import __graft_entry__ as g; g.build()" > gpurun_out/r4s22_build.log 2>&1 || { echo build failed; tail -5 gpurun_out/r4s22_build.log; exit 1; }
TAILN=4 step r4s22_tests 600 python -u -m pytest tests/test_bf16_stats.py tests/test_gemm.py tests/test_fp32_path.py -x -q -m gpu --timeout 300 --timeout-method thread
TAILN=12 step r4s22_gemm_a 300 python -u bench/bench_gemm.py --rounds 5
TAILN=1 step r4s22_bench 400 python -u bench.py
