set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_fno_r6o -o fno -- python3 bench/fno_probe.py > gpurun_out/r6o_prof.log 2>&1 || exit $?
python3 scripts/kernel_summary.py gpurun_out/prof_fno_r6o > gpurun_out/r6o_kernels.txt 2>&1 || exit $?
find gpurun_out -name "*.csv" -size +5M -delete
cat gpurun_out/r6o_kernels.txt | head -20
