set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
bash $S r6d_tests 900 python -u -m pytest tests/test_dft_gpu.py tests/test_fno.py -m gpu -x -q --timeout 300 --timeout-method thread || exit $?
for i in 1 2; do
  bash $S r6d_fft_new_$i 200 python bench/bench_fft.py --rounds 10 || exit $?
  MI_DFT_LIB=ab/colpw0_C.so bash $S r6d_fft_old_$i 200 python bench/bench_fft.py --rounds 10 || exit $?
  bash $S r6d_fno_new_$i 200 python bench/bench_fno.py --amd-only --rounds 10 || exit $?
  MI_DFT_LIB=ab/colpw0_C.so bash $S r6d_fno_old_$i 200 python bench/bench_fno.py --amd-only --rounds 10 || exit $?
done
B="SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS SQ_INSTS_SMEM"
bash $S r6d_pmc_new 120 timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $B -d gpurun_out/r6d_pmc_new -o B -- python3 bench/bench_fft.py --rounds 1 --iters 5 || exit $?
MI_DFT_LIB=ab/colpw0_C.so bash $S r6d_pmc_old 120 timeout -s KILL 90 rocprofv3 --kernel-trace --output-format csv --pmc $B -d gpurun_out/r6d_pmc_old -o B -- python3 bench/bench_fft.py --rounds 1 --iters 5 || exit $?
python3 scripts/pmc_table.py gpurun_out/r6d_pmc_new > gpurun_out/r6d_pmc_new.txt
python3 scripts/pmc_table.py gpurun_out/r6d_pmc_old > gpurun_out/r6d_pmc_old.txt
find gpurun_out -name "*.csv" -size +5M -delete
