set -u
S=scripts/gpu_step.sh
export TMPDIR=/tmp
A="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE"
for m in step captured random random1 gemmgap; do
  bash $S r6c_kt_$m 240 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r6c_kt_$m -o run -- python bench/afno_gap.py --mode $m || exit $?
  bash $S r6c_pmc_$m 240 timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv --pmc $A -d gpurun_out/r6c_pmc_$m -o run -- python bench/afno_gap.py --mode $m --replays 1 || exit $?
done
for m in step captured random random1 gemmgap; do
  python scripts/dispatch_table.py 'afno_spectral|gemm_bf16' gpurun_out/r6c_kt_$m gpurun_out/r6c_pmc_$m > gpurun_out/r6c_table_$m.txt
done
find gpurun_out -name "*.csv" -size +5M -delete
