set -u
S=scripts/gpu_step.sh
bash $S r5i_tests 600 python -u -m pytest tests/test_fp32_path.py tests/test_gemm.py -m gpu -x -q -s --timeout 300 --timeout-method thread || exit $?
ab() { bash $S r5i_bench_$1_$2 600 python -c "import sys, runpy; import tensorrt_dft_plugins_amd.ops.spectral as S; S.F32_RESIDUAL = '$1'; sys.argv = ['bench.py', '--extra-steps', '0']; runpy.run_path('bench.py', run_name='__main__')"; }
ab fp32 1 && ab pairs 1 && ab lo2 1 && ab fp32 2 && ab pairs 2 && ab lo2 2 || exit $?
