# round check, then the 128-pixel parity subset with chunk 1's exact-scale path forced (INFLOW_FUSED_DBG=16)
cd $GRAFT_REPO_ROOT
bash tools/round_check.sh ${1:-cur} || exit 1
INFLOW_FUSED_DBG=16 timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "k128 or headline" > gpurun_out/gpu_tests_forced_exact_${1:-cur}.log 2>&1; tail -2 gpurun_out/gpu_tests_forced_exact_${1:-cur}.log
