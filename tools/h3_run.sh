cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread -s -k "split_bf16_error or (fused_313 and 2)" > gpurun_out/h3_tests.log 2>&1 || { echo TESTS_FAILED; tail -30 gpurun_out/h3_tests.log; exit 1; }
for S in 0 1 2; do for M in 1 2; do
  timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma $M --reps 5 2>&1 | grep -a "us/term" | sed "s/^/S$S M$M /" || exit 1
  INFLOW_LIB=gpurun_alt/lib_stamps.so timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma $M --reps 1 2>&1 | grep -a "mode2" | sed "s/^/S$S M$M /" || exit 1
done; done
