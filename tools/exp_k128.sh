# 128-pixel K-chunked VJP: parity tests, then per-scale series timing against the 64-pixel kernel
#   bash tools/exp_k128.sh
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread -k "k128 or (fused_313 and 16 and 2-)" > gpurun_out/k128_tests.log 2>&1 || { tail -30 gpurun_out/k128_tests.log; exit 1; }
tail -2 gpurun_out/k128_tests.log
for S in 0 1; do
  for rep in 1 2; do
    timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 2 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/k128 /' || exit 1
    INFLOW_FUSED_K128=0 timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 2 --reps 5 2>&1 | grep -a "us/term" | sed "s/^/k64  /" || exit 1
  done
  INFLOW_LIB=gpurun_alt/lib_stamps.so timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 2 --reps 1 2>&1 | grep -a "mode2" || exit 1
done
