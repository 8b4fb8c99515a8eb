cd $GRAFT_REPO_ROOT
ALT=$GRAFT_REPO_ROOT/gpurun_alt
for S in 0 1 2; do
for rep in 1 2; do
  timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/cur  /' || exit 1
  for L in nt xcd both; do
  INFLOW_LIB=$ALT/lib_$L.so timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed "s/^/$L /" || exit 1
  done
done
done
INFLOW_LIB=$ALT/lib_both.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q -k "fused_313 or golden" --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; tail -1 gpurun_out/t.log
