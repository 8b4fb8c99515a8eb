cd $GRAFT_REPO_ROOT
ALT=$GRAFT_REPO_ROOT/gpurun_alt
for S in 0 1 2; do
for rep in 1 2; do
  timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/cur  /' || exit 1
  INFLOW_LIB=$ALT/lib_head.so timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/head /' || exit 1
done
done
