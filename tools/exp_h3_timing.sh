cd $GRAFT_REPO_ROOT
for S in 0 1 2; do
  timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 2 --reps 5 2>&1 | grep -a "us/term" || exit 1
  INFLOW_LIB=gpurun_alt/lib_stamps.so timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 2 --reps 1 2>&1 | grep -a "timing" || exit 1
done
