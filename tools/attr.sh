cd $GRAFT_REPO_ROOT
ALT=$GRAFT_REPO_ROOT/gpurun_alt
for S in 0 1; do
  INFLOW_FUSED_TIMING=1 timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 1 2>&1 | grep -a -v amdgpu.ids | grep -a "mode2" || exit 1
for rep in 1 2; do
  timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/cur  /' || exit 1
  INFLOW_LIB=$ALT/lib_head.so timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/head /' || exit 1
done
done
timeout -k 5 200 python3 tools/probe_split.py 2>/dev/null | head -4
