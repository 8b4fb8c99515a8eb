cd $GRAFT_REPO_ROOT
ALT=$GRAFT_REPO_ROOT/gpurun_alt
for S in 0 1; do
  INFLOW_FUSED_TIMING=1 timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 1 2>&1 | grep -a -v amdgpu.ids | grep -a "mode2" | sed 's/^/cur /' || exit 1
  INFLOW_LIB=$ALT/lib_nod1.so INFLOW_FUSED_TIMING=1 timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 1 2>&1 | grep -a -v amdgpu.ids | grep -a "mode2" | sed 's/^/nod1 /' || exit 1
  timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/cur  /' || exit 1
  INFLOW_LIB=$ALT/lib_nod1.so timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/nod1 /' || exit 1
done
