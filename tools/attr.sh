cd $GRAFT_REPO_ROOT
for S in 2; do
for rep in 1 2; do
  timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/auto /' || exit 1
  INFLOW_FUSED_VARIANT=2 timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/wide /' || exit 1
  INFLOW_FUSED_VARIANT=2 timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 --batch 128 2>&1 | grep -a "us/term" | sed 's/^/wide /' || exit 1
  timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 --batch 128 2>&1 | grep -a "us/term" | sed 's/^/auto /' || exit 1
done
INFLOW_FUSED_VARIANT=2 INFLOW_FUSED_TIMING=1 timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 1 2>&1 | grep -a -v amdgpu.ids | grep -a "mode2" || exit 1
done
