# fused vs generic (INFLOW_NO_FUSED=1) per-term time of the paired series, per scale and batch
cd $GRAFT_REPO_ROOT
for S in 2 1; do for B in 64 256; do
  timeout -k 5 90 python3 tools/series_only.py --scale $S --batch $B --reps 3 2>&1 | grep -a "us/term" | sed 's/^/fused   /' || exit 1
  INFLOW_NO_FUSED=1 timeout -k 5 90 python3 tools/series_only.py --scale $S --batch $B --reps 3 2>&1 | grep -a "us/term" | sed 's/^/generic /' || exit 1
done; done
