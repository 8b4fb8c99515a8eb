# A/B of a fused-kernel runtime knob (INFLOW_FUSED_DBG bits) on the paired series, per CIFAR10 scale:
#   bash tools/exp_dbg_ab.sh <dbg-value> [mfma]
cd $GRAFT_REPO_ROOT
V=$1; M=${2:-2}
for S in 0 1 2; do
  for rep in 1 2; do
    timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma $M --reps 5 2>&1 | grep -a "us/term" | sed 's/^/cur   /' || exit 1
    INFLOW_FUSED_DBG=$V timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma $M --reps 5 2>&1 | grep -a "us/term" | sed "s/^/dbg$V /" || exit 1
  done
  INFLOW_FUSED_TIMING=1 timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma $M --reps 1 2>&1 | grep -a "mode2" || exit 1
done
