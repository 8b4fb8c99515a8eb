# A/B timing of the paired log-det series per CIFAR10 scale (run on the GPU box, from the repo root):
# the current build, optionally against alternative builds placed in gpurun_alt/lib_<name>.so, plus the
# per-phase s_memtime breakdown (INFLOW_FUSED_TIMING).
#   bash tools/attr.sh [alt-name ...]
cd $GRAFT_REPO_ROOT
ALT=$GRAFT_REPO_ROOT/gpurun_alt
for S in 0 1 2; do
  INFLOW_LIB=gpurun_alt/lib_stamps.so timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 1 2>&1 | grep -a "mode2" || exit 1
  for rep in 1 2; do
    timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/cur  /' || exit 1
    for L in "$@"; do
      INFLOW_LIB=$ALT/lib_$L.so timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed "s/^/$L /" || exit 1
    done
  done
done
