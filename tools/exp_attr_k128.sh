# Time attribution of the 128-pixel VJP with diagnostic builds (tools/build_alt_k128.py; wrong results): per-scale
# paired-series time and phase stamps for the tree's library and each gpurun_alt/lib_<name>.so given.
#   bash tools/exp_attr_k128.sh <name> ...
cd $GRAFT_REPO_ROOT
for L in cur "$@"; do
  E=""; [ $L != cur ] && E="INFLOW_LIB=$GRAFT_REPO_ROOT/gpurun_alt/lib_$L.so"
  for S in 0 1 2; do
    env $E timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 2 --reps 5 2>&1 | grep -a "us/term" | sed "s/^/$L /" || exit 1
    env $E timeout -k 5 60 python3 tools/series_only.py --scale $S --mfma 2 --reps 1 2>&1 | grep -a "mode2 split" | sed "s/^/$L /" || exit 1
  done
done
