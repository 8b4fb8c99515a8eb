# Phase-B attribution: per-wave phase-B spread and per-term time for alternative builds (tools/build_alt.sh)
# and environment knobs.   bash tools/exp_phaseb.sh "name|ENV=VAL ..." ...     (name "cur" = the in-tree build)
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
for SPEC in "$@"; do
  L=${SPEC%%|*}; E=""; case "$SPEC" in *"|"*) E=${SPEC#*|};; esac
  if [ $L = cur ]; then LIBV=""; else LIBV=$GRAFT_REPO_ROOT/gpurun_alt/lib_$L.so; fi
  for S in 0 1; do
    env $E INFLOW_LIB=$LIBV timeout -k 5 90 python3 tools/series_only.py --scale $S --reps 1 2>&1 | grep -a "mode2" | sed "s/^/$SPEC s$S /" || exit 1
    env $E INFLOW_LIB=$LIBV timeout -k 5 90 python3 tools/series_only.py --scale $S --reps 5 2>&1 | grep -a "us/term" | sed "s/^/$SPEC /" || exit 1
  done
done
