# rocprofv3 kernel-trace stats + HBM traffic PMC passes for the bench command (run on the GPU box).
#   bash tools/profile_round.sh <tag> [bench args]   -> gpurun_out/prof_<tag>/{kernel_stats.csv, fetch/, write/, *.log}
# The sequential eval schedule (INFLOW_EVAL_OVERLAP=0) matches the bench's per-kernel timing step.  Each PMC pass is
# a run of its own (rocprofv3 does not split counters over passes).
set -e
T=${1:-r01}
shift || true
BARGS="$*"
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
P=$R/gpurun_out/prof_$T
mkdir -p $P
INFLOW_EVAL_OVERLAP=0 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $P/trace -o run -- python3 $R/bench.py --cpu-baseline 0 $BARGS > $P/bench_trace.log 2>&1
cp "$(find $P/trace -name '*kernel_stats.csv' | head -1)" $P/kernel_stats.csv
rm -rf $P/trace
for C in FETCH_SIZE WRITE_SIZE; do
  D=$P/$(echo $C | tr 'A-Z' 'a-z' | cut -d_ -f1)
  INFLOW_EVAL_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc $C --output-format csv -d $D.raw -o run -- python3 $R/bench.py --cpu-baseline 0 --steps 2 --warmup 1 $BARGS > $D.log 2>&1
  mkdir -p $D
  cp "$(find $D.raw -name '*counter_collection.csv' | head -1)" $D/run_counter_collection.csv
  rm -rf $D.raw
done
ls -R $P | head -20
