# rocprofv3 kernel-trace stats + HBM traffic PMC passes for the bench command (run on the GPU box).
#   bash tools/profile_round.sh <tag>
set -e
T=${1:-r01}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
mkdir -p $R/gpurun_out/prof_$T
INFLOW_EVAL_OVERLAP=0 timeout -s KILL 240 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/prof_$T/trace -o run -- python3 $R/bench.py --cpu-baseline 0 > $R/gpurun_out/prof_$T/bench_trace.log 2>&1
INFLOW_EVAL_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $R/gpurun_out/prof_$T/fetch -o run -- python3 $R/bench.py --cpu-baseline 0 --steps 2 --warmup 1 > $R/gpurun_out/prof_$T/fetch.log 2>&1
INFLOW_EVAL_OVERLAP=0 timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $R/gpurun_out/prof_$T/write -o run -- python3 $R/bench.py --cpu-baseline 0 --steps 2 --warmup 1 > $R/gpurun_out/prof_$T/write.log 2>&1
ls -R $R/gpurun_out/prof_$T | head -30
