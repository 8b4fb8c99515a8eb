# rocprofv3 kernel-trace stats + HBM traffic PMC passes for the CelebA-HQ 256 config (BASELINE configs[4]), B=4
#   bash tools/profile_c5.sh <tag>   -> gpurun_out/prof_c5_<tag>/
set -e
T=${1:-r03}
R=$GRAFT_REPO_ROOT
cd /tmp && export TMPDIR=/tmp
D=$R/gpurun_out/prof_c5_$T
mkdir -p $D
ARGS="--config celebahq256 --batch 4 --cpu-baseline 0"
INFLOW_EVAL_OVERLAP=0 timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/trace -o run -- python3 $R/bench.py $ARGS --steps 2 --warmup 1 > $D/bench_trace.log 2>&1
INFLOW_EVAL_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $D/fetch -o run -- python3 $R/bench.py $ARGS --steps 1 --warmup 1 > $D/fetch.log 2>&1
INFLOW_EVAL_OVERLAP=0 timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $D/write -o run -- python3 $R/bench.py $ARGS --steps 1 --warmup 1 > $D/write.log 2>&1
ls -R $D | head -30
