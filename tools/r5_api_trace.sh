# HIP API trace (no counters) of a short default bench run: which memcpy / memset calls the eval step makes
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_api
mkdir -p $O
INFLOW_EVAL_OVERLAP=0 timeout -s KILL 240 rocprofv3 --hip-trace --kernel-trace --stats --output-format csv -d $O/raw -o run -- python3 $R/bench.py --cpu-baseline 0 --steps 2 --warmup 1 > $O/bench.log 2>&1
find $O/raw -name "*hip_api_stats.csv" -exec cp {} $O/hip_api_stats.csv \;
find $O/raw -name "*hip_api_trace.csv" -exec cp {} $O/hip_api_trace.csv \;
find $O/raw -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
rm -rf $O/raw
ls -la $O
