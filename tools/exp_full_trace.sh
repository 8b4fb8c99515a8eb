# Full GPU test suite, then a rocprofv3 kernel trace of the POWER bench (timed steps) for the idle-gap analysis
#   bash tools/exp_full_trace.sh <tag>   -> gpurun_out/<tag>/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4m}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
tail -1 $O/gpu_tests.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --config power --cpu-baseline 0 --steps 5 --warmup 2 > $O/trace.log 2>&1
F=$(find $O/trace -name '*kernel_trace.csv' | head -1)
cp $F $O/power_kernel_trace.csv
rm -rf $O/trace
