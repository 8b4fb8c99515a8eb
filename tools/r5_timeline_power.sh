# rocprofv3 kernel trace of the POWER bench's timed steps, then the idle-gap analysis (tools/timeline_gaps.py)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/tl_power
mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $O/trace -o run -- python3 $R/bench.py --config ${CFG:-power} --cpu-baseline 0 --steps 30 --warmup 3 > $O/bench.log 2>&1
F=$(find $O/trace -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline_gaps.py $F --skip 0.3 --window ${WIN:-60} > $O/gaps.txt
rm -rf $O/trace
tail -62 $O/gaps.txt
