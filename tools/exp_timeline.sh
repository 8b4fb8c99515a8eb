# rocprofv3 kernel trace of the default bench's timed steps (overlapped eval schedule), then the idle-gap analysis:
# the union of kernel intervals over the trace after warm-up is the GPU busy fraction of the timed steps
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/tl
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/tl/trace -o run -- python3 $R/bench.py --cpu-baseline 0 --steps 10 --warmup 3 > $R/gpurun_out/tl/bench.log 2>&1
F=$(find $R/gpurun_out/tl/trace -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline_gaps.py $F --skip 0.3 > $R/gpurun_out/tl/gaps.txt
cp $F $R/gpurun_out/tl/kernel_trace.csv
rm -rf $R/gpurun_out/tl/trace
