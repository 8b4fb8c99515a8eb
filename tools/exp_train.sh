# training step: parts breakdown, the bench line, and the idle-gap analysis of a kernel trace
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/tr
cd $R
timeout -k 10 300 python3 tools/train_step_parts.py --steps 4 > gpurun_out/tr/parts.txt 2>&1
timeout -k 10 300 python3 bench.py --mode train --steps 6 --warmup 2 > gpurun_out/tr/bench.log 2>&1
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/tr/trace -o run -- python3 $R/bench.py --mode train --steps 4 --warmup 2 > $R/gpurun_out/tr/bench_prof.log 2>&1
F=$(find $R/gpurun_out/tr/trace -name '*kernel_trace.csv' | head -1)
python3 $R/tools/timeline_gaps.py $F --skip 0.4 --top 40 > $R/gpurun_out/tr/gaps.txt
S=$(find $R/gpurun_out/tr/trace -name '*kernel_stats.csv' | head -1)
cp $S $R/gpurun_out/tr/kernel_stats.csv
rm -rf $R/gpurun_out/tr/trace
