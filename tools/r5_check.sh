# Round 5: GPU tests, the POWER bench line and its kernel trace (per-launch timeline) on the current sha.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5_check}
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
tail -3 $O/gpu_tests.log
timeout -k 10 200 python bench.py --config power --steps 5 --warmup 2 --cpu-baseline 0 > $O/bench_power.json 2>$O/bench_power.err
cat $O/bench_power.json | head -c 400; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_power -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config power --steps 3 --warmup 1 --cpu-baseline 0 > $GRAFT_REPO_ROOT/$O/trace_power.log 2>&1
echo done
