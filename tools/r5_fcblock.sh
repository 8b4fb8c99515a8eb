# Round 5: the device-resident fc block kernel -- its tests, the fc goldens, the POWER bench line and a kernel trace.
set -e
cd $GRAFT_REPO_ROOT
O=gpurun_out/${1:-r5_fcblock}
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_fcblock.py -x -v --timeout 200 --timeout-method thread > $O/tests_fcblock.log 2>&1 || { tail -40 $O/tests_fcblock.log; exit 1; }
tail -3 $O/tests_fcblock.log
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "power or toy or fc or prot_break or tabular" > $O/tests_fc.log 2>&1 || { tail -40 $O/tests_fc.log; exit 1; }
tail -3 $O/tests_fc.log
timeout -k 10 200 python bench.py --config power --steps 5 --warmup 2 --cpu-baseline 0 > $O/bench_power.json 2>$O/bench_power.err
head -c 300 $O/bench_power.json; echo
cd /tmp && export TMPDIR=/tmp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/$O/trace_power -o run -- python3 $GRAFT_REPO_ROOT/bench.py --config power --steps 3 --warmup 1 --cpu-baseline 0 > $GRAFT_REPO_ROOT/$O/trace_power.log 2>&1
echo done
