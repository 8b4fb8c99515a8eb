# A/B of the current library against gpurun_alt/lib_base.so on the paired series (two alternating rounds), then a
# rocprofv3 kernel trace of the POWER bench for its idle gaps
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4i
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4i/trace -o run -- python3 $R/bench.py --config power --cpu-baseline 0 --steps 5 --warmup 2 > $R/gpurun_out/r4i/power_trace.log 2>&1
F=$(find $R/gpurun_out/r4i/trace -name '*kernel_trace.csv' | head -1)
cp $F $R/gpurun_out/r4i/power_kernel_trace.csv
rm -rf $R/gpurun_out/r4i/trace
cd $R && timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gpu_parity.py -k "k128 or power or toy or fc or headline" > $R/gpurun_out/r4i/tests.log 2>&1
tail -1 $R/gpurun_out/r4i/tests.log
timeout -k 10 200 python bench.py --config power --steps 5 --warmup 2 > $R/gpurun_out/r4i/bench_power.json 2>/dev/null
tail -c 200 $R/gpurun_out/r4i/bench_power.json
