# Round-6 final, part A: the GPU test suite and smoke() on the final build, then the default bench line (as the driver
# runs it: CIFAR-10 B = 64 with the CPU baseline) and the POWER line
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_final
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/gpu_tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_cifar10.json 2> $O/bench_cifar10.err || { tail $O/bench_cifar10.err; exit 1; }
timeout -k 10 200 python bench.py --config power > $O/bench_power.json 2> $O/bench_power.err || { tail $O/bench_power.err; exit 1; }
for f in $O/bench_*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('traffic'), d.get('cpu_baseline',{}).get('value'))"; done
