#!/bin/bash
# Host-side step-start change (cached log-det weights, raw-stream lookup): the host window again, the GPU suite,
# then the CIFAR-10 bench line without the CPU leg, twice
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_hostgap
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/r6_hostgap.py 20 > $O/after.txt 2>&1 || { tail $O/after.txt; exit 1; }
head -2 $O/after.txt | tail -1
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/gpu_tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; }
for r in 1 2; do
  timeout -k 10 400 python bench.py --steps 60 --cpu-baseline 0 > $O/bench_cifar10_$r.json 2> $O/bench_$r.err || { tail $O/bench_$r.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_cifar10_$r.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
  # the previous commit's host Python (bench.py + lib/, same libinflow.so) on the same box
  timeout -k 10 400 python altlib/base_py/bench.py --steps 60 --cpu-baseline 0 > $O/bench_base_$r.json 2> $O/bench_base_$r.err || { tail $O/bench_base_$r.err; exit 1; }
  python -c "import json;d=json.loads(open('$O/bench_base_$r.json').read().strip().splitlines()[-1]);print('base', d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
done
