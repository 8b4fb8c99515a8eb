#!/bin/bash
# Round-6 final, part E (after the host-side step-start change): smoke() and the default bench line as the driver runs
# it (CIFAR-10 B = 64 with the CPU baseline), then the POWER line
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_final_e
mkdir -p $O
cd $R
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 400 python bench.py > $O/bench_cifar10.json 2> $O/bench_cifar10.err || { tail $O/bench_cifar10.err; exit 1; }
timeout -k 10 200 python bench.py --config power > $O/bench_power.json 2> $O/bench_power.err || { tail $O/bench_power.err; exit 1; }
for f in $O/bench_*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('traffic'), (d.get('cpu_baseline') or {}).get('value'))"; done
