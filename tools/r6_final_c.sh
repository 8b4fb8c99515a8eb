# Round-6 final, part C (after the last kernel change): the GPU suite and smoke, the default bench line, then rocprofv3
# kernel stats + HBM PMC passes of the default bench command on these sources
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_final_c
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/gpu_tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/gpu_tests.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1 || { tail $O/smoke.txt; exit 1; }
tail -1 $O/smoke.txt
timeout -k 10 300 python bench.py --cpu-baseline 0 > $O/bench_cifar10.json 2> $O/bench_cifar10.err || { tail $O/bench_cifar10.err; exit 1; }
python -c "import json;d=json.loads(open('$O/bench_cifar10.json').read().strip().splitlines()[-1]);print('c10', d['value'], d['ms_per_step'], d['roofline'].get('frac'))"
bash tools/profile_round.sh r06g > $O/prof.log 2>&1 || { tail $O/prof.log; exit 1; }
tail -2 $O/prof.log
