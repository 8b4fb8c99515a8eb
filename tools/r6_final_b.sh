# Round-6 final, part B: the other BASELINE configs' bench lines, the two-rank rehearsal, then rocprofv3 kernel stats and
# the HBM PMC passes of the default bench command on the final sources (tools/profile_round.sh)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_final
mkdir -p $O
cd $R
timeout -k 10 200 python bench.py --config power --mode trainfwd --steps 20 --warmup 3 --cpu-baseline 0 > $O/bench_power_trainfwd.json 2> $O/bench_power_trainfwd.err
timeout -k 10 200 python bench.py --config toy --cpu-baseline 0 > $O/bench_toy.json 2> $O/bench_toy.err
timeout -k 10 240 python bench.py --config cifar10_c4 --steps 3 --warmup 1 --cpu-baseline 0 > $O/bench_c4_n1.json 2> $O/bench_c4.err
timeout -k 10 240 python bench.py --config celebahq256 --batch 4 --steps 5 --warmup 2 --cpu-baseline 0 > $O/bench_celebahq256_b4.json 2> $O/bench_celebahq.err
timeout -k 10 240 python bench.py --gpus 2 --steps 3 --warmup 1 --cpu-baseline 0 > $O/bench_gpus2.json 2> $O/bench_gpus2.err
for f in $O/bench_power_trainfwd.json $O/bench_toy.json $O/bench_c4_n1.json $O/bench_celebahq256_b4.json $O/bench_gpus2.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['roofline'].get('frac'))"; done
bash tools/profile_round.sh r06f > $O/prof.log 2>&1
tail -2 $O/prof.log
