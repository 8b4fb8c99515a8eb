# Round-6 final, part D: the BASELINE configs' bench lines on the final sources (after the last kernel change)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_final_d
mkdir -p $O
cd $R
timeout -k 10 200 python bench.py --config power --cpu-baseline 0 > $O/bench_power.json 2> $O/bench_power.err
timeout -k 10 200 python bench.py --config power --mode trainfwd --steps 20 --warmup 3 --cpu-baseline 0 > $O/bench_power_trainfwd.json 2> $O/bench_power_trainfwd.err
timeout -k 10 200 python bench.py --config toy --cpu-baseline 0 > $O/bench_toy.json 2> $O/bench_toy.err
timeout -k 10 240 python bench.py --config cifar10_c4 --steps 3 --warmup 1 --cpu-baseline 0 > $O/bench_c4_n1.json 2> $O/bench_c4.err
timeout -k 10 240 python bench.py --config celebahq256 --batch 4 --steps 5 --warmup 2 --cpu-baseline 0 > $O/bench_celebahq256_b4.json 2> $O/bench_celebahq.err
timeout -k 10 240 python bench.py --cpu-baseline 0 --steps 60 --warmup 5 > $O/bench_cifar10_60.json 2> $O/bench_cifar10_60.err
for f in $O/bench_*.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('traffic'))"; done
