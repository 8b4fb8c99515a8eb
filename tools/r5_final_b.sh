# Round-5 final, part B: the bench lines of every BASELINE config on the final build
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_final
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py > $O/bench_cifar10.json 2> $O/bench_cifar10.err
timeout -k 10 200 python bench.py --config power > $O/bench_power.json 2> $O/bench_power.err
timeout -k 10 200 python bench.py --config power --mode trainfwd --steps 20 --warmup 3 > $O/bench_power_trainfwd.json 2> $O/bench_power_trainfwd.err
timeout -k 10 240 python bench.py --config cifar10_c4 --steps 3 --warmup 1 --cpu-baseline 0 > $O/bench_c4_n1.json 2> $O/bench_c4.err
timeout -k 10 240 python bench.py --config celebahq256 --batch 4 --steps 5 --warmup 2 > $O/bench_celebahq256_b4.json 2> $O/bench_celebahq.err
timeout -k 10 240 python bench.py --gpus 2 --steps 3 --warmup 1 --cpu-baseline 0 > $O/bench_gpus2.json 2> $O/bench_gpus2.err
for f in $O/bench_*.json; do python -c "import json,sys;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['roofline'].get('frac'), d['roofline'].get('traffic'))"; done
