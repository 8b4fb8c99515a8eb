# Round-5 final, part C: the toy line and the POWER two-rank rehearsal on the final build
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_final
mkdir -p $O
cd $R
timeout -k 10 200 python bench.py --config toy > $O/bench_toy.json 2> $O/bench_toy.err
timeout -k 10 240 python bench.py --config power --gpus 2 --steps 10 --warmup 2 --cpu-baseline 0 > $O/bench_power_gpus2.json 2> $O/bench_power_gpus2.err
timeout -k 10 200 python bench.py --config power --cpu-baseline 0 > $O/bench_power_rep2.json 2> /dev/null
for f in $O/bench_toy.json $O/bench_power_gpus2.json $O/bench_power_rep2.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['n_gpus'])"; done
