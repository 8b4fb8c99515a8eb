# Round-end measurement part 2: the other BASELINE configs' bench lines, then rocprofv3 kernel stats and the HBM
# PMC passes of the default bench command (tools/profile_round.sh).
set -e
T=${1:-final}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
timeout -k 10 200 python bench.py --config power --steps 5 --warmup 2 > $OUT/bench_power.json 2>/dev/null
timeout -k 10 240 python bench.py --config cifar10_c4 --steps 3 --warmup 1 --cpu-baseline 0 > $OUT/bench_c4_n1.json 2>/dev/null
timeout -k 10 240 python bench.py --config celebahq256 --batch 4 --steps 5 --warmup 2 > $OUT/bench_celebahq256_b4.json 2>/dev/null
timeout -k 10 240 python bench.py --gpus 2 --steps 3 --warmup 1 > $OUT/bench_gpus2.json 2>/dev/null
bash $R/tools/profile_round.sh $T
