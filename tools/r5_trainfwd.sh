# POWER train-mode forward (the power series) bench line, twice
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_tf
mkdir -p $O
cd $R
for rep in 1 2; do
  timeout -k 10 200 python bench.py --config power --mode trainfwd --steps 20 --warmup 3 --cpu-baseline 0 > $O/tf.$rep.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/tf.$rep.json').read().strip().splitlines()[-1]);print('trainfwd', d['value'], d['ms_per_step'])"
done
