# POWER / toy bench lines, several repetitions on one box (run-to-run spread)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_reps
mkdir -p $O
cd $R
for rep in 1 2 3 4; do
  timeout -k 10 150 python bench.py --config power --cpu-baseline 0 --steps 40 --warmup 5 > $O/power.$rep.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/power.$rep.json').read().strip().splitlines()[-1]);print('power', d['value'], d['ms_per_step'])"
done
for rep in 1 2; do
  timeout -k 10 150 python bench.py --config toy --cpu-baseline 0 --steps 40 > $O/toy.$rep.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/toy.$rep.json').read().strip().splitlines()[-1]);print('toy', d['value'], d['ms_per_step'])"
done
