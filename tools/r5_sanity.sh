# Final build sanity: the default bench line and the POWER line
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_sanity
mkdir -p $O
cd $R
timeout -k 10 300 python bench.py --cpu-baseline 0 > $O/c10.json 2>/dev/null
timeout -k 10 200 python bench.py --config power --cpu-baseline 0 > $O/power.json 2>/dev/null
for f in $O/c10.json $O/power.json; do python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'])"; done
