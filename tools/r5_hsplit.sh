# The hidden-split series VJP: its parity test, the CIFAR-10 reference goldens and k128 / series tests, then the default
# bench line against the 32-pixel kernel (INFLOW_HSPLIT=0) on the same box
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_hs
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py -k "hidden_split or headline or cifar or series or k128" > $O/tests.log 2>&1 || (tail -30 $O/tests.log; exit 1)
tail -1 $O/tests.log
for rep in 1 2; do
  for hs in 1 0; do
    INFLOW_HSPLIT=$hs timeout -k 10 300 python bench.py --cpu-baseline 0 > $O/c10.$hs.$rep.json 2>/dev/null
    python -c "import json;d=json.loads(open('$O/c10.$hs.$rep.json').read().strip().splitlines()[-1]);print('hsplit $hs', d['value'], d['ms_per_step'], d['roofline']['frac'])"
  done
done
