# CIFAR-10 path check: the reference-pinned conv tests, then the default bench line (twice)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_c10
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edges.py -k "headline or cifar or prot_break or broyden" > $O/tests.log 2>&1
tail -1 $O/tests.log
for rep in 1 2; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 > $O/c10.$rep.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/c10.$rep.json').read().strip().splitlines()[-1]);print('c10', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
