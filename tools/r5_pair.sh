# The fc JAC pair launch in the chain call: fc / Broyden / golden tests, then POWER and toy bench lines
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_pair
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fcblock.py tests/test_gpu_fcseries.py tests/test_gpu_streams.py tests/test_gpu_parity.py tests/test_gpu_edges.py -k "golden or power or toy or prot_break or chain or block_kernel or fused_fc or fcseries or concurrent or broyden" > $O/tests.log 2>&1
tail -2 $O/tests.log
for rep in 1 2; do
  timeout -k 10 150 python bench.py --config power --cpu-baseline 0 --steps 30 --warmup 3 > $O/power.$rep.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/power.$rep.json').read().strip().splitlines()[-1]);print('power', d['value'], d['ms_per_step'])"
done
timeout -k 10 150 python bench.py --config toy --cpu-baseline 0 --steps 30 > $O/toy.json 2>/dev/null
python -c "import json;d=json.loads(open('$O/toy.json').read().strip().splitlines()[-1]);print('toy', d['value'], d['ms_per_step'])"
