# The overlapped fc chain (engine.hip chain_overlapped): the chain / fc-block / fcseries / parity tests, then the chain
# vs block-by-block A/B on POWER (launch path), then the POWER bench line.
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_chain
mkdir -p $O
cd $R
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fcblock.py tests/test_gpu_fcseries.py > $O/tests.log 2>&1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "power or toy or prot_break or fused_fc" > $O/parity.log 2>&1
timeout -k 10 200 python tools/ab_chain.py --reps 10 --fcb 1 > $O/ab.txt 2>&1
timeout -k 10 200 python bench.py --config power --cpu-baseline 0 --steps 30 --warmup 3 > $O/bench_power.json 2> $O/bench_power.err
tail -3 $O/tests.log $O/parity.log; cat $O/ab.txt
python -c "import json;d=json.loads(open('$O/bench_power.json').read().strip().splitlines()[-1]);print(d['value'], d['ms_per_step'])"
