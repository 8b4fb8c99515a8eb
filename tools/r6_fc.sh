# Round 6: the fc-path GPU tests (block kernel, series, fc goldens, edges), then the POWER / toy bench lines.
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/${TAG:-fc}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest tests/test_gpu_fcblock.py tests/test_gpu_fcseries.py tests/test_gpu_edges.py \
  "tests/test_gpu_parity.py" -k "${K:-fc or power or toy or prot or block or series or edge or threshold or stall or degenerate or banach or chain}" \
  -x -v --timeout 120 --timeout-method thread -m gpu > $O/tests.log 2>&1 || { echo "tests failed"; tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
timeout -k 10 200 python -u bench.py --config power --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench_power.json 2> $O/bench_power.err || { echo "bench power failed"; tail -20 $O/bench_power.err; exit 1; }
timeout -k 10 200 python -u bench.py --config toy --steps 20 --warmup 5 --cpu-baseline 0 > $O/bench_toy.json 2> $O/bench_toy.err || { echo "bench toy failed"; exit 1; }
python - <<PY
import json
for n in ('power', 'toy'):
    d = json.loads(open('$O/bench_%s.json' % n).read().strip().splitlines()[-1])
    print(n, d['value'], d['unit'], d.get('roofline', {}).get('frac'))
PY
