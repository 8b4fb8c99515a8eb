# Round 6: the full -m gpu suite and smoke on this build, then ${NB:-2} CIFAR-10 bench lines (60 steps) with the
# per-kernel times of the residual / Broyden launches.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/${TAG:-check}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in $(seq 1 ${NB:-2}); do
  timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 60 --warmup 5 > $O/b$i.json 2> $O/b$i.err || { echo "bench failed"; tail $O/b$i.err; exit 1; }
  python - "$O/b$i.json" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {k['kernel']: k for k in d['path']['kernels']}
ph = d['roofline'].get('phases', {}).get('broyden', {})
print('value %.1f frac %.4f' % (d['value'], d['roofline']['frac']), 'broyden', ph.get('launches'), ph.get('ms'),
      {k: (v['launches'], v['ms']) for k, v in ks.items() if 'conv_out' in k or 'VJP' in k})
PY
done
exit 0
