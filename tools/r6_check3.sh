# Round 6: full -m gpu suite + smoke on this build, then A/B bench lines: default vs ${ALT} (60 steps, twice each).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/${TAG:-check3}
mkdir -p $O
cd $R
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
fi
i=0
for cfg in "" "INFLOW_LIB=$ALT" "" "INFLOW_LIB=$ALT"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 60 --warmup 5 > $O/b$i.json 2> $O/b$i.err || { echo "bench [$cfg] failed"; tail $O/b$i.err; exit 1; }
  python - "$O/b$i.json" "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {k['kernel']: k for k in d['path']['kernels']}
ph = d['roofline'].get('phases', {}).get('broyden', {})
print('%-32s %.1f frac %.4f' % (sys.argv[2][-30:] or 'DEFAULT', d['value'], d['roofline']['frac']), 'broyden', ph.get('launches'), ph.get('ms'),
      {k: round(v['ms'], 3) for k, v in ks.items() if 'EVAL' in k or 'VJP' in k or 'SAVE' in k})
PY
done
exit 0
