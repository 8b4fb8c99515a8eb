# Round 6 A/B, second pass: the full -m gpu suite on the new build (zero-copy conv residual sums, fused Broyden update,
# k128 im2col pre-split), then bench lines (60 steps) per variant, then PMC pass ${PASS} of the fc block kernel (last).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/${TAG:-ab2}
mkdir -p $O
cd $R
if [ -z "$NOTEST" ]; then
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
fi
i=0
L=INFLOW_LIB=altlib/lib_
for cfg in ${CFGS:-"" "INFLOW_FUSED_PRESPLIT=0" ${L}ps_a.so ${L}ps_b.so ${L}ps_c.so ${L}ps_d2.so ${L}nosums.so ${L}nobrf.so "" "INFLOW_FUSED_PRESPLIT=0"}; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 60 --warmup 5 > $O/b$i.json 2> $O/b$i.err || { echo "bench [$cfg] failed"; tail $O/b$i.err; exit 1; }
  python - "$O/b$i.json" "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {k['kernel']: k for k in d['path']['kernels']}
f = lambda n: '%s %.3f/%d' % (n.split('<')[0][7:] + n[n.index('<'):n.index('<') + 4], ks[n]['ms'], ks[n]['launches']) if n in ks else ''
ph = d['roofline'].get('phases', {}).get('broyden', {})
print('%-40s %8.1f %.4f' % (sys.argv[2][:40] or 'DEFAULT', d['value'], d['roofline']['frac']), f('net313k_kernel<VJP>'),
      f('net313_kernel_w<VJP>'), f('net313_kernel_w<EVAL>'), 'broyden', ph.get('launches'), ph.get('ms'))
PY
done
[ -n "$PASS" ] && bash tools/r6_pmc_fcb_one.sh
exit 0
