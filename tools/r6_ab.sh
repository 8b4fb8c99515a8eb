# Round 6 A/B on one box: the parity / edge tests on the new build, then bench lines (value, VJP kernel times) for the
# round-6 changes each turned off alone (ENV=... pairs), all off (= the round-5 schedule) and all on, then (last: it
# may crash at exit) one PMC pass of the fc block kernel with the process maps.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/${TAG:-ab}
mkdir -p $O
cd $R
if [ -z "$NOTEST" ]; then
timeout -k 10 800 python -u -m pytest ${TESTS:-tests/test_gpu_parity.py tests/test_gpu_edges.py} -m gpu -x -v --timeout 200 \
  --timeout-method thread ${K:+-k "$K"} > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1
[ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $O/tests.log | head -20; exit $rc; }
fi
OFF="INFLOW_XCD=0 INFLOW_FUSED_PRESPLIT=0 INFLOW_BROYDEN_FUSED=0 INFLOW_LIB=altlib/lib_nopsa.so"
i=0
for cfg in "$OFF" "" "INFLOW_XCD=0" "INFLOW_FUSED_PRESPLIT=0" "INFLOW_LIB=altlib/lib_nopsa.so" "INFLOW_BROYDEN_FUSED=0" "" "$OFF"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --cpu-baseline 0 ${BARGS} > $O/b$i.json 2> $O/b$i.err || { echo "bench [$cfg] failed"; tail $O/b$i.err; exit 1; }
  python - "$O/b$i.json" "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {k['kernel']: k for k in d['path']['kernels']}
f = lambda n: '%s %.3f/%d' % (n.split('<')[0][7:] + n[n.index('<'):n.index('<') + 4], ks[n]['ms'], ks[n]['launches']) if n in ks else ''
ph = d['roofline'].get('phases', {}).get('broyden', {})
print('%-40s %8.1f %.4f' % (sys.argv[2][:40] or 'ALL ON', d['value'], d['roofline']['frac']), f('net313k_kernel<VJP>'),
      f('net313_kernel_w<VJP>'), f('net313_kernel_w<EVAL>'), 'broyden', ph.get('launches'), ph.get('ms'))
PY
done
[ -n "$PMC" ] && PASS=a bash tools/r6_pmc_fcb_one.sh
exit 0
