# Round 6: readback-contract test, A/B of the s2 pre-split (phases A + C vs A only), rocprofv3 kernel stats + HBM PMC
# passes of the default bench command on this build, then PMC pass ${PASS} of the fc block kernel (last: it may crash
# at exit, after its counters are written).
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/${TAG:-prof}
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest tests/test_gpu_readback.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1
[ $rc -eq 0 ] || { tail -30 $O/tests.log; exit $rc; }
i=0
for cfg in "" INFLOW_LIB=altlib/lib_ps_a.so "" INFLOW_LIB=altlib/lib_ps_a.so; do
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
bash tools/profile_round.sh r06c > $O/prof.log 2>&1 || { echo "profile failed"; tail $O/prof.log; exit 1; }
tail -3 $O/prof.log
[ -n "$PASS" ] && bash tools/r6_pmc_fcb_one.sh
exit 0
