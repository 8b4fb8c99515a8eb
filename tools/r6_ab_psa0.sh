# Round 6: s1 stamps with chunk 0's im2col planes in the chunk buffer, the k128 / golden tests, then bench A/B against
# K128_PSA0 = 0 and (the wide kernel) PSD = 2
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/psa0
mkdir -p $O
cd $R
INFLOW_LIB=$R/altlib/lib_stamps.so timeout -k 10 120 python tools/series_only.py --scale 1 --mfma 2 --reps 2 --k128 1 > $O/s1.txt 2>&1 || exit 1
grep -h "mode2\|pair" $O/s1.txt | cut -c1-330
INFLOW_LIB=altlib/lib_psa0.so timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "k128 or cifar or headline or split_bf16" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; [ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head; exit $rc; }
i=0
for cfg in "" "INFLOW_LIB=altlib/lib_psa0.so" "INFLOW_LIB=altlib/lib_psd2.so" "" "INFLOW_LIB=altlib/lib_psa0.so" "INFLOW_LIB=altlib/lib_psd2.so"; do
  i=$((i+1))
  env $cfg timeout -k 10 300 python bench.py --cpu-baseline 0 --steps 60 --warmup 5 > $O/b$i.json 2> $O/b$i.err || { echo "bench [$cfg] failed"; tail $O/b$i.err; exit 1; }
  python - "$O/b$i.json" "$cfg" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ks = {k['kernel']: k for k in d['path']['kernels']}
print('%-32s %.1f frac %.4f' % (sys.argv[2][-30:] or 'DEFAULT', d['value'], d['roofline']['frac']),
      {k: round(v['ms'], 3) for k, v in ks.items() if 'VJP' in k or 'EVAL>' in k})
PY
done
exit 0
