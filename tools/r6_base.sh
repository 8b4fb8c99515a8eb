# Round 6 baseline on a fresh box: the whole -m gpu suite, smoke, the CIFAR-10 and POWER bench lines, then the fc
# block kernel's three SQ passes (each pass's status recorded; a failed pass ends the script) with their summaries.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/${TAG:-base}
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 300 python bench.py --cpu-baseline 0 > $O/c10.json 2> $O/c10.err || { echo c10 failed; tail $O/c10.err; exit 1; }
timeout -k 10 200 python bench.py --config power --cpu-baseline 0 > $O/power.json 2> $O/power.err || { echo power failed; exit 1; }
for f in c10 power; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f', d['value'], d['ms_per_step'], d['roofline']['frac'])"; done
[ -n "$NOPMC" ] && exit 0
FCB=2 bash tools/r6_pmc_fcblock.sh > $O/pmc_fcb.log 2>&1
rc=$?
cat $O/pmc_fcb.log
python tools/sq_summary.py $R/gpurun_out/r6_pmc_fcb2 fcblock_kernel > $O/pmc_fcb_summary.txt 2>&1
cat $O/pmc_fcb_summary.txt
exit $rc
