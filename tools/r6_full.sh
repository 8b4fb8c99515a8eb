# Round 6: the whole -m gpu suite (as the driver runs it) and smoke, logs under gpurun_out/r6/${TAG:-full}.
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/${TAG:-full}
mkdir -p $O
cd $R
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread ${ARGS} > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed" $O/tests.log | tail -2
[ $rc -eq 0 ] || { grep -E "FAILED|Error" $O/tests.log | head -20; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo smoke failed; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
