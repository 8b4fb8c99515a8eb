# Round 6: s2 phase stamps with the phase-B ring and the 6-unit staging, the wide-kernel tests, then bench A/B against WB_DEPTH = 2 / STAGE_WU = 4
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/wb
mkdir -p $O
cd $R
INFLOW_LIB=$R/altlib/lib_stamps.so timeout -k 10 120 python tools/series_only.py --scale 2 --mfma 2 --reps 2 --k128 1 > $O/s2.txt 2>&1 || exit 1
grep -h "mode2\|pair" $O/s2.txt | cut -c1-330
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -v --timeout 200 --timeout-method thread -k "presplit or wide_variant or cifar or headline" > $O/tests.log 2>&1
rc=$?; grep -E "passed|failed" $O/tests.log | tail -1; [ $rc -eq 0 ] || exit $rc
NOTEST=1 TAG=wb_ab ALT=altlib/lib_wb2.so bash tools/r6_check3.sh
