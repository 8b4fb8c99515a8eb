# Round-5 final, part A: the GPU test suite and smoke() on the final build
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05_final
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -q --timeout 120 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.txt 2>&1
tail -3 $O/gpu_tests.log; cat $O/smoke.txt | tail -2
