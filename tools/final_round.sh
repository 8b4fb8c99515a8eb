# Round-end measurement part 1: full GPU test suite, smoke, the default bench line and the other configs' lines.
#   bash tools/final_round.sh <tag>      (results under gpurun_out/<tag>)
set -e
T=${1:-final}
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/$T
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/ > $OUT/gpu_tests.log 2>&1 || { tail -20 $OUT/gpu_tests.log; exit 1; }
tail -1 $OUT/gpu_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.txt 2>&1
tail -2 $OUT/smoke.txt
timeout -k 10 420 python bench.py > $OUT/bench_b64.json 2> $OUT/bench_b64.err
tail -c 300 $OUT/bench_b64.json
