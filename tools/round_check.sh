# Full GPU check of the current tree (run on the GPU box from the repo root):
#   bash tools/round_check.sh <tag>  -> gpurun_out/{gpu_tests,smoke,bench,bench_celeba}_<tag>.log + rocprof stats / PMC
set -o pipefail
T=${1:-cur}
cd $GRAFT_REPO_ROOT
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_tests_$T.log 2>&1
rc=$?
tail -3 gpurun_out/gpu_tests_$T.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
[ $rc -eq 1 ] && echo TESTS_FAILED   # the later steps still run for their data; the script exits 1 at the end
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_$T.log 2>&1 || { cat gpurun_out/smoke_$T.log; exit 1; }
tail -1 gpurun_out/smoke_$T.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_$T.log 2>&1 || { tail -20 gpurun_out/bench_$T.log; exit 1; }
cut -c1-300 gpurun_out/bench_$T.log
timeout -k 10 300 python bench.py --config celebahq256 --batch 4 --steps 3 --warmup 1 > gpurun_out/bench_celeba_$T.log 2>&1 || { tail -20 gpurun_out/bench_celeba_$T.log; exit 1; }
cut -c1-300 gpurun_out/bench_celeba_$T.log
bash tools/profile_round.sh $T > /dev/null 2>&1 || { echo PROFILE_FAILED; exit 1; }
echo PROFILE_OK
if [ $rc -eq 1 ]; then echo TESTS_FAILED; exit 1; fi
