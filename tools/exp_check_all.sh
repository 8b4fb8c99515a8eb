# Full GPU test suite, then the CIFAR and POWER bench lines without the CPU baseline (A/B against a base library when
# gpurun_alt/lib_base.so exists)
#   bash tools/exp_check_all.sh <tag>   -> gpurun_out/<tag>/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4q}
mkdir -p $O
cd $R
[ -n "$SKIP_TESTS" ] || timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
[ -n "$SKIP_TESTS" ] || tail -1 $O/gpu_tests.log
for rep in 1 2; do
  for n in base cur; do
    L=; [ $n = base ] && L=gpurun_alt/lib_base.so
    [ $n = base ] && [ ! -f gpurun_alt/lib_base.so ] && continue
    INFLOW_LIB=$L timeout -k 10 240 python bench.py --cpu-baseline 0 --steps 20 --warmup 5 > $O/b64_${n}_$rep.json 2>/dev/null
    INFLOW_LIB=$L timeout -k 10 200 python bench.py --config power --cpu-baseline 0 --steps 10 --warmup 3 > $O/power_${n}_$rep.json 2>/dev/null
    python -c "import json
for c in ('b64', 'power'):
  d=json.loads(open('$O/'+c+'_${n}_$rep.json').read().strip().splitlines()[-1]); print('$n', c, d['value'], d['ms_per_step'], d['path']['kernel_busy_frac'])"
  done
done
