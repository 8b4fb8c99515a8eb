# A/B: engine events without (default) / with (gpurun_alt/lib_sysfence.so) the system-scope fence, POWER and CIFAR-10
# bench lines, interleaved; then the parity tests that read Broyden norms through those events
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_evfence
mkdir -p $O
cd $R
for rep in 1 2; do
for v in nofence sysfence; do
  if [ $v = nofence ]; then L=""; else L=$R/gpurun_alt/lib_sysfence.so; fi
  INFLOW_LIB=$L timeout -k 10 150 python bench.py --config power --cpu-baseline 0 --steps 30 --warmup 3 > $O/power_$v.$rep.json 2>/dev/null
  INFLOW_LIB=$L timeout -k 10 150 python bench.py --cpu-baseline 0 --steps 10 --warmup 2 > $O/c10_$v.$rep.json 2>/dev/null
  for c in power c10; do python -c "import json;d=json.loads(open('$O/${c}_$v.$rep.json').read().strip().splitlines()[-1]);print('$c $v', d['value'], d['ms_per_step'], d['roofline']['achieved'], d['roofline']['frac'])" >> $O/summary.txt; done
done; done
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fcblock.py tests/test_gpu_parity.py -k "golden or power or toy or prot_break or chain or block_kernel or overlap" > $O/tests.log 2>&1
cat $O/summary.txt; tail -2 $O/tests.log
