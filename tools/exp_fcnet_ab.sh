# A/B of the fused fc kernels (current library against gpurun_alt/lib_base.so) on the POWER bench, a kernel trace of
# the current one, and the fc parity tests
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r4j
mkdir -p $O
cd $R
for rep in 1 2; do
  INFLOW_LIB=gpurun_alt/lib_base.so timeout -k 10 200 python bench.py --config power --cpu-baseline 0 --steps 10 --warmup 3 > $O/base_$rep.json 2>/dev/null
  timeout -k 10 200 python bench.py --config power --cpu-baseline 0 --steps 10 --warmup 3 > $O/cur_$rep.json 2>/dev/null
  python -c "import json,sys
for n in ('base','cur'):
  d=json.loads(open('$O/'+n+'_$rep.json').read().strip().splitlines()[-1]); print(n, d['value'], d['ms_per_step'], [ (k['kernel'], k['launches'], round(k['ms'],3)) for k in d['path']['kernels'][:3]])"
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "power or toy or fc or exact or tabular or prot_break or broyden" > $O/tests.log 2>&1
tail -1 $O/tests.log
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --config power --cpu-baseline 0 --steps 5 --warmup 2 > $O/prof.log 2>&1
F=$(find $O/prof -name '*kernel_stats.csv' | head -1)
cp $F $O/kernel_stats_power.csv
head -6 $O/kernel_stats_power.csv | cut -c1-160
rm -rf $O/prof
