# A/B of the fused fc kernels on the POWER bench: gpurun_alt/lib_base.so, the current library and (if present)
# gpurun_alt/lib_alt.so, alternating; then the fc parity tests and a kernel trace of the current library
#   bash tools/exp_fcnet_ab.sh <tag>   -> gpurun_out/<tag>/
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4j}
mkdir -p $O
cd $R
LIBS=${LIBS:-"base cur"}
[ -f gpurun_alt/lib_alt.so ] && LIBS="$LIBS alt"
for rep in 1 2; do
  for n in $LIBS; do
    EV=
    case $n in
      base) L=gpurun_alt/lib_base.so ;;
      noov) L=gpurun_alt/lib_base.so; EV=0 ;;
      alt) L=gpurun_alt/lib_alt.so ;;
      *) L= ;;
    esac
    INFLOW_EVAL_OVERLAP=$EV INFLOW_LIB=$L timeout -k 10 200 python bench.py --config power --cpu-baseline 0 --steps 10 --warmup 3 > $O/${n}_$rep.json 2>/dev/null
    python -c "import json
d=json.loads(open('$O/${n}_$rep.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], d['path']['kernel_busy_frac'], [(k['kernel'], k['launches'], round(k['ms'],3)) for k in d['path']['kernels'][:3]])"
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/ -k "power or toy or fc or exact or tabular or prot_break or broyden" > $O/tests.log 2>&1
tail -1 $O/tests.log
timeout -k 10 200 python tools/host_profile_power.py --steps 5 > $O/host_profile_power.txt 2>&1
head -1 $O/host_profile_power.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 $R/bench.py --config power --cpu-baseline 0 --steps 5 --warmup 2 > $O/prof.log 2>&1
F=$(find $O/prof -name '*kernel_stats.csv' | head -1)
cp $F $O/kernel_stats_power.csv
cp $(find $O/prof -name "*kernel_trace.csv" | head -1) $O/power_kernel_trace.csv
head -4 $O/kernel_stats_power.csv | cut -c1-160
rm -rf $O/prof
