# A/B of the FWD fc kernel's column blocks per workgroup (FC_FWD_NCB 1 / 2 / 3) on the POWER bench (2 rounds)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/ab_fc_fwd
mkdir -p $O
cd $R
for rep in 1 2; do
for v in base n1 n2; do
  if [ $v = base ]; then L=""; else L=$R/gpurun_alt/lib_$v.so; fi
  INFLOW_LIB=$L timeout -k 10 120 python bench.py --config power --cpu-baseline 0 --steps 30 --warmup 3 > $O/$v.$rep.json 2> $O/$v.$rep.err
  python -c "import json;d=json.loads(open('$O/$v.$rep.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'], [(k['kernel'],k['ms'],k['launches']) for k in d['path']['kernels'][:2]])" >> $O/summary.txt
done; done
cat $O/summary.txt
