# Same-box A/B/A/B of the POWER bench line: in-tree library vs altlib/lib_$1.so
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_abp
mkdir -p $O
cd $R
V=$1
L=implicit-normalizing-flows_amd/lib/_hip/libinflow.so
cp $L /tmp/libinflow_base.so
for run in base1 alt1 base2 alt2; do
  case $run in alt*) cp altlib/lib_$V.so $L;; *) cp /tmp/libinflow_base.so $L;; esac
  timeout -k 10 200 python bench.py --config power --cpu-baseline 0 --steps 40 --warmup 5 > $O/$run.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$run.json').read().strip().splitlines()[-1]);print('$run', d['value'], d['ms_per_step'])"
done
cp /tmp/libinflow_base.so $L
