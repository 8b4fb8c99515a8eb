# Same-box comparison of POWER bench lines across libraries: the in-tree one ("base") and altlib/lib_<v>.so for each
# argument, interleaved twice
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_ab3
mkdir -p $O
cd $R
L=implicit-normalizing-flows_amd/lib/_hip/libinflow.so
cp $L /tmp/libinflow_base.so
for rep in 1 2; do
  for v in base "$@"; do
    if [ $v = base ]; then cp /tmp/libinflow_base.so $L; else cp altlib/lib_$v.so $L; fi
    timeout -k 10 200 python bench.py --config ${CFG:-power} --cpu-baseline 0 --steps 40 --warmup 5 > $O/$v.$rep.json 2>/dev/null
    python -c "import json;d=json.loads(open('$O/$v.$rep.json').read().strip().splitlines()[-1]);print('$v', d['value'], d['ms_per_step'])"
  done
done
cp /tmp/libinflow_base.so $L
