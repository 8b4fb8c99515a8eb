# Same-box A/B/A of a bench line: the in-tree library, altlib/lib_$1.so, the in-tree library again (bench args after $1)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_ab
mkdir -p $O
cd $R
V=$1; shift
L=implicit-normalizing-flows_amd/lib/_hip/libinflow.so
cp $L /tmp/libinflow_base.so
for run in base1 alt base2; do
  if [ $run = alt ]; then cp altlib/lib_$V.so $L; else cp /tmp/libinflow_base.so $L; fi
  timeout -k 10 300 python bench.py "$@" > $O/$run.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$run.json').read().strip().splitlines()[-1]);print('$run', d['value'], d['ms_per_step'], d['roofline']['frac'])"
done
cp /tmp/libinflow_base.so $L
