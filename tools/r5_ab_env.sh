# Same-box A/B of the default bench line: the in-tree library vs altlib/lib_$1.so (INFLOW_LIB), interleaved twice
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_abe
mkdir -p $O
cd $R
V=$1; shift
for rep in 1 2; do
  timeout -k 10 300 python bench.py --cpu-baseline 0 "$@" > $O/base.$rep.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/base.$rep.json').read().strip().splitlines()[-1]);print('base', d['value'], d['ms_per_step'])"
  INFLOW_LIB=$R/altlib/lib_$V.so timeout -k 10 300 python bench.py --cpu-baseline 0 "$@" > $O/$V.$rep.json 2>/dev/null
  python -c "import json;d=json.loads(open('$O/$V.$rep.json').read().strip().splitlines()[-1]);print('$V', d['value'], d['ms_per_step'])"
done
