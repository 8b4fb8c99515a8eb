# 8 x 8 block tiles at CelebA-HQ 256's 64 x 64 scale: the parity tests that run it, then the C5 bench against
# gpurun_alt/lib_base.so (alternating)
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${1:-r4z}
mkdir -p $O
cd $R
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ -k "wide_variant or celebahq or headline or golden" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -1 $O/tests.log
for rep in 1 2; do
  for n in base cur; do
    L=; [ $n = base ] && L=gpurun_alt/lib_base.so
    INFLOW_LIB=$L timeout -k 10 240 python bench.py --config celebahq256 --batch 4 --cpu-baseline 0 --steps 4 --warmup 1 > $O/c5_${n}_$rep.json 2>/dev/null
    python -c "import json
d=json.loads(open('$O/c5_${n}_$rep.json').read().strip().splitlines()[-1]); print('$n', d['value'], d['ms_per_step'], [(k['kernel'], k['launches'], round(k['ms'],3)) for k in d['path']['kernels'][:4]])"
  done
done
