# Parity subset + bench of an alternative build gpurun_alt/lib_<name>.so against the tree's library (GPU box):
#   bash tools/exp_alt_lib.sh <name>
cd $GRAFT_REPO_ROOT
L=$GRAFT_REPO_ROOT/gpurun_alt/lib_$1.so
INFLOW_LIB=$L timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -q -x --timeout 120 --timeout-method thread > gpurun_out/alt_$1_tests.log 2>&1 || { tail -30 gpurun_out/alt_$1_tests.log; exit 1; }
tail -1 gpurun_out/alt_$1_tests.log
for r in 1 2; do
  timeout -k 10 240 python bench.py --cpu-baseline 0 --steps 10 > gpurun_out/b_cur.log 2>&1 || exit 1
  echo "cur  $(tail -1 gpurun_out/b_cur.log | cut -c100-140)"
  INFLOW_LIB=$L timeout -k 10 240 python bench.py --cpu-baseline 0 --steps 10 > gpurun_out/b_alt.log 2>&1 || exit 1
  echo "$1 $(tail -1 gpurun_out/b_alt.log | cut -c100-140)"
done
