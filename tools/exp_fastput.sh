# chunk-1 fast put: A/B timing, the k128 parity subset, and the same subset with the exact-scale path forced
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
bash tools/exp_ab.sh prev || exit 1
INFLOW_FUSED_DBG=16 timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "k128 or headline or golden" 2>&1 | tail -2
