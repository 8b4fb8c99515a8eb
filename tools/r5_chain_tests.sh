set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_chain
timeout -k 10 400 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_fcblock.py -k "chain" > gpurun_out/r5_chain/t.log 2>&1 || (tail -40 gpurun_out/r5_chain/t.log; exit 1)
tail -1 gpurun_out/r5_chain/t.log
