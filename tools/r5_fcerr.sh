set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r5_fcerr
timeout -k 10 300 python -u -m pytest -q -s --timeout 120 --timeout-method thread tests/test_gpu_fcblock.py -k "error_at_fp32" > gpurun_out/r5_fcerr/t.log 2>&1
grep "max error" gpurun_out/r5_fcerr/t.log; tail -1 gpurun_out/r5_fcerr/t.log
