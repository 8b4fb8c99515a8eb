# k128 SAVE / EVALSAVE: parity subset, then the bench's per-kernel table (sequential profile step)
cd $GRAFT_REPO_ROOT && mkdir -p gpurun_out
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_edges.py tests/test_gpu_train.py -k "k128 or headline or golden or overlap or train" > gpurun_out/t19.log 2>&1; tail -2 gpurun_out/t19.log
timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --cpu-baseline 0 > gpurun_out/b19.log 2>&1 || exit 1
python3 -c "
import json; d=json.loads(open('gpurun_out/b19.log').read().strip().split('\n')[-1]); print(d['value'], d['ms_per_step'])
for k in d['path']['kernels']: print(k)"
