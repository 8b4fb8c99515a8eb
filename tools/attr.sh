cd $GRAFT_REPO_ROOT
for rep in 1 2; do
  timeout -k 5 60 python3 tools/series_only.py --scale 0 --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/rec   /' || exit 1
  INFLOW_D1_RECOMP=0 timeout -k 5 60 python3 tools/series_only.py --scale 0 --mfma 1 --reps 5 2>&1 | grep -a "us/term" | sed 's/^/norec /' || exit 1
done
INFLOW_FUSED_TIMING=1 timeout -k 5 60 python3 tools/series_only.py --scale 0 --mfma 1 --reps 1 2>&1 | grep -a -v amdgpu.ids | grep -a "mode2" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t.log 2>&1; tail -2 gpurun_out/t.log
