# per-phase / per-wave cycles of the 64-px VJP kernel (INFLOW_FUSED_TIMING build stamps)
set -e
mkdir -p gpurun_out
INFLOW_LIB=gpurun_alt/lib_stamps.so timeout -k 10 120 python tools/series_only.py --scale 0 --batch 64 --reps 2 >> gpurun_out/exp3.log 2>&1
INFLOW_LIB=gpurun_alt/lib_stamps.so timeout -k 10 120 python tools/series_only.py --scale 1 --batch 64 --reps 2 >> gpurun_out/exp3.log 2>&1
