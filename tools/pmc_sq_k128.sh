# SQ counters of the 128-pixel VJP (paired series at CIFAR scales 0 and 1, f16x3), one rocprofv3 pass per scale
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc_k128
for S in 0 1; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $R/gpurun_out/pmc_k128/s$S -o run -- python3 $R/tools/series_only.py --scale $S --mfma 2 --reps 1 > $R/gpurun_out/pmc_k128/s$S.log 2>&1
done
ls $R/gpurun_out/pmc_k128/s0 $R/gpurun_out/pmc_k128/s1
