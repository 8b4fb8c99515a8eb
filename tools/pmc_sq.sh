set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmc
for M in 0 1; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS -d $R/gpurun_out/pmc/sq_m$M -o run -- python3 $R/tools/series_only.py --mfma $M --reps 1 > $R/gpurun_out/pmc/sq_m$M.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_VALU_MFMA_COEXEC_CYCLES TCC_HIT_sum -d $R/gpurun_out/pmc/sq2_m$M -o run -- python3 $R/tools/series_only.py --mfma $M --reps 1 > $R/gpurun_out/pmc/sq2_m$M.log 2>&1
done
