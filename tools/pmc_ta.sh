# TA / TD / TCP pressure of the fused VJP kernel (s0 series, x6 and exact fp32), one pass per counter group.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/pmcta
for M in 1 0; do
timeout -s KILL 90 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max TD_TD_BUSY_sum GRBM_GUI_ACTIVE --output-format csv -d $R/gpurun_out/pmcta/a_m$M -o run -- python3 $R/tools/series_only.py --mfma $M --reps 1 > $R/gpurun_out/pmcta/a_m$M.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc TCP_TCC_READ_REQ_LATENCY_sum TCP_TCC_READ_REQ_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum --output-format csv -d $R/gpurun_out/pmcta/b_m$M -o run -- python3 $R/tools/series_only.py --mfma $M --reps 1 > $R/gpurun_out/pmcta/b_m$M.log 2>&1
done
