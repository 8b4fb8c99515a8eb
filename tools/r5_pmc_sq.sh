# Round 5: SQ counters of the 128-pixel VJP on the current sha (paired series, CIFAR scales 0 and 1, f16x3).
# Two passes per scale (each within the SQ block's 8-counter limit), plus the device's counter list.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_pmc_sq
mkdir -p $O
timeout -s KILL 60 rocprofv3 -L > $O/counters.txt 2>&1 || true
for S in 0 1; do
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/a$S -o run -- python3 $R/tools/series_only.py --scale $S --mfma 2 --reps 1 > $O/a$S.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES --output-format csv -d $O/b$S -o run -- python3 $R/tools/series_only.py --scale $S --mfma 2 --reps 1 > $O/b$S.log 2>&1 || echo "pass b$S failed rc=$?"
done
find $O -name "*.csv"
