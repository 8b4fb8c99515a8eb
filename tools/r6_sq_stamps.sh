# Round 6: phase stamps (INFLOW_PHASE_STAMPS build with sub-stamps) and SQ counters of the 128-pixel VJP on the kept
# sources, CIFAR-10 s0 / s1 paired series (tools/series_only.py).
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/sq_stamps
mkdir -p $O
cd $R
for S in 0 1; do
  INFLOW_LIB=$R/altlib/lib_stamps.so timeout -k 10 120 python tools/series_only.py --scale $S --mfma 2 --reps 2 --k128 1 > $O/stamps_s$S.txt 2>&1
done
grep -h "timing\|us" $O/stamps_s0.txt | tail -4
cd /tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/a -o run -- python3 $R/tools/series_only.py --scale 0 --mfma 2 --reps 1 --k128 1 > $O/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LEVEL_WAVES SQ_WAVES --output-format csv -d $O/b -o run -- python3 $R/tools/series_only.py --scale 0 --mfma 2 --reps 1 --k128 1 > $O/b.log 2>&1
python $R/tools/sq_summary.py $O > $O/sq_summary.txt; cat $O/sq_summary.txt
