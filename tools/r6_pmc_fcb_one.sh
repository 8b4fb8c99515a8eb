# Round 6: ONE rocprofv3 --pmc pass over the fc block kernel (fcblock.hip, forced on: --fcb 2) at POWER B = 10000, global
# rule, with the process's /proc/self/maps written at exit, so the frames of an exit-time crash map to their libraries.
# PASS=a|b|c picks the counter set; the exit status is recorded, nothing runs after the pass.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_pmc_fcb_${PASS:-a}
mkdir -p $O
case ${PASS:-a} in
  a) C="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS";;
  b) C="SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES";;
  c) C="SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES";;
esac
timeout -s KILL 90 rocprofv3 --pmc $C --output-format csv -d $O/out -o run -- \
  python3 $R/tools/fcblock_probe.py --batch 10000 --reps 1 --modes global --fcb ${FCB:-2} --maps $O/maps.txt > $O/log.txt 2>&1
rc=$?
echo "pass ${PASS:-a} fcb ${FCB:-2} rc=$rc counters: $C" > $O/status.txt
cat $O/status.txt
python $R/tools/sq_summary.py $O/out fcblock_kernel > $O/summary.txt 2>&1; cat $O/summary.txt
exit 0
