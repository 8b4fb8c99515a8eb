# Round 6: SQ counters of the fc block kernel (fcblock.hip) at POWER B = 10000, global rule; three passes.  Each pass's
# exit status goes to status.txt; a failed pass (fault, abort, crash at exit) ends the script there, recorded.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6_pmc_fcb${FCB:-2}
mkdir -p $O
: > $O/status.txt
PROBE="python3 $R/tools/fcblock_probe.py --batch 10000 --reps 1 --modes global --fcb ${FCB:-2}"
run_pass() {
  local name=$1; shift
  timeout -s KILL 90 rocprofv3 --pmc "$@" --output-format csv -d $O/$name -o run -- $PROBE > $O/$name.log 2>&1
  local rc=$?
  echo "pass $name rc=$rc counters: $*" >> $O/status.txt
  return $rc
}
run_pass a SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS &&
run_pass b SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES &&
run_pass c SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES
rc=$?
echo "done rc=$rc" >> $O/status.txt
cat $O/status.txt
exit $rc
