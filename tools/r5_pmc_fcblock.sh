# Round 5: SQ counters of the fc block kernel (fcblock.hip) at POWER B = 10000, global rule; two passes.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_pmc_fcb
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/a -o run -- python3 $R/tools/fcblock_probe.py --batch 10000 --reps 1 --modes global --fcb 1 > $O/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_COEXEC_CYCLES SQ_WAVES --output-format csv -d $O/b -o run -- python3 $R/tools/fcblock_probe.py --batch 10000 --reps 1 --modes global --fcb 1 > $O/b.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_SMEM SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_BRANCH SQ_IFETCH SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES --output-format csv -d $O/c -o run -- python3 $R/tools/fcblock_probe.py --batch 10000 --reps 1 --modes global --fcb 1 > $O/c.log 2>&1 || echo "pass c failed"
echo done
