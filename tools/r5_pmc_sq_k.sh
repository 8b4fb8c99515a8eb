# SQ counters of the paired-series VJP at one INF_OPT_FUSED_K128 policy ($1), CIFAR scale $2 (two passes within the SQ
# block's 8-counter limit) -> gpurun_out/r5_sq_k$1_s$2/{a,b}
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
K=${1:-3}
S=${2:-0}
O=$R/gpurun_out/r5_sq_k${K}_s${S}
mkdir -p $O
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE SQ_WAIT_INST_LDS --output-format csv -d $O/a -o run -- python3 $R/tools/series_only.py --scale $S --mfma 2 --reps 1 --k128 $K > $O/a.log 2>&1
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_LEVEL_WAVES SQ_WAVES --output-format csv -d $O/b -o run -- python3 $R/tools/series_only.py --scale $S --mfma 2 --reps 1 --k128 $K > $O/b.log 2>&1
find $O -name "*.csv"
