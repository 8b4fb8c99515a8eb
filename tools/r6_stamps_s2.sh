# Round 6: phase stamps of the wide 32-pixel VJP (s2 pair series) on the kept sources, with and without the pre-split
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r6/stamps_s2
mkdir -p $O
cd $R
INFLOW_LIB=$R/altlib/lib_stamps.so timeout -k 10 120 python tools/series_only.py --scale 2 --mfma 2 --reps 2 --k128 1 > $O/s2.txt 2>&1
INFLOW_FUSED_PRESPLIT=0 INFLOW_LIB=$R/altlib/lib_stamps.so timeout -k 10 120 python tools/series_only.py --scale 2 --mfma 2 --reps 2 --k128 1 > $O/s2_nops.txt 2>&1
grep -h "mode2\|pair" $O/s2.txt $O/s2_nops.txt | cut -c1-330
