# Phase stamps of the 8x8-scale (s2) series VJP (INFLOW_PHASE_STAMPS build, altlib/lib_stamps.so): the pair and one net
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_stamps_s2
mkdir -p $O
cd $R
INFLOW_LIB=$R/altlib/lib_stamps.so timeout -k 10 120 python tools/series_only.py --scale 2 --mfma 2 --reps 2 > $O/s2_pair.txt 2>&1
INFLOW_LIB=$R/altlib/lib_stamps.so timeout -k 10 120 python tools/series_only.py --scale 2 --mfma 2 --reps 2 --single 1 > $O/s2_single.txt 2>&1
grep -h "timing\|us per" $O/s2_pair.txt $O/s2_single.txt | cut -c1-400
