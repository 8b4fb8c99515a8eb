# Phase stamps of the 128-pixel VJP (INFLOW_PHASE_STAMPS build, gpurun_alt/lib_stamps.so) on the paired series, s0 / s1
set -e
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_stamps
mkdir -p $O
cd $R
for S in 0 1; do
  INFLOW_LIB=$R/gpurun_alt/lib_stamps.so timeout -k 10 120 python tools/series_only.py --scale $S --mfma 2 --reps 2 --k128 1 > $O/s$S.txt 2>&1
done
cat $O/s0.txt $O/s1.txt
