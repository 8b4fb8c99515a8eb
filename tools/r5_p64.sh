# Round 5: the two-per-CU 64-pixel VJP (fused313p.hip, INF_OPT_FUSED_K128 = 3) against the 128-pixel kernel:
# parity (test_fused_k128_vjp_matches_64px_kernel), series timing per term, rocprofv3 kernel stats of both.
set -e
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r5_p64
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py -k "k128_vjp_matches" > $O/parity.log 2>&1
for S in 0 1; do for K in 1 3; do
  timeout -k 10 120 python tools/series_only.py --scale $S --mfma 2 --reps 5 --k128 $K >> $O/series.txt 2>&1
done; done
cd /tmp
for K in 1 3; do
  timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/st$K -o run -- python3 $R/tools/series_only.py --scale 0 --mfma 2 --reps 3 --k128 $K > $O/st$K.log 2>&1
  cp "$(find $O/st$K -name '*kernel_stats.csv' | head -1)" $O/kernel_stats_k$K.csv
done
cat $O/series.txt
