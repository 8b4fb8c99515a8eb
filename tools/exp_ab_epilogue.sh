# A/B of the current library against gpurun_alt/lib_base.so on the paired series (two alternating rounds), then a
# rocprofv3 kernel trace of the POWER bench for its idle gaps
set -e
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/r4i
for rep in 1 2; do
  for L in base cur; do
    for S in 0 1; do
      if [ $L = base ]; then
        INFLOW_LIB=gpurun_alt/lib_base.so timeout -k 5 90 python tools/series_only.py --scale $S --mfma 2 --reps 5 2>&1 | grep -a "us/term" | sed "s/^/$L /"
      else
        timeout -k 5 90 python tools/series_only.py --scale $S --mfma 2 --reps 5 2>&1 | grep -a "us/term" | sed "s/^/$L /"
      fi
    done
  done
done > $R/gpurun_out/r4i/ab.txt
cat $R/gpurun_out/r4i/ab.txt
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 200 rocprofv3 --kernel-trace --output-format csv -d $R/gpurun_out/r4i/trace -o run -- python3 $R/bench.py --config power --cpu-baseline 0 --steps 5 --warmup 2 > $R/gpurun_out/r4i/power_trace.log 2>&1
F=$(find $R/gpurun_out/r4i/trace -name '*kernel_trace.csv' | head -1)
cp $F $R/gpurun_out/r4i/power_kernel_trace.csv
rm -rf $R/gpurun_out/r4i/trace
