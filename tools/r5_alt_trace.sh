# Kernel trace of the POWER bench with the in-tree library and with altlib/lib_$1.so (a timing variant built on the
# CPU side); prints the per-kernel table of each (tools/timeline_gaps.py)
set -e
R=$GRAFT_REPO_ROOT
cd $R
L=implicit-normalizing-flows_amd/lib/_hip/libinflow.so
CFG=${CFG:-power} bash tools/r5_timeline_power.sh > /dev/null
grep -A6 "per kernel" gpurun_out/tl_power/gaps.txt
cp gpurun_out/tl_power/gaps.txt gpurun_out/tl_power/gaps_base.txt
cp $L /tmp/libinflow_base.so
cp altlib/lib_$1.so $L
CFG=${CFG:-power} bash tools/r5_timeline_power.sh > /dev/null
cp /tmp/libinflow_base.so $L
echo "--- alt $1"
grep -A6 "per kernel" gpurun_out/tl_power/gaps.txt
cp gpurun_out/tl_power/gaps.txt gpurun_out/tl_power/gaps_$1.txt
