# Kernel traces of the POWER bench (CFG to change the config) with the in-tree library and with each of
# altlib/lib_<name>.so (timing variants built on the CPU side, tools/r5_build_alt.sh); the per-kernel table of each
set -e
R=$GRAFT_REPO_ROOT
cd $R
L=implicit-normalizing-flows_amd/lib/_hip/libinflow.so
cp $L /tmp/libinflow_base.so
for v in base "$@"; do
  if [ $v != base ]; then cp altlib/lib_$v.so $L; fi
  CFG=${CFG:-power} bash tools/r5_timeline_power.sh > /dev/null
  cp /tmp/libinflow_base.so $L
  echo "--- $v"
  grep -A5 "per kernel" gpurun_out/tl_power/gaps.txt
  cp gpurun_out/tl_power/gaps.txt gpurun_out/tl_power/gaps_$v.txt
done
