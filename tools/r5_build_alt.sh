# Timing variant of libinflow.so: a copy of csrc with a python patch applied to one file, fcnet_h3.hip recompiled,
# linked with the in-tree objects -> altlib/lib_<name>.so (tools/r5_alt_trace.sh swaps it in on the GPU box)
#   bash tools/r5_build_alt.sh <name> <patch.py>     (patch.py edits files under $ALT, the copied csrc)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
rm -rf /tmp/alt_$1 && mkdir -p /tmp/alt_$1/x
cp -r $R/implicit-normalizing-flows_amd/csrc /tmp/alt_$1/x/csrc && cp -r $R/include /tmp/alt_$1/include
ALT=/tmp/alt_$1/x/csrc python3 $2
cd /tmp/alt_$1/x/csrc
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=fast -c -o /tmp/alt_$1/fcnet_h3.o fcnet_h3.hip
cd $R
mkdir -p altlib
objs=$(ls implicit-normalizing-flows_amd/lib/_hip/obj/*.o | grep -v fcnet_h3.o)
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o altlib/lib_$1.so /tmp/alt_$1/fcnet_h3.o $objs
echo built altlib/lib_$1.so
