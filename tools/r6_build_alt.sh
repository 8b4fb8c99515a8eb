# A/B variant of libinflow.so: one source file recompiled with extra flags (e.g. -DK128_PSA=0), linked with the in-tree
# objects of the others -> altlib/lib_<name>.so (bench / tests pick it with INFLOW_LIB=altlib/lib_<name>.so)
#   bash tools/r6_build_alt.sh <name> <file.hip> "<flags>"
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/implicit-normalizing-flows_amd/csrc
base=$(basename $2 .hip)
mkdir -p $R/altlib /tmp/alt_$1
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=fast $3 -c -o /tmp/alt_$1/$base.o $C/$2
objs=$(ls $R/implicit-normalizing-flows_amd/lib/_hip/obj/*.o | grep -v "/$base.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/altlib/lib_$1.so /tmp/alt_$1/$base.o $objs
echo built altlib/lib_$1.so
