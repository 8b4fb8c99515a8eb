# gpurun_alt/lib_<name>.so: the library with one kernel source taken from a git revision (A/B runs on one box:
# INFLOW_LIB=gpurun_alt/lib_<name>.so).   bash tools/build_base_alt.sh <name> <rev> <source.hip>
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/implicit-normalizing-flows_amd/csrc
O=$R/implicit-normalizing-flows_amd/lib/_hip/obj
NAME=$1; REV=$2; SRC=$3
mkdir -p $R/gpurun_alt
git -C $R show $REV:implicit-normalizing-flows_amd/csrc/$SRC > $C/_alt_$SRC
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast -c -o /tmp/alt_$NAME.o $C/_alt_$SRC
rm -f $C/_alt_$SRC
OTHERS=$(ls $O/*.o | grep -v "/${SRC%.hip}.o")
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/gpurun_alt/lib_$NAME.so /tmp/alt_$NAME.o $OTHERS
echo built gpurun_alt/lib_$NAME.so
