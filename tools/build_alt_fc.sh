# Alternative libinflow.so with extra compile flags on fcnet_h3.hip only (A/B experiments on the fc kernels):
#   bash tools/build_alt_fc.sh <name> "<flags>"   ->  gpurun_alt/lib_<name>.so  (INFLOW_LIB=gpurun_alt/lib_<name>.so)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/implicit-normalizing-flows_amd/csrc
O=$R/implicit-normalizing-flows_amd/lib/_hip/obj
mkdir -p $R/gpurun_alt
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=fast $2 -c -o /tmp/altfc_$1.o $C/fcnet_h3.hip
objs=""
for f in $O/*.o; do case $f in */fcnet_h3.o) ;; *) objs="$objs $f";; esac; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/gpurun_alt/lib_$1.so /tmp/altfc_$1.o $objs
echo built gpurun_alt/lib_$1.so
