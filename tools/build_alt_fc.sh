# Alternative libinflow.so with extra compile flags on fcnet_h3.hip only (A/B experiments on the fc kernels):
#   bash tools/build_alt_fc.sh <name> "<flags>"   ->  altlib/lib_<name>.so  (tools/r5_ab3_power.sh swaps it in)
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/implicit-normalizing-flows_amd/csrc
O=$R/implicit-normalizing-flows_amd/lib/_hip/obj
mkdir -p $R/altlib
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -ffp-contract=fast $2 -c -o /tmp/altfc_$1.o $C/fcnet_h3.hip
objs=""
for f in $O/*.o; do case $f in */fcnet_h3.o) ;; *) objs="$objs $f";; esac; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/altlib/lib_$1.so /tmp/altfc_$1.o $objs
echo built altlib/lib_$1.so
