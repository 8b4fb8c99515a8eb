# The product kernels with phase stamps (INFLOW_PHASE_STAMPS=1: s_memtime at phase boundaries, printed per kernel at
# exit) as altlib/lib_stamps.so; run a tool with INFLOW_LIB=altlib/lib_stamps.so.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/implicit-normalizing-flows_amd/csrc
O=$R/implicit-normalizing-flows_amd/lib/_hip/obj
rm -rf /tmp/stamps_obj; mkdir -p $R/altlib /tmp/stamps_obj
F="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast -DINFLOW_PHASE_STAMPS=1"
for f in fused313 fused313k; do /opt/rocm/bin/hipcc $F -c -o /tmp/stamps_obj/$f.o $C/$f.hip & done
wait
OTHERS=$(ls $O/*.o | grep -v -e '/fused313.o' -e '/fused313k.o')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/altlib/lib_stamps.so /tmp/stamps_obj/fused313.o /tmp/stamps_obj/fused313k.o $OTHERS
echo built $R/altlib/lib_stamps.so
