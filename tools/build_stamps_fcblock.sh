# The product library with phase stamps in the fc block kernel (fcblock.hip, INFLOW_PHASE_STAMPS=1: per-stage s_memtime
# means printed per launch) as gpurun_alt/lib_fcb_stamps.so; run a tool with INFLOW_LIB=gpurun_alt/lib_fcb_stamps.so.
set -e
R=$(cd "$(dirname "$0")/.." && pwd)
C=$R/implicit-normalizing-flows_amd/csrc
O=$R/implicit-normalizing-flows_amd/lib/_hip/obj
mkdir -p $R/gpurun_alt /tmp/fcb_stamps_obj
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=fast -DINFLOW_PHASE_STAMPS=1 -c -o /tmp/fcb_stamps_obj/fcblock.o $C/fcblock.hip
OTHERS=$(ls $O/*.o | grep -v -e '/fcblock.o')
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o $R/gpurun_alt/lib_fcb_stamps.so /tmp/fcb_stamps_obj/fcblock.o $OTHERS
echo built $R/gpurun_alt/lib_fcb_stamps.so
