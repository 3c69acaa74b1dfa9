set -o pipefail
# mesh primary kernel at 4 waves/SIMD (128 VGPR cap) vs the compiler's 142 VGPRs (3 waves)
R=${GRAFT_REPO_ROOT:-$(pwd)}
O=$R/gpurun_out/s4h
mkdir -p $O
for rep in 1 2; do
AB_VARIANTS=1x1,8x1,8x2 timeout -k 10 200 python tools/ab_batch.py bunny mesh_large >> $O/ab_base.log 2>&1 || { echo AFAIL; exit 1; }
RTAMD_LIB=$R/triangles-sdf-cpu-raytracing_amd/lib/var_mw4.so AB_VARIANTS=1x1,8x1,8x2 timeout -k 10 200 python tools/ab_batch.py bunny mesh_large >> $O/ab_mw4.log 2>&1 || { echo AFAIL2; exit 1; }
done
echo ALLOK
