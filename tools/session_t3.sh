set -o pipefail
bash tools/gpu_session.sh gpurun_out/r6_t3 tests && bash tools/ab_variants.sh gpurun_out/r6_t3/ab 2 "base ship" bunny mesh_large default_mode && bash tools/gpu_session.sh gpurun_out/r6_t3 bench
