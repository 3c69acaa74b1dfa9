set -o pipefail
bash tools/gpu_session.sh gpurun_out/r6_t4 tests && bash tools/oneframe_prof.sh gpurun_out/r6_t4/of bunny:stanford-bunny.obj:1920:1080:primary,dm:stanford-bunny.obj:1920:1080:default && bash tools/gpu_session.sh gpurun_out/r6_t4 bench && bash tools/ab_variants.sh gpurun_out/r6_t4/ab 2 "ship octmaj" octree octree_shipped
