#!/bin/bash
# Full verification of the shipping build on one box: GPU suite, full-size
# tests, smoke, the driver's bench command, and its rocprofv3 kernel trace.
#   tools/session_verify.sh OUT
set -o pipefail
OUT=${1:-gpurun_out/verify}
bash tools/gpu_session.sh "$OUT" tests fulltests smoke bench prof_driver
