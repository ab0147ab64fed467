#!/bin/bash
# Build and run the kernel experiment harness (tools/kbench.hip) on the GPU.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out build
if [ ! -x build/kbench ] || [ -n "$REBUILD" ]; then
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
    -Icsrc/include -Icsrc/hip tools/kbench.hip csrc/hip/kernels_table.hip \
    csrc/hip/kernels_model.hip csrc/hip/kernels_synth.hip -o build/kbench || exit 1
fi
timeout -k 10 300 build/kbench $KBENCH_ARGS 2>&1 | tee gpurun_out/kbench_${TAG:-x}.log
