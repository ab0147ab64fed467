#!/bin/bash
# dedup LDS level at 4 x kDedupChunk slots (d12) vs 2 x (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ai
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_kernels_misc.py tests/test_determinism.py tests/test_engine_numerics.py \
    > gpurun_out/r6ai/tests.log 2>&1 && tail -1 gpurun_out/r6ai/tests.log &&
STEPS=20 TAG=r6ai_lr ROUNDS=3 bash scripts/gpu.sh ab "base d12" "" &&
STEPS=20 TAG=r6ai_fms ROUNDS=2 bash scripts/gpu.sh ab "base d12" "--model fm --fm-math standard"
