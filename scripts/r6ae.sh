#!/bin/bash
# k_lr reduction tables of 4 x BLOCK slots (lr4x) vs 2 x BLOCK (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ae
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_csr_slices.py tests/test_plan_paths.py \
    > gpurun_out/r6ae/tests.log 2>&1 && tail -1 gpurun_out/r6ae/tests.log &&
STEPS=20 TAG=r6ae_lr ROUNDS=3 bash scripts/gpu.sh ab "base lr4x" "" &&
STEPS=20 TAG=r6ae_s64 ROUNDS=2 bash scripts/gpu.sh ab "base lr4x" "--slices 64" &&
STEPS=20 TAG=r6ae_s256 ROUNDS=2 bash scripts/gpu.sh ab "base lr4x" "--slices 256"
