#!/bin/bash
# k_lr: one 8 x BLOCK table, two barriers (lr8s) vs two 4 x BLOCK tables (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ag
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_plan_paths.py \
    > gpurun_out/r6ag/tests.log 2>&1 && tail -1 gpurun_out/r6ag/tests.log &&
STEPS=20 TAG=r6ag_lr ROUNDS=3 bash scripts/gpu.sh ab "base lr8s" "" &&
STEPS=20 TAG=r6ag_s64 ROUNDS=2 bash scripts/gpu.sh ab "base lr8s" "--slices 64"
