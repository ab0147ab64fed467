#!/bin/bash
# LR producer at 512 rows per workgroup (two per CU, 4 x BLOCK tables) vs 1024 (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6aj
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_plan_paths.py \
    > gpurun_out/r6aj/tests.log 2>&1 && tail -1 gpurun_out/r6aj/tests.log &&
STEPS=20 TAG=r6aj_lr ROUNDS=3 bash scripts/gpu.sh ab "base lr512" "" &&
STEPS=20 TAG=r6aj_lr2 ROUNDS=2 bash scripts/gpu.sh ab "lr512 base" ""
