#!/bin/bash
# compaction output staged in LDS and stored densely (cst) vs HEAD+dcas (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ab
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_kernels_misc.py tests/test_determinism.py tests/test_engine_numerics.py \
    tests/test_table_growth.py > gpurun_out/r6ab/tests.log 2>&1 &&
tail -1 gpurun_out/r6ab/tests.log && TAG=r6ab_smoke bash scripts/gpu.sh smoke &&
STEPS=20 TAG=r6ab_lr ROUNDS=3 bash scripts/gpu.sh ab "base cst" "" &&
STEPS=20 TAG=r6ab_fms ROUNDS=2 bash scripts/gpu.sh ab "base cst" "--model fm --fm-math standard"
