#!/bin/bash
# double-buffered standard-FM column tables (db: one barrier per column) vs HEAD (base):
# GPU tests on the in-tree build (= db), same-box A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6x
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_csr_slices.py \
    tests/test_many_slices.py tests/test_plan_paths.py tests/test_parity_reference.py \
    > gpurun_out/r6x/tests.log 2>&1 &&
tail -2 gpurun_out/r6x/tests.log &&
STEPS=20 TAG=r6x_fms ROUNDS=3 bash scripts/gpu.sh ab "base db" "--model fm --fm-math standard" &&
STEPS=20 TAG=r6x_fms64 ROUNDS=2 bash scripts/gpu.sh ab "base db" "--model fm --fm-math standard --slices 64" &&
STEPS=20 TAG=r6x_fms16 ROUNDS=2 bash scripts/gpu.sh ab "base db" "--model fm --fm-math standard --v-dim 16"
