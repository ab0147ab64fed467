#!/bin/bash
# MVM producer: one workgroup per CU with a 2x column table (mvm2x) vs two per CU (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ah
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_csr_slices.py tests/test_plan_paths.py \
    > gpurun_out/r6ah/tests.log 2>&1 && tail -1 gpurun_out/r6ah/tests.log &&
STEPS=20 TAG=r6ah_mvm ROUNDS=3 bash scripts/gpu.sh ab "base mvm2x" "--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9" &&
STEPS=20 TAG=r6ah_mvm64 ROUNDS=2 bash scripts/gpu.sh ab "base mvm2x" "--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --slices 64"
