#!/bin/bash
# standard-FM producer tail: sub-range starts from registers (tailr) vs HEAD (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ad
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_csr_slices.py tests/test_determinism.py tests/test_engine_numerics.py tests/test_plan_paths.py \
    > gpurun_out/r6ad/tests.log 2>&1 && tail -1 gpurun_out/r6ad/tests.log &&
STEPS=20 TAG=r6ad_fms ROUNDS=3 bash scripts/gpu.sh ab "base tailr" "--model fm --fm-math standard" &&
STEPS=20 TAG=r6ad_mvm ROUNDS=2 bash scripts/gpu.sh ab "base tailr" "--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9"
