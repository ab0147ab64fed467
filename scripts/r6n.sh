#!/bin/bash
# claimer-flushed ListAgg (lrcf) and chunk-prefetched column positions (pos,
# on top of lrcf): GPU tests on the in-tree build (= pos), then same-box A/B
# against the previous build (base) for LR, reference FM, standard FM, MVM
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6n
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_csr_slices.py \
    tests/test_many_slices.py tests/test_plan_paths.py tests/test_parity_reference.py \
    > gpurun_out/r6n/tests.log 2>&1 &&
tail -2 gpurun_out/r6n/tests.log &&
STEPS=20 TAG=r6n_lr ROUNDS=2 bash scripts/gpu.sh ab "base lrcf pos" "" &&
STEPS=20 TAG=r6n_fm ROUNDS=2 bash scripts/gpu.sh ab "base lrcf pos" "--model fm" &&
STEPS=20 TAG=r6n_fms ROUNDS=2 bash scripts/gpu.sh ab "base pos" "--model fm --fm-math standard" &&
STEPS=20 TAG=r6n_mvm ROUNDS=2 bash scripts/gpu.sh ab "base lrcf pos" "--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9"
