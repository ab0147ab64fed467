#!/bin/bash
# CAS-on-free column tables (u32 tags freed by their claimers): GPU tests on
# the in-tree build (= cas), phase timing (variants/ktime), A/B pos vs cas
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6p
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_csr_slices.py \
    tests/test_many_slices.py tests/test_plan_paths.py tests/test_parity_reference.py \
    > gpurun_out/r6p/tests.log 2>&1 &&
tail -2 gpurun_out/r6p/tests.log &&
(cd variants/ktime && timeout -k 10 300 python bench.py --model fm --fm-math standard --steps 20 \
    --warmup 5 > ../../gpurun_out/r6p/ktime.log 2>&1) && grep ktime gpurun_out/r6p/ktime.log | tail -1 &&
STEPS=20 TAG=r6p_lr ROUNDS=2 bash scripts/gpu.sh ab "pos cas" "" &&
STEPS=20 TAG=r6p_fm ROUNDS=2 bash scripts/gpu.sh ab "pos cas" "--model fm" &&
STEPS=20 TAG=r6p_fms ROUNDS=2 bash scripts/gpu.sh ab "pos cas" "--model fm --fm-math standard" &&
STEPS=20 TAG=r6p_mvm ROUNDS=2 bash scripts/gpu.sh ab "pos cas" "--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9" &&
STEPS=20 TAG=r6p_s256 ROUNDS=2 bash scripts/gpu.sh ab "pos cas" "--slices 256"
