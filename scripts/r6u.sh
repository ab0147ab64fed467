#!/bin/bash
# wave folding of repeated dests (fold) vs HEAD (base): GPU tests on the
# in-tree build (= fold), phase timing (ktime), same-box A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6u
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_csr_slices.py \
    tests/test_many_slices.py tests/test_plan_paths.py tests/test_parity_reference.py \
    > gpurun_out/r6u/tests.log 2>&1 &&
tail -2 gpurun_out/r6u/tests.log &&
(cd variants/ktime && timeout -k 10 300 python bench.py --steps 20 --warmup 5 > ../../gpurun_out/r6u/klr.log 2>&1 &&
 timeout -k 10 300 python bench.py --model fm --fm-math standard --steps 20 --warmup 5 > ../../gpurun_out/r6u/kfm.log 2>&1) &&
grep ktime gpurun_out/r6u/klr.log | tail -1 && grep ktime gpurun_out/r6u/kfm.log | tail -1 &&
STEPS=20 TAG=r6u_lr ROUNDS=3 bash scripts/gpu.sh ab "base fold" "" &&
STEPS=20 TAG=r6u_fm ROUNDS=2 bash scripts/gpu.sh ab "base fold" "--model fm" &&
STEPS=20 TAG=r6u_fms ROUNDS=2 bash scripts/gpu.sh ab "base fold" "--model fm --fm-math standard" &&
STEPS=20 TAG=r6u_mvm ROUNDS=2 bash scripts/gpu.sh ab "base fold" "--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9" &&
STEPS=20 TAG=r6u_s256 ROUNDS=2 bash scripts/gpu.sh ab "base fold" "--slices 256"
