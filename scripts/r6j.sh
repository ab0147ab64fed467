#!/bin/bash
# MVM quality rows at a 74 % CTR; scan A/B; then the claimer-flush FM-std
# producer: its tests, two benches and a PMC pass
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6j
TAG=r6j_quality ONLY="planted-bias" bash scripts/quality.sh &&
bash scripts/r6i.sh &&
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_csr_slices.py \
    tests/test_many_slices.py tests/test_plan_paths.py tests/test_step_plan.py \
    tests/test_parity_reference.py > gpurun_out/r6j/fm_tests.log 2>&1 &&
tail -3 gpurun_out/r6j/fm_tests.log &&
TAG=r6j_fm bash scripts/gpu.sh bench "--model fm --fm-math standard" &&
TAG=r6j_fm2 bash scripts/gpu.sh bench "--model fm --fm-math standard" &&
TAG=r6j_pmc bash scripts/gpu.sh pmc "--model fm --fm-math standard" "k_fm_std_red"
