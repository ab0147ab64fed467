#!/bin/bash
# FM-std producer with the larger int32 column table: tests, benches, kernel
# stats; MVM live bench (same kernel, int64 form); then the headline A/B (r6k)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6l
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_csr_slices.py \
    tests/test_many_slices.py tests/test_plan_paths.py tests/test_step_plan.py \
    tests/test_parity_reference.py > gpurun_out/r6l/fm_tests.log 2>&1 &&
tail -2 gpurun_out/r6l/fm_tests.log &&
TAG=r6l_fm bash scripts/gpu.sh bench "--model fm --fm-math standard" &&
TAG=r6l_fm2 bash scripts/gpu.sh bench "--model fm --fm-math standard" &&
TAG=r6l_fm64 bash scripts/gpu.sh bench "--model fm --fm-math standard --slices 64" &&
TAG=r6l_mvm bash scripts/gpu.sh bench "--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9" &&
TAG=r6l_prof MARKER=k_synth bash scripts/gpu.sh prof "--model fm --fm-math standard" &&
bash scripts/r6k.sh &&
bash scripts/r6m.sh
