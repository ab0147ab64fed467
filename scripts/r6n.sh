#!/bin/bash
# claimer-flushed ListAgg (LR / reference FM / MVM column producers): GPU
# tests on the in-tree build, same-box A/B against the previous build, and
# the LR step's kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6n
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_csr_slices.py \
    tests/test_many_slices.py tests/test_plan_paths.py tests/test_parity_reference.py \
    > gpurun_out/r6n/tests.log 2>&1 &&
tail -2 gpurun_out/r6n/tests.log &&
TAG=r6n_ab ROUNDS=3 bash scripts/gpu.sh ab "base lrcf" "" &&
TAG=r6n_abfm ROUNDS=2 bash scripts/gpu.sh ab "base lrcf" "--model fm" &&
TAG=r6n_prof bash scripts/gpu.sh prof ""
