#!/bin/bash
# Multi-slice A/B of variants/ (FM-8 reference / standard, LR, at --slices 8
# and one slice), then the slice / numerics GPU tests on the tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "slice or numerics or determin" > gpurun_out/abs_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/abs_tests.log; exit 1; }
tail -1 gpurun_out/abs_tests.log
ARGS="--model fm --v-dim 8 --slices 8" ROUNDS=2 bash scripts/gpu_abv.sh && \
ARGS="--model fm --v-dim 8 --fm-math standard --slices 8" ROUNDS=2 bash scripts/gpu_abv.sh && \
ARGS="--slices 8" ROUNDS=2 bash scripts/gpu_abv.sh && \
ARGS="--model fm --v-dim 8" ROUNDS=2 bash scripts/gpu_abv.sh && \
ARGS="" ROUNDS=2 bash scripts/gpu_abv.sh
