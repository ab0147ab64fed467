#!/bin/bash
# Slice-group applies that skip untouched keys: GPU tests on the tree, then A/B of variants/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "slice or determin or numerics or paths or sharded or multirank or fm or mvm" > gpurun_out/abskip_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/abskip_tests.log; exit 1; }
tail -1 gpurun_out/abskip_tests.log
ARGS="--model fm --v-dim 8 --slices 256" ROUNDS=2 bash scripts/gpu_abv.sh && \
ARGS="--model fm --v-dim 8 --slices 64" ROUNDS=1 bash scripts/gpu_abv.sh && \
ARGS="--model fm --v-dim 8 --fm-math standard --slices 64" ROUNDS=1 bash scripts/gpu_abv.sh && \
ARGS="--model fm --v-dim 8 --slices 8" ROUNDS=1 bash scripts/gpu_abv.sh && \
ARGS="--model fm --v-dim 8" ROUNDS=1 bash scripts/gpu_abv.sh
