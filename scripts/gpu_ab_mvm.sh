#!/bin/bash
# MVM A/B (live SGD and the degenerate default) of variants/, then the MVM GPU tests on the tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ARGS="--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9" ROUNDS=2 bash scripts/gpu_abv.sh && \
ARGS="--model mvm --v-dim 10" ROUNDS=2 bash scripts/gpu_abv.sh && \
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "mvm" > gpurun_out/abmvm_tests.log 2>&1; tail -2 gpurun_out/abmvm_tests.log
