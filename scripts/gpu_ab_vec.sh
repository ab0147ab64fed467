#!/bin/bash
# Vector-record (standard FM / MVM) A/B of variants/, after the FM / MVM /
# slice GPU tests on the tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "fm or mvm or slice or determin or numerics" > gpurun_out/abvec_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/abvec_tests.log; exit 1; }
tail -1 gpurun_out/abvec_tests.log
ARGS="--model fm --v-dim 8 --fm-math standard --slices 8" ROUNDS=1 bash scripts/gpu_abv.sh && \
ARGS="--model fm --v-dim 8 --fm-math standard --slices 64" ROUNDS=2 bash scripts/gpu_abv.sh && \
ARGS="--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --slices 64" ROUNDS=1 bash scripts/gpu_abv.sh && \
ARGS="--model fm --v-dim 8 --fm-math standard --slices 256" ROUNDS=1 bash scripts/gpu_abv.sh
