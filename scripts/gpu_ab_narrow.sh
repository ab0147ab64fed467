#!/bin/bash
# Many-slice A/B of variants/ (LR and reference FM at 64 / 256 slices, one
# slice unchanged), after the slice / determinism / numerics GPU tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests -k "slice or determin or numerics or paths" > gpurun_out/abn_tests.log 2>&1 || { echo "tests failed"; tail -30 gpurun_out/abn_tests.log; exit 1; }
tail -1 gpurun_out/abn_tests.log
ARGS="--slices 256" ROUNDS=2 bash scripts/gpu_abv.sh && \
ARGS="--slices 64" ROUNDS=2 bash scripts/gpu_abv.sh && \
ARGS="--model fm --v-dim 8 --slices 256" ROUNDS=1 bash scripts/gpu_abv.sh && \
ARGS="" ROUNDS=2 bash scripts/gpu_abv.sh
