#!/bin/bash
# synth: the per-field hash term precomputed (syn) vs HEAD (base); tests, smoke, A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6y
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_kernels_misc.py tests/test_determinism.py tests/test_engine_numerics.py \
    > gpurun_out/r6y/tests.log 2>&1 && tail -1 gpurun_out/r6y/tests.log &&
TAG=r6y_smoke bash scripts/gpu.sh smoke &&
STEPS=20 TAG=r6y_lr ROUNDS=3 bash scripts/gpu.sh ab "base syn" ""
