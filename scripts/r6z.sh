#!/bin/bash
# synth: per-field offsets in LDS (syn2) vs HEAD (base); tests, smoke, A/B
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6z
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_kernels_misc.py tests/test_determinism.py > gpurun_out/r6z/tests.log 2>&1 &&
tail -1 gpurun_out/r6z/tests.log && TAG=r6z_smoke bash scripts/gpu.sh smoke &&
STEPS=20 TAG=r6z_lr ROUNDS=3 bash scripts/gpu.sh ab "base syn2" ""
