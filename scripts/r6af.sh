#!/bin/bash
# reference-FM producer: one 4 x BLOCK table, two barriers (fv4) vs two 2 x BLOCK tables (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6af
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_determinism.py tests/test_engine_numerics.py tests/test_csr_slices.py tests/test_plan_paths.py \
    tests/test_parity_reference.py > gpurun_out/r6af/tests.log 2>&1 && tail -1 gpurun_out/r6af/tests.log &&
STEPS=20 TAG=r6af_fm ROUNDS=3 bash scripts/gpu.sh ab "base fv4" "--model fm" &&
STEPS=20 TAG=r6af_fm8 ROUNDS=2 bash scripts/gpu.sh ab "base fv4" "--model fm --slices 8"
