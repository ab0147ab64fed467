#!/bin/bash
# CSR reduction / column-atomic tables with one CAS per probe step (ccas) vs HEAD (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6ac
timeout -k 10 600 python -u -m pytest -x -q --timeout 240 --timeout-method thread -m gpu \
    tests/test_csr_slices.py tests/test_many_slices.py tests/test_plan_paths.py tests/test_determinism.py \
    > gpurun_out/r6ac/tests.log 2>&1 && tail -1 gpurun_out/r6ac/tests.log &&
STEPS=20 TAG=r6ac_s256 ROUNDS=2 bash scripts/gpu.sh ab "base ccas" "--slices 256" &&
STEPS=20 TAG=r6ac_s64 ROUNDS=2 bash scripts/gpu.sh ab "base ccas" "--slices 64" &&
STEPS=20 TAG=r6ac_fm256 ROUNDS=2 bash scripts/gpu.sh ab "base ccas" "--model fm --slices 256" &&
STEPS=20 TAG=r6ac_fms64 ROUNDS=2 bash scripts/gpu.sh ab "base ccas" "--model fm --fm-math standard --slices 64"
