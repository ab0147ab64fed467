#!/bin/bash
# Session-3 check: GPU tests on the working tree, then same-box A/B of the
# FM apply variants (variants/base vs variants/fmw).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_s3.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -60 gpurun_out/pytest_gpu_s3.log; exit 1; }
tail -2 gpurun_out/pytest_gpu_s3.log
ABV="${ABV:-base fmw}" ARGS="--model fm --v-dim 8" ROUNDS=2 bash scripts/gpu_abv.sh
ABV="${ABV:-base fmw}" ARGS="--model mvm --v-dim 10" ROUNDS=1 bash scripts/gpu_abv.sh
