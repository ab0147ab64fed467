#!/bin/bash
# quality rows, standard-FM PMC, async-PS GPU tests (incl. the async Trainer)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6h
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_async_ps_gpu.py > gpurun_out/r6h/async_tests.log 2>&1 &&
TAG=r6g_quality bash scripts/quality.sh &&
TAG=r6g_pmc bash scripts/gpu.sh pmc "--model fm --fm-math standard" "k_fm_std_red|k_red_sum_vec"
