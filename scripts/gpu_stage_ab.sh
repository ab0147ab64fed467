#!/bin/bash
# GPU tests of the current tree, ABAB of variants named in $ABV (default
# "base stage"; create them first with scripts/make_variant.sh), and kernel
# stats of the current tree.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
ABV="${ABV:-base stage}" ROUNDS=3 bash scripts/gpu_abv.sh || exit 1
BENCH_ARGS="--steps 10 --warmup 3" bash scripts/profile_bench.sh | grep -i "compact\|dedup" 
