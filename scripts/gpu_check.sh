#!/bin/bash
# First-contact GPU validation: numerics tests, smoke, 1-GPU bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -50 gpurun_out/pytest_gpu.log; exit 1; }
tail -3 gpurun_out/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/smoke.log; exit 1; }
cat gpurun_out/smoke.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 > gpurun_out/bench1.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench1.log; exit 1; }
cat gpurun_out/bench1.log
