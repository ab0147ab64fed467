#!/bin/bash
# GPU tests touched this session + models bench + xfb input path.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3r}
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_kernels_misc.py tests/test_reader.py tests/test_engine_numerics.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u scripts/xfb_bench.py --rows 8388608 --epochs 4 --test-rows 10000000 > gpurun_out/${TAG}_xfb_stream.log 2>&1 || { tail -20 gpurun_out/${TAG}_xfb_stream.log; exit 1; }
tail -1 gpurun_out/${TAG}_xfb_stream.log
timeout -k 10 300 python -u scripts/xfb_bench.py --rows 8388608 --epochs 3 --resident > gpurun_out/${TAG}_xfb_resident.log 2>&1 || { tail -20 gpurun_out/${TAG}_xfb_resident.log; exit 1; }
tail -1 gpurun_out/${TAG}_xfb_resident.log
TAG=$TAG SKIP_TESTS=1 SKIP_PROF=1 bash scripts/gpu_models.sh
