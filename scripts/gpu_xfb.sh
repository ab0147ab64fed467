#!/bin/bash
# GPU tests touching the trainer input path, then the .xfb input-path bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu \
    tests/test_reader.py tests/test_gpu_paths.py > gpurun_out/xfb_tests.log 2>&1 &&
timeout -k 10 300 python -u scripts/xfb_bench.py --rows ${ROWS:-4194304} --epochs 3 > gpurun_out/xfb_stream.log 2>&1 &&
timeout -k 10 300 python -u scripts/xfb_bench.py --rows ${ROWS:-4194304} --epochs 3 --resident > gpurun_out/xfb_resident.log 2>&1 &&
timeout -k 10 300 python -u scripts/xfb_bench.py --rows ${ROWS:-4194304} --epochs 3 --csr-only > gpurun_out/xfb_csr.log 2>&1
rc=$?
tail -3 gpurun_out/xfb_tests.log; tail -1 gpurun_out/xfb_*.log
exit $rc
