#!/bin/bash
# Streamed .xfb input path after dropping the copy stream's wait on compute:
# throughput, then a kernel + memory-copy trace showing H2D next to kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-xfbov}
if [ -z "$SKIP_BENCH" ]; then
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reader.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python -u scripts/xfb_bench.py --rows 8388608 --epochs 4 --test-rows 10000000 > gpurun_out/${TAG}_stream.log 2>&1 || { tail -20 gpurun_out/${TAG}_stream.log; exit 1; }
tail -1 gpurun_out/${TAG}_stream.log
fi
timeout -k 10 300 rocprofv3 --kernel-trace ${PROF_COPY---memory-copy-trace} --output-format csv -d gpurun_out/${TAG}_prof -o run -- python3 scripts/xfb_bench.py --rows 8388608 --epochs 3 > gpurun_out/${TAG}_prof.log 2>&1 || { tail -20 gpurun_out/${TAG}_prof.log; exit 1; }
tail -1 gpurun_out/${TAG}_prof.log
python3 tools/copy_overlap.py gpurun_out/${TAG}_prof > gpurun_out/${TAG}_overlap.txt 2>&1; cat gpurun_out/${TAG}_overlap.txt
find gpurun_out/${TAG}_prof -name "*trace.csv" -size +30M -delete
