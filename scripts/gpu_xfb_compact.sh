#!/bin/bash
# Streamed .xfb input path: 64-bit keys vs compact (u32) keys, with the
# H2D/step overlap from HIP events (XFLOW_STREAM_TIMELINE=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-xfbc}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reader.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for mode in wide compact; do
  hs=0; [ $mode = compact ] && hs=1000000000
  XFLOW_STREAM_TIMELINE=1 timeout -k 10 400 python -u scripts/xfb_bench.py --rows ${ROWS:-8388608} --epochs 4 \
      --hash-space $hs --dir /tmp/xfb_$mode > gpurun_out/${TAG}_$mode.log 2>&1 || { echo "$mode failed"; tail -20 gpurun_out/${TAG}_$mode.log; exit 1; }
  tail -1 gpurun_out/${TAG}_$mode.log
done
