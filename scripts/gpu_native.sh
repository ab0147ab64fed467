#!/bin/bash
# Native binary input path on the GPU: xflow_lr on a synthetic Criteo-shaped
# libffm shard with synchronous (XFLOW_SYNC_STAGING=1) vs double-buffered
# async H2D staging, then a kernel + memory-copy trace of the async run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-native}
mkdir -p $O /tmp/xfdata
python3 tools/gen_libffm.py /tmp/xfdata/tr ${ROWS:-300000} --seed 1 && python3 tools/gen_libffm.py /tmp/xfdata/te 20000 --seed 2 || exit 1
ls -la /tmp/xfdata
for mode in sync async; do
  extra=""; [ $mode = sync ] && export XFLOW_SYNC_STAGING=1 || unset XFLOW_SYNC_STAGING
  s=$(date +%s.%N)
  (cd $O && timeout -k 10 300 ../../build/bin/xflow_lr /tmp/xfdata/tr /tmp/xfdata/te 0 ${EPOCHS:-3} --threads 1 --device 0 --train-block-bytes ${BLOCK:-33554432} > native_$mode.log 2>&1) || { echo "$mode failed"; tail $O/native_$mode.log; exit 1; }
  e=$(date +%s.%N)
  echo "$mode: $(python3 -c "print(round($e - $s, 3))") s  $(grep logloss $O/native_$mode.log)"
done
unset XFLOW_SYNC_STAGING
(cd $O && timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --stats --output-format csv -d trace -o run -- ../../build/bin/xflow_lr /tmp/xfdata/tr /tmp/xfdata/te 0 1 --threads 1 --device 0 --train-block-bytes ${BLOCK:-33554432} > native_trace.log 2>&1) || { echo "trace failed"; tail $O/native_trace.log; exit 1; }
find $O/trace -name "*_stats.csv" | head
find $O/trace -name "*kernel_trace.csv" -size +20M -delete
