#!/bin/bash
# Streamed libffm text through the Trainer with the GPU tokenizer: parallel
# positional reads per block (8 / 16 / 24), 64 MB blocks, 4 epochs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
for t in ${THREADS:-8 16 24}; do
  timeout -k 10 400 python -u scripts/text_bench.py --rows ${ROWS:-4000000} --block-mb 64 --epochs 4 --copy-threads $t --dir /tmp/text_bench > gpurun_out/text_t$t.log 2>&1 || { echo "text bench $t failed"; tail -20 gpurun_out/text_t$t.log; exit 1; }
  echo "copy_threads=$t"; grep "^gpu_parse" gpurun_out/text_t$t.log
done
