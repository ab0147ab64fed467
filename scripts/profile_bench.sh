#!/bin/bash
# rocprofv3 kernel trace + stats of the 1-GPU bench; summaries -> gpurun_out/prof
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
ARGS=${BENCH_ARGS:-"--steps 10 --warmup 3"}
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run -- python3 bench.py $ARGS > gpurun_out/prof/bench.log 2>&1 || { echo "profile failed"; tail -30 gpurun_out/prof/bench.log; exit 1; }
find gpurun_out/prof -name "*kernel_stats.csv" | head -3
f=$(find gpurun_out/prof -name "*kernel_stats.csv" | head -1)
cut -d, -f1-8 "$f" | head -30
tail -1 gpurun_out/prof/bench.log
# drop the big per-dispatch trace; keep stats
find gpurun_out/prof -name "*kernel_trace.csv" -size +20M -delete
