#!/bin/bash
# Kernel trace of the fused and the multi-rank (world 1) bench step; idle time
# between dispatches over the timed steps (tools/trace_gaps.py --marker).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/gaps
for v in ${GAP_VARIANTS:-fused sharded}; do
  extra=""; [ "$v" = sharded ] && extra="--sharded"; [ "$v" = async ] && extra="--async"
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gaps/$v -o run -- python3 bench.py --steps 20 --warmup 3 $extra > gpurun_out/gaps/$v.log 2>&1 || { echo "$v failed"; tail -20 gpurun_out/gaps/$v.log; exit 1; }
  f=$(find gpurun_out/gaps/$v -name "*kernel_trace.csv" | head -1)
  echo "== $v"; tail -1 gpurun_out/gaps/$v.log | cut -c1-200
  python3 tools/trace_gaps.py "$f" --marker k_synth --steps 18 | tee gpurun_out/gaps/$v.txt
  find gpurun_out/gaps/$v -name "*kernel_trace.csv" -size +20M -delete
done
