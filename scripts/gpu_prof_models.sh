#!/bin/bash
# rocprofv3 kernel stats of a few bench configurations (PROF_CFGS: "name|args;...").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/profm
IFS=';' read -ra CFGS <<< "$PROF_CFGS"
for c in "${CFGS[@]}"; do
  n="${c%%|*}"; a="${c#*|}"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profm/$n -o run -- python3 bench.py --steps 20 --warmup 5 $a > gpurun_out/profm/$n.log 2>&1 || { echo "profile $n failed"; tail -5 gpurun_out/profm/$n.log; exit 1; }
  f=$(find gpurun_out/profm/$n -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/profm/${n}_kernel_stats.csv
  find gpurun_out/profm/$n -name "*kernel_trace.csv" -delete
  echo "$n: $(tail -1 gpurun_out/profm/$n.log | cut -c1-120)"
done
