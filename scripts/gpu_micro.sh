#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-micro}
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 tools/microbench.py $MICRO_ARGS > gpurun_out/prof_$TAG.log 2>&1 || { echo "micro failed"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
grep n_unique gpurun_out/prof_$TAG.log
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f} {float(x['Percentage']):6.2f}%")
PY
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -size +20M -delete
