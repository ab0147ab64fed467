#!/bin/bash
# rocprofv3 kernel stats of one bench configuration: ARGS="--model fm --fm-math standard"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-prof1}
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG} -o run -- python3 bench.py --steps 10 --warmup 3 $ARGS > gpurun_out/${TAG}.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/${TAG}.log; exit 1; }
f=$(find gpurun_out/${TAG} -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${TAG}_kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:16]:
    print(f"{x['Name'][:80]:80s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f} {float(x['Percentage']):6.2f}%")
PY
find gpurun_out/${TAG} -name "*kernel_trace.csv" -size +20M -delete
