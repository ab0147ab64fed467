#!/bin/bash
# One GPU iteration: gpu tests, 1-GPU bench, rocprofv3 kernel stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/prof
TAG=${TAG:-iter}
ARGS=${BENCH_ARGS:-"--steps 20 --warmup 5"}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_gpu_$TAG.log
fi
timeout -k 10 300 python bench.py $ARGS > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/bench_$TAG.log; exit 1; }
grep metric gpurun_out/bench_$TAG.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py $ARGS > gpurun_out/prof_$TAG.log 2>&1 || { echo "profile failed"; tail -30 gpurun_out/prof_$TAG.log; exit 1; }
f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f} {float(x['Percentage']):6.2f}%")
PY
find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -size +20M -delete
