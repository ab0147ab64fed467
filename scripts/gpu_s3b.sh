#!/bin/bash
# GPU tests on the working tree + FM-8 / MVM-10 kernel stats (rocprofv3).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-s3b}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -60 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu_$TAG.log
fi
for m in ${MODELS:-"fm --v-dim 8"}; do :; done
IFS="|" read -ra MS <<< "${MODELS:-fm --v-dim 8|mvm --v-dim 10}"
for m in "${MS[@]}"; do
  mt=$(echo $m | tr -d ' -')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$mt -o run -- python3 bench.py --steps 20 --warmup 5 --model $m > gpurun_out/prof_${TAG}_$mt.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/prof_${TAG}_$mt.log; exit 1; }
  f=$(find gpurun_out/prof_${TAG}_$mt -name "*kernel_stats.csv" | head -1)
  echo "== $m"
  python3 - "$f" <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:16]:
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f} {float(x['Percentage']):6.2f}%")
PY
  find gpurun_out/prof_${TAG}_$mt -name "*kernel_trace.csv" -size +20M -delete
done
