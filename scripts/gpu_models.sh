#!/bin/bash
# GPU tests + bench of every model family (1 GPU), with kernel stats for FM
# and MVM.  SKIP_TESTS=1 skips pytest.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-models}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu_$TAG.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu_$TAG.log; exit 1; }
  tail -1 gpurun_out/pytest_gpu_$TAG.log
fi
MODELS=${MODELS:-"lr|lr --slices 8|lr --sharded|lr --async|fm --v-dim 8|fm --v-dim 8 --fm-math standard|fm --v-dim 10|mvm --v-dim 10|lr --optimizer sgd"}
IFS='|' read -ra MLIST <<< "$MODELS"
for m in "${MLIST[@]}"; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --model $m > gpurun_out/bench_${TAG}.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/bench_${TAG}.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_${TAG}.log').read().strip().splitlines()[-1]); print('$m', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],3), 'ms/step logloss', round(d['logloss'],4))"
done
[ -n "$SKIP_PROF" ] && exit 0
for m in "fm --v-dim 8" "mvm --v-dim 10"; do
  mt=$(echo $m | tr -d ' -')
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_${TAG}_$mt -o run -- python3 bench.py --steps 5 --warmup 2 --model $m > gpurun_out/prof_${TAG}_$mt.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/prof_${TAG}_$mt.log; exit 1; }
  f=$(find gpurun_out/prof_${TAG}_$mt -name "*kernel_stats.csv" | head -1)
  echo "== $m"
  python3 - "$f" <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:10]:
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f} {float(x['Percentage']):6.2f}%")
PY
  find gpurun_out/prof_${TAG}_$mt -name "*kernel_trace.csv" -size +20M -delete
done
