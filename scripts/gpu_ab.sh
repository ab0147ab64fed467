#!/bin/bash
# A/B of bench.py variants on one GPU (each a separate process), then the
# rocprofv3 kernel stats of the default configuration.
#   VARIANTS="|--overlap on|--sharded" TAG=x bash scripts/gpu_ab.sh   (empty entry = defaults)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-ab}
mkdir -p gpurun_out
IFS="|" read -ra VS <<< "${VARIANTS-|--overlap on|--sharded}"
for v in "${VS[@]}"; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 $v > gpurun_out/ab_$TAG.log 2>&1 || { echo "bench [$v] failed"; tail -20 gpurun_out/ab_$TAG.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/ab_$TAG.log').read().strip().splitlines()[-1]); print('[$v]', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],3), 'ms/step')"
done
if [ -z "$NO_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_$TAG -o run -- python3 bench.py --steps 20 --warmup 5 $PROF_ARGS > gpurun_out/prof_$TAG.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/prof_$TAG.log; exit 1; }
  f=$(find gpurun_out/prof_$TAG -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f} {float(x['Percentage']):6.2f}%")
PY
  find gpurun_out/prof_$TAG -name "*kernel_trace.csv" -size +20M -delete
fi
