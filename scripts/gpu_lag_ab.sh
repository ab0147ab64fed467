#!/bin/bash
# Bench run-to-run spread vs the host run-ahead bound (--monitor-lag), with
# the host's issue time per step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-lag}
for rep in 1 2 3; do
  for lag in ${LAGS:-2 8 64}; do
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 --monitor-lag $lag ${EXTRA:-} > gpurun_out/${TAG}.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/${TAG}.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}.log').read().strip().splitlines()[-1]); print('lag', $lag, round(d['value']/1e6,1), 'M', round(d['ms_per_step'],4), 'ms/step, host issue', round(d['host_issue_ms_per_step'],4))"
  done
done
