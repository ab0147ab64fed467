#!/bin/bash
# Same-box A/B of an env knob on bench configurations, interleaved.
#   ENVB="XFLOW_NO_SLOT_HINT=1" CONFIGS="lr|fm --v-dim 8" REPS=3 bash scripts/gpu_ab_env.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-abenv}
if [ -n "$TESTS" ]; then
  timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu $TESTS > gpurun_out/${TAG}_tests.log 2>&1 || { tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
  tail -1 gpurun_out/${TAG}_tests.log
fi
IFS='|' read -ra CL <<< "${CONFIGS:-lr}"
for i in $(seq 1 ${REPS:-3}); do
  for c in "${CL[@]}"; do
    for v in A B; do
      if [ $v = B ]; then envs="$ENVB"; else envs="$ENVA"; fi
      env $envs timeout -k 10 300 python bench.py --steps 20 --warmup 5 --model $c > gpurun_out/${TAG}.log 2>&1 || { echo "bench failed: $v $c"; tail -20 gpurun_out/${TAG}.log; exit 1; }
      python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}.log').read().strip().splitlines()[-1]); print('$v', '$c'.ljust(24), round(d['value']/1e6,1), round(d['ms_per_step'],4))"
    done
  done
done
