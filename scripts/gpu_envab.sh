#!/bin/bash
# Same-box A/B of environment settings, interleaved (ROUNDS times):
#   ENVS="|XFLOW_LR_SLOT_GRADS=1" ARGS="--model lr" bash scripts/gpu_envab.sh
set -o pipefail
mkdir -p gpurun_out
IFS="|" read -ra ES <<< "${ENVS-|}"
for r in $(seq 1 ${ROUNDS:-2}); do
  for e in "${ES[@]}"; do
    env $e timeout -k 10 300 python bench.py --steps 30 --warmup 5 ${ARGS:-} > gpurun_out/envab.log 2>&1 || { echo "[$e] failed"; tail -20 gpurun_out/envab.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/envab.log').read().strip().splitlines()[-1]); print('round $r [$e]', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],4), 'ms/step', 'logloss', round(d['logloss'],5))"
  done
done
