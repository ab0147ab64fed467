#!/bin/bash
# Same-box A/B of variants/<name>/ snapshots, interleaved ABAB (ROUNDS times).
set -o pipefail
mkdir -p gpurun_out
ARGS=${ARGS:-}
for r in $(seq 1 ${ROUNDS:-2}); do
  for v in $ABV; do
    (cd variants/$v && timeout -k 10 300 python bench.py --steps 30 --warmup 5 $ARGS) > gpurun_out/abv_$v.log 2>&1 || { echo "variant $v failed"; tail -20 gpurun_out/abv_$v.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/abv_$v.log').read().strip().splitlines()[-1]); print('round $r [$v]', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],4), 'ms/step')"
  done
done
