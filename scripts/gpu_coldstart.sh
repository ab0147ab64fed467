#!/bin/bash
# Cold-box bench: the first GPU process of a fresh box without the warmup
# time floor, then with it (bench.py --min-warmup-s).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for cfg in "--min-warmup-s 0" "" ""; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 $cfg > gpurun_out/cold.log 2>&1 || { tail -20 gpurun_out/cold.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/cold.log').read().strip().splitlines()[-1]); print('[$cfg]', round(d['value']/1e6,1), 'M', round(d['ms_per_step'],4), 'ms warmup run', d['warmup_steps_run'])"
done
