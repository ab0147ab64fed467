#!/bin/bash
# MVM numerics (GPU) then bench: reduction path vs XFLOW_MVM_ATOMICS=1, + kernel stats.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu \
    tests/test_engine_numerics.py > gpurun_out/mvm_tests.log 2>&1 || { tail -40 gpurun_out/mvm_tests.log; exit 1; }
tail -2 gpurun_out/mvm_tests.log
for v in red atomics red_live atomics_live; do
  extra=""; case $v in *live) extra="--v-init-scale 1.0";; esac
  case $v in atomics*) export XFLOW_MVM_ATOMICS=1;; *) unset XFLOW_MVM_ATOMICS;; esac
  timeout -k 10 300 python bench.py --model mvm --v-dim 10 --steps 20 --warmup 5 $extra > gpurun_out/mvm_$v.log 2>&1 || { tail -20 gpurun_out/mvm_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/mvm_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],3), 'ms', 'logloss', round(d['logloss'],5))"
done
unset XFLOW_MVM_ATOMICS
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mvmred -o run -- python3 bench.py --model mvm --v-dim 10 --steps 10 --warmup 3 --v-init-scale 1.0 > gpurun_out/prof_mvmred.log 2>&1 || { tail -20 gpurun_out/prof_mvmred.log; exit 1; }
f=$(find gpurun_out/prof_mvmred -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f}")
PY
find gpurun_out/prof_mvmred -name "*kernel_trace.csv" -delete
