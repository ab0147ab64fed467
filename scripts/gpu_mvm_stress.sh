#!/bin/bash
# MVM backward under load: SGD + O(1) init keeps every row's field product
# non-zero, so every occurrence emits a record every step.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in red atomics; do
  case $v in atomics*) export XFLOW_MVM_ATOMICS=1;; *) unset XFLOW_MVM_ATOMICS;; esac
  timeout -k 10 300 python bench.py --model mvm --v-dim 10 --optimizer sgd --v-init-scale 1.0 --steps 20 --warmup 5 > gpurun_out/mvms_$v.log 2>&1 || { tail -20 gpurun_out/mvms_$v.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/mvms_$v.log').read().strip().splitlines()[-1]); print('$v', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],3), 'ms', 'logloss', round(d['logloss'],5))"
done
unset XFLOW_MVM_ATOMICS
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_mvms -o run -- python3 bench.py --model mvm --v-dim 10 --optimizer sgd --v-init-scale 1.0 --steps 10 --warmup 3 > gpurun_out/prof_mvms.log 2>&1 || { tail -20 gpurun_out/prof_mvms.log; exit 1; }
f=$(find gpurun_out/prof_mvms -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f} min_us={float(x['MinNs'])/1000:9.1f} max_us={float(x['MaxNs'])/1000:9.1f}")
PY
find gpurun_out/prof_mvms -name "*kernel_trace.csv" -size +20M -delete
