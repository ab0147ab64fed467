#!/bin/bash
# LR-FTRL bench at increasing table occupancy (bench.py --table-load): the
# prefilled keys are never touched by the batches, like the keys a long run
# has accumulated.  Then rocprofv3 kernel stats of the LOAD_PROF load.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-occ}
mkdir -p $O
for load in ${LOADS:-0 0.35 0.47 0.6}; do
  timeout -k 10 300 python bench.py --steps ${STEPS:-100} --warmup 5 --table-load $load $EXTRA > $O/bench_$load.log 2>&1 || { echo "bench $load failed"; tail -20 $O/bench_$load.log; exit 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('$O/bench_$load.log') if l.startswith('{')][-1]); print('load', $load, 'Msamples/s %.1f' % (d['value']/1e6), 'ms/step %.4f' % d['ms_per_step'], 'table_load %.3f' % d['table_load'], 'logloss %.4f' % d['logloss'])"
done
if [ -n "$LOAD_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 50 --warmup 5 --table-load $LOAD_PROF $EXTRA > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
  f=$(find $O/prof -name "*kernel_stats.csv" | head -1)
  python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f} {float(x['Percentage']):6.2f}%")
PY
  find $O/prof -name "*kernel_trace.csv" -delete
fi
