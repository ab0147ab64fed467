#!/bin/bash
# Same-box A/B of an environment switch: ROUNDS x (A, B) bench runs of ARGS,
# then (PROF=1) kernel stats of each.  ENVA / ENVB: "NAME=1" or empty.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ab}
for r in $(seq 1 ${ROUNDS:-3}); do
  for v in A B; do
    if [ $v = A ]; then E="$ENVA"; else E="$ENVB"; fi
    env $E timeout -k 10 300 python bench.py --steps ${STEPS:-40} --warmup 5 $ARGS > gpurun_out/${TAG}_$v.log 2>&1 || { echo "bench $v failed"; tail -20 gpurun_out/${TAG}_$v.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/${TAG}_$v.log').read().strip().splitlines()[-1]); print('$v [$E]', round(d['value']/1e6,1), 'M/s', round(d['ms_per_step'],4), 'ms', 'issue', round(d.get('host_issue_ms_per_step',0),3))"
  done
done
if [ -n "$PROF" ]; then
  for v in A B; do
    if [ $v = A ]; then E="$ENVA"; else E="$ENVB"; fi
    d=gpurun_out/${TAG}_prof_$v
    if [ -n "$E" ]; then export $E; fi
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 10 --warmup 3 $ARGS > $d.log 2>&1 || { echo "prof $v failed"; tail -5 $d.log; exit 1; }
    if [ -n "$E" ]; then unset ${E%%=*}; fi
    f=$(find $d -name "*kernel_stats.csv" | head -1); cp $f gpurun_out/${TAG}_${v}_kernel_stats.csv
    echo "== $v [$E]"
    python3 - "$f" <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[2:16]:
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:8.1f}")
PY
    find $d -name "*kernel_trace.csv" -delete
  done
fi
