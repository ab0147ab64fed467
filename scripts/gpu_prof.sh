#!/bin/bash
# rocprofv3 kernel stats of one bench configuration: TAG, BENCH_ARGS.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-prof}
mkdir -p $O
timeout -k 10 300 python bench.py $BENCH_ARGS > $O/bench.log 2>&1 || { echo "bench failed"; tail -20 $O/bench.log; exit 1; }
python3 -c "import json; d=json.loads([l for l in open('$O/bench.log') if l.startswith('{')][-1]); print('$TAG', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],4), 'ms/step load', round(d['table_load'],3))"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p -o run -- python3 bench.py $BENCH_ARGS > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
f=$(find $O/p -name "*kernel_stats.csv" | head -1)
cp "$f" $O/kernel_stats.csv
python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    if float(x['Percentage']) < 0.3: continue
    print(f"{x['Name'][:64]:64s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f} {float(x['Percentage']):6.2f}%")
PY
rm -rf $O/p
