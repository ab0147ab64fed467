#!/bin/bash
# rocprofv3 kernel stats of bench.py variants (MODELS: '|'-separated flags),
# top kernels printed per variant; the summaries stay under gpurun_out/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-prof}
mkdir -p gpurun_out
MODELS=${MODELS:-"--model lr"}
IFS='|' read -ra MLIST <<< "$MODELS"
i=0
for m in "${MLIST[@]}"; do
  i=$((i + 1))
  d=gpurun_out/${TAG}_$i
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps ${STEPS:-10} --warmup 3 $m > $d.log 2>&1 || { echo "profile $m failed"; tail -20 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/${TAG}_${i}_kernel_stats.csv
  echo "== $m"
  grep '^{' $d.log | tail -1 | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],3), 'ms/step', 'records/step', d.get('reduction_records_per_step'), 'logloss', round(d['logloss'],4))"
  python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for x in rows[:14]:
    print(f"{x['Name'][:80]:80s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:9.1f} {float(x['Percentage']):6.2f}%")
PY
  find $d -name "*kernel_trace.csv" -size +20M -delete
done
