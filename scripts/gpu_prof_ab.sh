#!/bin/bash
# Kernel stats of one bench configuration under two env settings (same box):
#   ENVB="XFLOW_PULL_SPLIT=1" CONFIG="fm --v-dim 8" TAG=x bash scripts/gpu_prof_ab.sh
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-profab}
mkdir -p gpurun_out
for v in A B; do
  if [ $v = B ]; then envs="$ENVB"; else envs="$ENVA"; fi
  d=gpurun_out/prof_${TAG}_$v
  env $envs timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 bench.py --steps 10 --warmup 3 --model ${CONFIG:-lr} > $d.log 2>&1 || { echo "profile $v failed"; tail -20 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  echo "== $v ($envs) ${CONFIG:-lr}"
  python3 - "$f" <<'PY'
import csv, sys
rows = [x for x in csv.DictReader(open(sys.argv[1])) if int(x['Calls']) >= 10]
for x in rows[:14]:
    print(f"{x['Name'][:64]:64s} n={x['Calls']:>4} avg_us={float(x['AverageNs'])/1000:8.1f}")
PY
  find $d -name "*kernel_trace.csv" -size +20M -delete
done
