#!/bin/bash
# Capacity-monitor cost A/B on the headline bench (same box, interleaved).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${TAG:-monab}
timeout -k 10 300 python -u -m pytest tests/test_table_growth.py -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/${TAG}_pytest.log 2>&1 || { echo "growth tests failed"; tail -40 gpurun_out/${TAG}_pytest.log; exit 1; }
tail -1 gpurun_out/${TAG}_pytest.log
show() { grep metric "$1" | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('$2', round(d['value']/1e6,1), round(d['ms_per_step'],4))"; }
for i in 1 2 3; do
  for v in "lag2:" "lag7:--monitor-lag 7" "nomon:" ; do
    name=${v%%:*}; args=${v#*:}
    if [ "$name" = nomon ]; then export XFLOW_NO_MONITOR=1; else unset XFLOW_NO_MONITOR; fi
    timeout -k 10 300 python bench.py --steps 20 --warmup 5 $args > gpurun_out/${TAG}_${name}_$i.log 2>&1 || { echo "bench $name failed"; tail -20 gpurun_out/${TAG}_${name}_$i.log; exit 1; }
    show gpurun_out/${TAG}_${name}_$i.log "$name"
  done
done
