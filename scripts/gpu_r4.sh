#!/bin/bash
# Round-4 GPU check: selected GPU tests (TESTS), then bench of each model
# variant (MODELS, '|'-separated bench.py flags).  SKIP_TESTS=1 skips pytest.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r4}
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  TESTS=${TESTS:-tests}
  timeout -k 10 ${TEST_TIMEOUT:-600} python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread $TESTS > gpurun_out/pytest_$TAG.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -60 gpurun_out/pytest_$TAG.log; exit 1; }
  tail -2 gpurun_out/pytest_$TAG.log
fi
MODELS=${MODELS:-"lr"}
IFS='|' read -ra MLIST <<< "$MODELS"
for m in "${MLIST[@]}"; do
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 $m > gpurun_out/bench_$TAG.log 2>&1 || { echo "bench $m failed"; tail -20 gpurun_out/bench_$TAG.log; exit 1; }
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/bench_$TAG.log').read().strip().splitlines()[-1]); print('$m |', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],3), 'ms/step logloss', round(d.get('logloss',0),4))"
done
