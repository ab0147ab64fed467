#!/bin/bash
# Round-4 second half: GPU tests of the changed paths, FM-std / LR variant
# A/Bs, native vs Python sharded step (bench --sharded, shared-GPU RCCL N=2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread ${TESTS:-tests/test_engine_numerics.py tests/test_determinism.py tests/test_many_slices.py tests/test_rccl_multiprocess.py tests/test_table_growth.py} > gpurun_out/r4b_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/r4b_tests.log; exit 1; }
tail -1 gpurun_out/r4b_tests.log
if [ -n "$ABV_FM" ]; then ARGS="--model fm --v-dim 8 --fm-math standard" ABV="$ABV_FM" bash scripts/gpu_abv.sh || exit 1; fi
if [ -n "$ABV_LR" ]; then ARGS="--model lr" ABV="$ABV_LR" bash scripts/gpu_abv.sh || exit 1; fi
for v in 0 1 0 1; do
  XFLOW_NATIVE_STEP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded > gpurun_out/r4b_sh.log 2>&1 || { echo "sharded bench failed"; tail -20 gpurun_out/r4b_sh.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/r4b_sh.log').read().strip().splitlines()[-1]); print('sharded native=$v', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],3), 'ms/step host_issue', d.get('host_issue_ms_per_step'))"
done
