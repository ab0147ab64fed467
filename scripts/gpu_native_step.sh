#!/bin/bash
# Native (C++) vs Python sharded step, same box: the world-1 step (aliased
# self-exchange, and XFLOW_SELF_EXCHANGE=comm: every exchange through RCCL),
# then N ranks sharing GPU 0 over RCCL's socket transport (host cost per rank).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 400 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_rccl_multiprocess.py tests/test_gpu_paths.py > gpurun_out/native_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/native_tests.log; exit 1; }
  tail -1 gpurun_out/native_tests.log
fi
for se in alias comm; do
  for v in 0 1 0 1; do
    XFLOW_SELF_EXCHANGE=$se XFLOW_NATIVE_STEP=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 --sharded > gpurun_out/native_sh.log 2>&1 || { echo "sharded bench failed"; tail -20 gpurun_out/native_sh.log; exit 1; }
    python3 -c "import json; d=json.loads(open('gpurun_out/native_sh.log').read().strip().splitlines()[-1]); print('world1 $se native=$v', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],3), 'ms/step host_issue', round(d.get('host_issue_ms_per_step'),4), 'mid_waits', d.get('mid_step_waits'))"
  done
done
for v in 0 1; do
  XFLOW_NATIVE_STEP=$v NS="${NS:-2 4}" TAG=native$v bash scripts/gpu_shared_rccl.sh || exit 1
done
