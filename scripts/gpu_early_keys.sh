#!/bin/bash
# Early key exchange (next batch's keys ride with the gradients: 2 group
# calls per multi-rank step): GPU tests of the multi-rank paths, then the
# shared-GPU RCCL rehearsal (N processes on GPU 0) and the emulated W=8 step
# with XFLOW_EARLY_KEYS=1 (default) vs 0.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-ek}
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests/test_gpu_paths.py tests/test_w8_loopback.py tests/test_rccl_multiprocess.py > gpurun_out/${TAG}_tests.log 2>&1 || { echo "tests failed"; tail -40 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for rep in 1 2; do
  for ek in 1 0; do
    XFLOW_EARLY_KEYS=$ek TAG=${TAG}_ek${ek}_r$rep NS="2 4" bash scripts/gpu_shared_rccl.sh 2>&1 | grep -v '^{' | sed "s/^/early=$ek rep=$rep /" || exit 1
  done
done
for ek in 1 0; do
  XFLOW_EARLY_KEYS=$ek timeout -k 10 300 python tools/w8_emulate.py > gpurun_out/${TAG}_w8_ek$ek.log 2>&1 || { echo "w8 failed"; tail -20 gpurun_out/${TAG}_w8_ek$ek.log; exit 1; }
  echo "w8 early=$ek $(grep -o '"ms_per_rank_step": [0-9.]*' gpurun_out/${TAG}_w8_ek$ek.log)"
done
