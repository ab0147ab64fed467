#!/bin/bash
# Round-3 session-3 GPU iteration: GPU tests + smoke, fused-apply A/B on the
# headline bench, the model benches, the emulated 8-GPU owner-path A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3s3}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 700 python -u -m pytest tests -x -v -m gpu --timeout 200 --timeout-method thread \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -60 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -2 gpurun_out/${TAG}_pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${TAG}_smoke.log 2>&1 || { echo "smoke failed"; cat gpurun_out/${TAG}_smoke.log; exit 1; }
  tail -3 gpurun_out/${TAG}_smoke.log
fi
if [ -z "$SKIP_AB" ]; then
  TAG=${TAG}_ab ENVB="${ENVB:-XFLOW_LR_SEPARATE_APPLY=1}" CONFIGS="${AB_CONFIGS:-lr}" REPS=${REPS:-3} bash scripts/gpu_ab_env.sh || exit 1
fi
if [ -z "$SKIP_MODELS" ]; then
  TAG=${TAG} SKIP_TESTS=1 SKIP_PROF=1 bash scripts/gpu_models.sh || exit 1
fi
if [ -z "$SKIP_W8" ]; then
  TAG=${TAG}_w8 bash scripts/gpu_w8_ab.sh || exit 1
fi
