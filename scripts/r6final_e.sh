#!/bin/bash
# round-6 final HEAD, part E: the model table, the config-4 rehearsal, the
# shared-GPU lock-step RCCL step at 2 and 4 ranks
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r6fe_models bash scripts/models.sh &&
TAG=r6fe_async bash scripts/async_rehearsal.sh 4 20 --slices 64 &&
TAG=r6fe_shared bash scripts/gpu.sh shared "2 4" ""
