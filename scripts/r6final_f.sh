#!/bin/bash
# the driver's headline command four times on one box (its run-to-run spread)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r6ff_1 bash scripts/gpu.sh bench "" && TAG=r6ff_2 bash scripts/gpu.sh bench "" &&
TAG=r6ff_3 bash scripts/gpu.sh bench "" && TAG=r6ff_4 bash scripts/gpu.sh bench ""
