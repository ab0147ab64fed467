#!/bin/bash
# round-6 final HEAD, part D: the whole GPU suite, smoke, the driver's bench twice,
# LR and standard-FM step profiles
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r6fd_head bash scripts/gpu.sh head &&
TAG=r6fd_fmprof bash scripts/gpu.sh prof "--model fm --fm-math standard"
