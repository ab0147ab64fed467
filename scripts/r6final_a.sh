#!/bin/bash
# round-6 final, part A: the whole GPU suite, smoke, two headline benches, the LR
# step profile, the standard-FM step profile
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r6f_head bash scripts/gpu.sh head &&
TAG=r6f_fmprof bash scripts/gpu.sh prof "--model fm --fm-math standard"
