#!/bin/bash
# round-6 final, part C (HEAD incl. the one-CAS inserts, synth precompute and the
# standard-FM tail from registers): the whole GPU suite, smoke, the tail A/B,
# the headline twice, the model table
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=r6fc_head bash scripts/gpu.sh tests && TAG=r6fc_head bash scripts/gpu.sh smoke &&
STEPS=20 TAG=r6fc_fms ROUNDS=3 bash scripts/gpu.sh ab "base tailr" "--model fm --fm-math standard" &&
TAG=r6fc_head bash scripts/gpu.sh bench "" && TAG=r6fc_head2 bash scripts/gpu.sh bench "" &&
TAG=r6fc_models bash scripts/models.sh
