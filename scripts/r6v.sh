#!/bin/bash
# read-first insert (rf: read the tag, CAS only a free slot) vs CAS-first (base)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
STEPS=20 TAG=r6v_lr ROUNDS=3 bash scripts/gpu.sh ab "base rf" "" &&
STEPS=20 TAG=r6v_fm ROUNDS=2 bash scripts/gpu.sh ab "base rf" "--model fm" &&
STEPS=20 TAG=r6v_fms ROUNDS=2 bash scripts/gpu.sh ab "base rf" "--model fm --fm-math standard" &&
STEPS=20 TAG=r6v_mvm ROUNDS=2 bash scripts/gpu.sh ab "base rf" "--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9"
