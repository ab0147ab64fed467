#!/bin/bash
# standard-FM record stores in 3 vector stores (st3) vs cas; phase timing
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out/r6r
(cd variants/ktime && timeout -k 10 300 python bench.py --model fm --fm-math standard --steps 20 \
    --warmup 5 > ../../gpurun_out/r6r/ktime.log 2>&1) && grep ktime gpurun_out/r6r/ktime.log | tail -1 &&
STEPS=20 TAG=r6r_fms ROUNDS=3 bash scripts/gpu.sh ab "cas st3" "--model fm --fm-math standard" &&
STEPS=20 TAG=r6r_mvm ROUNDS=2 bash scripts/gpu.sh ab "cas st3" "--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9"
