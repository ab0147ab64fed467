#!/bin/bash
# LR producer phase timing (variants/ktime)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6t
mkdir -p $O
cd variants/ktime &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/lr.log 2>&1 && grep "ktime" $O/lr.log | tail -1
