#!/bin/bash
# standard-FM producer phase timing (variants/ktime, XFLOW_KTIMING=1 build)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6q
mkdir -p $O
cd variants/ktime &&
timeout -k 10 300 python bench.py --model fm --fm-math standard --steps 20 --warmup 5 > $O/s1.log 2>&1 &&
grep "ktime" $O/s1.log | tail -1
