#!/bin/bash
# per-phase cycle counters of the standard-FM producer (diagnostic build,
# variants/ktime = XFLOW_KTIMING=1); 1 and 64 slices
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=$PWD/gpurun_out/r6o
mkdir -p $O
cd variants/ktime &&
timeout -k 10 300 python bench.py --model fm --fm-math standard --steps 20 --warmup 5 > $O/s1.log 2>&1 &&
grep "ktime\|samples" $O/s1.log | tail -3 &&
timeout -k 10 300 python bench.py --model fm --fm-math standard --steps 20 --warmup 5 --slices 64 > $O/s64.log 2>&1 &&
grep "ktime" $O/s64.log | tail -2
