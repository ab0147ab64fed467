#!/bin/bash
# scan A/B at 256 slices (XFLOW_SCAN_ONE=0: the three-launch scan) + kernel
# stats of both, then the headline LR bench twice.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6i
mkdir -p $O
sum() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:32s} {d['value']/1e6:8.1f} M samples/s {d['ms_per_step']:.4f} ms/step")
PY
}
ab() {  # tag env
  env $2 timeout -k 10 300 python bench.py --steps 30 --warmup 5 --slices 256 > $O/$1.log 2>&1 &&
    sum $O/$1.log "$1"
}
for r in 1 2 3; do
  ab "s256_scan_one_r$r" "XFLOW_SCAN_ONE=1" && ab "s256_scan3_r$r" "XFLOW_SCAN_ONE=0" || exit 1
done
for v in 1 0; do
  XFLOW_SCAN_ONE=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv \
      -d $O/prof$v -o run -- python3 bench.py --steps 20 --warmup 5 --slices 256 > $O/prof$v.log 2>&1 || exit 1
  f=$(find $O/prof$v -name "*kernel_stats.csv" | head -1)
  cp "$f" $O/kernel_stats_scan$v.csv
  find $O/prof$v -name "*kernel_trace.csv" -size +20M -delete
done
timeout -k 10 300 python bench.py > $O/head1.log 2>&1 && sum $O/head1.log head1 &&
timeout -k 10 300 python bench.py > $O/head2.log 2>&1 && sum $O/head2.log head2
