#!/bin/bash
# headline steadiness: the driver's command (20 steps, 5 warmup, 0.25 s clock
# warmup) against a longer clock warmup and a longer step warmup, same box
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6k
mkdir -p $O
sum() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:36s} {d['value']/1e6:8.1f} M samples/s {d['ms_per_step']:.4f} ms/step")
PY
}
i=0
for r in 1 2; do
  for a in "" "--clock-warmup-s 2" "--warmup 100" "--steps 100"; do
    i=$((i + 1))
    timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 $a > $O/b$i.log 2>&1 &&
      sum $O/b$i.log "r$r ${a:-(driver command)}" || exit 1
  done
done
