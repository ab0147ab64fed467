#!/bin/bash
# Streamed compact .xfb: host staging threads 8 vs 16 (the box's CPU share),
# interleaved, with the H2D/step/host-stage timeline.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp XFLOW_STREAM_TIMELINE=1
mkdir -p gpurun_out
TAG=${TAG:-xfbt}
for rep in 1 2; do
  for ct in 8 16; do
    timeout -k 10 400 python -u scripts/xfb_bench.py --rows 8388608 --epochs 4 --hash-space 1000000000 \
        --copy-threads $ct --dir /tmp/xfb_compact > gpurun_out/${TAG}_ct$ct.log 2>&1 || { echo "ct $ct failed"; tail -20 gpurun_out/${TAG}_ct$ct.log; exit 1; }
    python3 - gpurun_out/${TAG}_ct$ct.log "ct=$ct rep=$rep" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
tl = d.get("timeline_by_epoch", [{}])[-1]
print(sys.argv[2].ljust(12), "samples/s by epoch", [round(x / 1e6, 1) for x in d["samples_per_s_by_epoch"]],
      "last epoch: h2d %.1f ms, steps %.1f, host stage %.1f ms" % (
      tl.get("h2d_ms", 0), tl.get("step_busy_ms", 0), tl.get("host_stage_ms", 0)))
PY
  done
done
