#!/bin/bash
# Streamed .xfb input: pread staging (default) vs copying from the mapping
# (XFLOW_NO_PREAD=1), 64-bit and compact keys, with the H2D/step/host-stage
# timeline (XFLOW_STREAM_TIMELINE=1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp XFLOW_STREAM_TIMELINE=1
mkdir -p gpurun_out
TAG=${TAG:-xfbp}
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_reader.py > gpurun_out/${TAG}_tests.log 2>&1 || { tail -30 gpurun_out/${TAG}_tests.log; exit 1; }
tail -1 gpurun_out/${TAG}_tests.log
for mode in ${MODES:-compact wide}; do
  hs=0; [ $mode = compact ] && hs=1000000000
  for v in pread mmap pread; do
    envs=""; [ $v = mmap ] && envs="XFLOW_NO_PREAD=1"
    env $envs timeout -k 10 400 python -u scripts/xfb_bench.py --rows ${ROWS:-8388608} --epochs 4 \
        --hash-space $hs --copy-threads ${CT:-8} --dir /tmp/xfb_$mode > gpurun_out/${TAG}_${mode}_$v.log 2>&1 || { echo "$mode $v failed"; tail -20 gpurun_out/${TAG}_${mode}_$v.log; exit 1; }
    python3 - gpurun_out/${TAG}_${mode}_$v.log "$mode $v" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
tl = d.get("timeline_by_epoch", [{}])[-1]
print(sys.argv[2].ljust(14), "samples/s by epoch", [round(x / 1e6, 1) for x in d["samples_per_s_by_epoch"]],
      "last epoch: h2d %.1f ms, during steps %.1f, steps %.1f, host stage %.1f ms" % (
      tl.get("h2d_ms", 0), tl.get("h2d_during_step_ms", 0), tl.get("step_busy_ms", 0), tl.get("host_stage_ms", 0)))
PY
  done
done
