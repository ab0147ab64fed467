#!/bin/bash
# Config 4 rehearsal on a 1-GPU box: N ranks share GPU 0 (XFLOW_SHARED_GPU=1).
# The async parameter server (bench.py --async: HIP-IPC windows, no RCCL)
# with and without a straggler (XFLOW_FAULT=slow_rank:<N-1>:<ms>), then the
# lock-step sharded step (RCCL over sockets) the same two ways.  One summary
# line per run: each rank's steps/s, max staleness, max lead.
#   bash scripts/async_rehearsal.sh [N] [SLOW_MS] [extra bench args]
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp XFLOW_SHARED_GPU=1
N=${1:-4}
SLOW=${2:-20}
shift 2 2>/dev/null
EXTRA="$*"
O=gpurun_out/${TAG:-async_rehearsal}
mkdir -p "$O"
ARGS="--gpus $N --steps ${STEPS:-30} --warmup 3 --batch ${BATCH:-65536} --log2-cap ${LOG2CAP:-26} --clock-warmup-s 0 $EXTRA"

show() {
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
pr = d.get("per_rank")
line = f"{sys.argv[2]:34s} {d['value']/1e6:8.2f} M samples/s  {d['ms_per_step']:.3f} ms/step"
if pr:
    line += "  per-rank steps/s " + " ".join(f"{r['steps_per_s']:.1f}" for r in pr)
    line += f"  max_staleness {d['max_staleness']} (bound {d['staleness_bound']})"
    line += "  max_lead " + " ".join(str(r["max_lead"]) for r in pr)
    line += f"  bytes/step {d['bytes_moved_per_step']}"
else:
    line += f"  bytes/step {d.get('bytes_moved_per_step')}"
print(line)
PY
}

run() {  # tag, fault, mode args
  local log=$O/$1.log port=$((29700 + RANDOM % 200))
  XFLOW_FAULT="$2" timeout -k 10 ${TLIM:-300} python -m torch.distributed.run --nnodes=1 \
      --nproc-per-node $N --master-addr 127.0.0.1 --master-port $port bench.py $ARGS $3 \
      > "$log" 2>&1 || { echo "run $1 failed"; tail -30 "$log"; exit 1; }
  show "$log" "$1"
}

run async_unslowed "" "--async" &&
run async_slow_rank$((N - 1)) "slow_rank:$((N - 1)):$SLOW" "--async" &&
run lockstep_unslowed "" "" &&
run lockstep_slow_rank$((N - 1)) "slow_rank:$((N - 1)):$SLOW" ""
