#!/bin/bash
# Device idle inside the multi-rank CSR step (ShardedStep::csr_gradients reads
# the per-owner entry totals on the host between its two group calls): two
# ranks share GPU 0, each under rocprofv3 --kernel-trace, started as separate
# processes (no launcher between the profiler and python).  Reports per rank
# the idle gaps of its stream and the one after the totals exchange.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp XFLOW_SHARED_GPU=1 MASTER_ADDR=127.0.0.1 MASTER_PORT=$((29800 + RANDOM % 100)) WORLD_SIZE=2
O=gpurun_out/${TAG:-csr_bubble}
mkdir -p "$O"
ARGS="--gpus 2 --slices ${SLICES:-64} --batch ${BATCH:-65536} --log2-cap 26 --steps 10 --warmup 3 --clock-warmup-s 0"
for r in 0 1; do
  RANK=$r LOCAL_RANK=$r timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d "$O/tr$r" -o run -- \
      python3 bench.py $ARGS > "$O/rank$r.log" 2>&1 &
done
wait -n || { echo "a rank failed"; tail -20 "$O"/rank*.log; wait; exit 1; }
wait || { echo "a rank failed"; tail -20 "$O"/rank*.log; exit 1; }
tail -1 "$O/rank0.log" | cut -c1-300
for r in 0 1; do
  python3 - "$(find "$O/tr$r" -name '*kernel_trace.csv' | head -1)" "$r" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted(((int(x["Start_Timestamp"]), int(x["End_Timestamp"]), x["Kernel_Name"]) for x in rows))
# the timed window: from the 4th-to-last-step region on -- use the last 8 ncclKernel-bracketed steps
names = [k[2] for k in ks]
t0 = ks[len(ks) // 3][0]
win = [k for k in ks if k[0] >= t0]
busy = 0; last_end = win[0][0]; idle = []
for s, e, n in win:
    if s > last_end:
        idle.append((s - last_end, prev))
    busy += max(0, e - max(s, last_end)); last_end = max(last_end, e); prev = n
    prev = n
span = win[-1][1] - win[0][0]
idle.sort(reverse=True)
nccl = [g for g in idle if "nccl" in g[1].lower()]
print(f"rank {sys.argv[2]}: window {span/1e3:.1f} us, busy {100*busy/span:.1f} %, idle {sum(g for g,_ in idle)/1e3:.1f} us "
      f"in {len(idle)} gaps; after RCCL kernels {sum(g for g,_ in nccl)/1e3:.1f} us")
for g, n in idle[:8]:
    print(f"   gap {g/1e3:8.1f} us after {n[:80]}")
PY
done
