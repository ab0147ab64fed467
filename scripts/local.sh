#!/bin/bash
# Local multi-process launcher, argument compatible with the reference's
# scripts/local.sh (ps-lite): local.sh <num_servers> <num_workers> <bin> [args..]
#
# The reference starts 1 scheduler + N servers + M workers of one binary with
# DMLC_ROLE set.  Here every worker rank owns a shard of the HBM parameter
# table, so servers/scheduler have no work: they are started for fidelity with
# DMLC_ROLE set and exit immediately.  The M workers get torchrun-style env
# (RANK/WORLD_SIZE/LOCAL_RANK/MASTER_ADDR/MASTER_PORT) and DMLC_* equivalents;
# worker r uses GPU r (round robin) or the CPU backend when no GPU exists.
# The native single-rank binary (build/bin/xflow_lr) is swapped for the
# Python launcher when more than one worker is requested.
if [ $# -lt 3 ]; then
    echo "usage: $0 num_servers num_workers bin [args..]"
    exit 255
fi
ROOT=$(cd "$(dirname "$0")/.." && pwd)
export DMLC_NUM_SERVER=$1; shift
export DMLC_NUM_WORKER=$1; shift
bin=$1; shift
arg="$@"
if [ "$(basename "$bin")" = "xflow_lr" ] && [ "$DMLC_NUM_WORKER" -gt 1 ]; then
    bin="python3 -m xflow_amd.cli"
fi
export PYTHONPATH=$ROOT:$PYTHONPATH
export DMLC_PS_ROOT_URI=${DMLC_PS_ROOT_URI:-127.0.0.1}
export DMLC_PS_ROOT_PORT=${DMLC_PS_ROOT_PORT:-$((20000 + RANDOM % 20000))}
export MASTER_ADDR=$DMLC_PS_ROOT_URI
export MASTER_PORT=$DMLC_PS_ROOT_PORT
export WORLD_SIZE=$DMLC_NUM_WORKER

# every started process is recorded here; scripts/stop.sh kills exactly these
pidfile=${XFLOW_PIDFILE:-/tmp/xflow_workers.$(id -u).pid}
: > "$pidfile"
DMLC_ROLE=scheduler ${bin} ${arg} &
echo $! >> "$pidfile"
for ((i=0; i<${DMLC_NUM_SERVER}; ++i)); do
    DMLC_ROLE=server ${bin} ${arg} &
    echo $! >> "$pidfile"
done
pids=()
for ((i=0; i<${DMLC_NUM_WORKER}; ++i)); do
    DMLC_ROLE=worker DMLC_WORKER_ID=$i RANK=$i LOCAL_RANK=$i XFLOW_DEVICE=$i ${bin} ${arg} &
    pids+=($!)
    echo $! >> "$pidfile"
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
wait
rm -f "$pidfile"
exit $rc
