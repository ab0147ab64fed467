#!/bin/bash
# Reference compat (scripts/start_worker.sh): start this machine's workers.
# usage: start_worker.sh <first_rank> <num_local_workers> <world_size> <bin> [args..]
# Needs DMLC_PS_ROOT_URI / DMLC_PS_ROOT_PORT of the rendezvous (worker rank 0).
first=$1; n=$2; world=$3; shift 3
bin=$1; shift
ROOT=$(cd "$(dirname "$0")/.." && pwd)
if [ "$(basename "$bin")" = "xflow_lr" ] && [ "$world" -gt 1 ]; then bin="python3 -m xflow_amd.cli"; fi
export PYTHONPATH=$ROOT:$PYTHONPATH
export MASTER_ADDR=${DMLC_PS_ROOT_URI:-127.0.0.1} MASTER_PORT=${DMLC_PS_ROOT_PORT:-8000}
export WORLD_SIZE=$world DMLC_NUM_WORKER=$world
for ((i=0; i<n; ++i)); do
    r=$((first + i))
    DMLC_ROLE=worker DMLC_WORKER_ID=$r RANK=$r LOCAL_RANK=$i XFLOW_DEVICE=$i $bin "$@" &
done
wait
