#!/bin/bash
# Reference compat (scripts/start_scheduler.sh): the scheduler role only
# provides the rendezvous address.  torch.distributed's TCPStore lives in
# worker rank 0, so this script just exports the address for the workers.
# usage: start_scheduler.sh <bin> [args..]
export DMLC_PS_ROOT_URI=${DMLC_PS_ROOT_URI:-$(hostname -I 2>/dev/null | awk '{print $1}')}
export DMLC_PS_ROOT_PORT=${DMLC_PS_ROOT_PORT:-8000}
echo "rendezvous: $DMLC_PS_ROOT_URI:$DMLC_PS_ROOT_PORT (workers use it as MASTER_ADDR/PORT)"
DMLC_ROLE=scheduler "$@"
