#!/bin/bash
# Multi-node / multi-GPU recipe (the reference's run_ps_dist.sh is prose).
#
# One node, N GPUs (one worker rank per GPU; the table is sharded over the
# GPUs' HBM and Pull/Push are RCCL all-to-alls over xGMI):
#   python3 -m torch.distributed.run --nnodes=1 --nproc-per-node N \
#       --master-addr 127.0.0.1 --master-port 29500 \
#       -m xflow_amd.cli <train_prefix> <test_prefix> <model> <epochs> [flags]
#
# Several nodes: run the same command on every node with --nnodes M,
# --node-rank i and --master-addr <node 0 address>.  Worker r reads
# <train_prefix>-%05d with its global rank r.
#
# Reference-style per-role scripts are kept in scripts/start_{scheduler,server,worker}.sh.
set -e
N=${1:-$(python3 -c "import torch;print(max(1,torch.cuda.device_count()))")}
shift || true
exec python3 -m torch.distributed.run --nnodes=1 --nproc-per-node "$N" \
    --master-addr 127.0.0.1 --master-port ${MASTER_PORT:-29500} -m xflow_amd.cli "$@"
