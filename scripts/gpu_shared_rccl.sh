#!/bin/bash
# Multi-process RCCL rehearsal on a 1-GPU box: N ranks share GPU 0
# (XFLOW_SHARED_GPU=1: per-rank NCCL_HOSTID, socket transport on lo).
# Correctness of the multi-rank bench / trainer path over real RCCL between
# processes; the numbers are not scaling measurements.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp XFLOW_SHARED_GPU=1 NCCL_DEBUG=${NCCL_DEBUG:-WARN}
mkdir -p gpurun_out
TAG=${TAG:-shared}
IFS='|' read -ra XL <<< "${EXTRAS:-}"
[ ${#XL[@]} -eq 0 ] && XL=("")
for n in ${NS:-2}; do
  for extra in "${XL[@]}"; do
    log=gpurun_out/${TAG}_n${n}$(echo "$extra" | tr -d ' -').log
    timeout -k 10 ${TLIM:-240} python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
        --master-addr 127.0.0.1 --master-port $((29611 + n)) bench.py --gpus $n \
        --steps ${STEPS:-5} --warmup 2 --batch ${BATCH:-65536} --log2-cap ${LOG2CAP:-26} $extra \
        > $log 2>&1 || { echo "shared-GPU bench n=$n '$extra' failed"; tail -40 $log; exit 1; }
    grep '"metric"' $log | cut -c1-200
    grep -o '"a2a_transport": "[a-z]*"\|"logloss": [0-9.]*\|"host_waits": [0-9]*\|"mid_step_waits": [0-9]*\|"host_per_rank": [^}]*\]\]\|"shared_gpu_rehearsal": true' $log | tr '\n' ' '; echo
  done
done
