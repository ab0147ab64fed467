#!/bin/bash
# N ranks sharing GPU 0 (XFLOW_SHARED_GPU=1, RCCL socket transport), each
# bench.py process under its own rocprofv3 kernel trace (no torchrun: the
# ranks get RANK / WORLD_SIZE / MASTER_* directly), then the union of the
# ranks' kernels: does the device idle (tools/trace_gaps.py)?
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp XFLOW_SHARED_GPU=1 NCCL_DEBUG=${NCCL_DEBUG:-WARN}
N=${N:-2}
TAG=${TAG:-shprof}
mkdir -p gpurun_out
pids=()
for r in $(seq 0 $((N - 1))); do
  RANK=$r LOCAL_RANK=$r WORLD_SIZE=$N LOCAL_WORLD_SIZE=$N MASTER_ADDR=127.0.0.1 MASTER_PORT=${PORT:-29733} \
    timeout -k 10 ${TLIM:-240} rocprofv3 --kernel-trace --output-format csv -d gpurun_out/${TAG}_r$r -o run -- \
    python3 bench.py --gpus $N --steps ${STEPS:-20} --warmup 3 --batch ${BATCH:-65536} --log2-cap ${LOG2CAP:-26} $ARGS \
    > gpurun_out/${TAG}_r$r.log 2>&1 &
  pids+=($!)
done
rc=0
for p in "${pids[@]}"; do wait $p || rc=$?; done
[ $rc -eq 0 ] || { echo "a rank failed rc=$rc"; tail -30 gpurun_out/${TAG}_r0.log; exit 1; }
grep '"metric"' gpurun_out/${TAG}_r0.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(round(d['value']/1e6,1),'M/s', round(d['ms_per_step'],3),'ms/step', 'host_per_rank', d.get('host_per_rank'))"
traces=$(for r in $(seq 0 $((N - 1))); do find gpurun_out/${TAG}_r$r -name "*kernel_trace.csv" | head -1; done)
python3 tools/trace_gaps.py $traces --marker k_synth --steps ${WIN:-30} --top 10 > gpurun_out/${TAG}_gaps.txt; sed -n "1p;/^window/,\$p" gpurun_out/${TAG}_gaps.txt
