set -o pipefail
cd "${GRAFT_REPO_ROOT}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/mvm_prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 > gpurun_out/mvm_prof.log 2>&1
f=$(find gpurun_out/mvm_prof -name "*kernel_stats.csv" | head -1); cp "$f" gpurun_out/mvm_live_kernel_stats.csv
find gpurun_out/mvm_prof -name "*kernel_trace.csv" -delete
tail -1 gpurun_out/mvm_prof.log | cut -c1-200
