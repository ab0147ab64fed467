#!/bin/bash
# Round-end check, as the driver runs it: every GPU test, smoke(), then the
# driver's bench command (N = 1) twice, and a kernel-stats profile of it.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests > gpurun_out/final_tests.log 2>&1 || { echo "GPU tests failed"; tail -40 gpurun_out/final_tests.log; exit 1; }
tail -1 gpurun_out/final_tests.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/final_smoke.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
for k in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/final_bench.log; exit 1; }
  tail -1 gpurun_out/final_bench.log | cut -c1-220
done
if [ -z "$SKIP_PROF" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/final_prof -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final_prof.log 2>&1 || { echo "profile failed"; tail -20 gpurun_out/final_prof.log; exit 1; }
  f=$(find gpurun_out/final_prof -name "*kernel_stats.csv" | head -1)
  cp "$f" gpurun_out/final_lr_kernel_stats.csv
  find gpurun_out/final_prof -name "*kernel_trace.csv" -size +20M -delete
  tail -1 gpurun_out/final_prof.log | cut -c1-160
fi
