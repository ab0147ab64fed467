#!/bin/bash
# One GPU round trip: GPU tests, smoke, fused + sharded 1-GPU bench, kernel
# trace of the sharded step with launch-gap analysis.  TAG names the outputs.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-round}
O=gpurun_out/$TAG
mkdir -p $O
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 600 python -u -m pytest tests -x -v -m gpu --timeout 120 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest gpu failed rc=$?"; tail -60 $O/pytest_gpu.log; exit 1; }
  tail -2 $O/pytest_gpu.log
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
  cat $O/smoke.log
fi
timeout -k 10 300 python bench.py ${BENCH_ARGS:-} > $O/bench_fused.log 2>&1 || { echo "bench failed"; tail -30 $O/bench_fused.log; exit 1; }
grep metric $O/bench_fused.log | cut -c1-400
timeout -k 10 300 python bench.py --sharded ${BENCH_ARGS:-} > $O/bench_sharded.log 2>&1 || { echo "sharded bench failed"; tail -30 $O/bench_sharded.log; exit 1; }
grep metric $O/bench_sharded.log | cut -c1-400
if [ -z "$SKIP_GAPS" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $O/gaps -o run -- python3 bench.py --steps 20 --warmup 3 --sharded > $O/gaps.log 2>&1 || { echo "gaps failed"; tail -20 $O/gaps.log; exit 1; }
  f=$(find $O/gaps -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_gaps.py "$f" --marker k_synth --steps 18 > $O/gaps_sharded.txt && head -40 $O/gaps_sharded.txt
  find $O/gaps -name "*kernel_trace.csv" -size +20M -delete
fi
