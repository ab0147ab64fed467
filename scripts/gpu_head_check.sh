#!/bin/bash
# HEAD check on one MI355X: full GPU tests + smoke, the driver's bench
# command, and a rocprofv3 kernel-stats profile of the headline step (timed
# steps only, from the trace: tools/trace_gaps.py).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-head}
O=gpurun_out/$TAG
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; cat $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
for i in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$i.log 2>&1 || { echo "bench failed"; tail -20 $O/bench_$i.log; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/bench_$i.log').read().strip().splitlines()[-1]); print('bench', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],4), 'ms/step')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 20 --warmup 5 > $O/prof.log 2>&1 || { echo "profile failed"; tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/kernel_stats.csv
t=$(find $O/prof -name "*kernel_trace.csv" | head -1)
python3 tools/trace_gaps.py "$t" --marker k_synth --steps 18 > $O/gaps.txt && head -16 $O/gaps.txt
find $O/prof -name "*kernel_trace.csv" -size +20M -delete
