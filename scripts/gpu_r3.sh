#!/bin/bash
# Round-3 GPU iteration: full GPU test suite, headline bench (+ monitor A/B),
# the emulated 8-GPU step under rocprofv3.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-r3}
if [ -z "$SKIP_TESTS" ]; then
  timeout -k 10 900 python -u -m pytest tests -x -v -m gpu --timeout 300 --timeout-method thread \
      > gpurun_out/${TAG}_pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -60 gpurun_out/${TAG}_pytest_gpu.log; exit 1; }
  tail -3 gpurun_out/${TAG}_pytest_gpu.log
fi
for i in 1 2; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_$i.log 2>&1 || { echo "bench failed"; tail -30 gpurun_out/${TAG}_bench_$i.log; exit 1; }
  grep metric gpurun_out/${TAG}_bench_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench', d['value']/1e6, d['ms_per_step'])"
  XFLOW_NO_MONITOR=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_nomon_$i.log 2>&1 || { echo "bench failed"; exit 1; }
  grep metric gpurun_out/${TAG}_bench_nomon_$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('bench nomon', d['value']/1e6, d['ms_per_step'])"
done
[ -n "$SKIP_W8" ] && exit 0
timeout -k 10 600 python tools/w8_emulate.py --out gpurun_out/${TAG}_w8.json > gpurun_out/${TAG}_w8.log 2>&1 || { echo "w8 failed"; tail -30 gpurun_out/${TAG}_w8.log; exit 1; }
cat gpurun_out/${TAG}_w8.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/${TAG}_w8prof -o run -- python3 tools/w8_emulate.py > gpurun_out/${TAG}_w8prof.log 2>&1 || { echo "w8 profile failed"; tail -30 gpurun_out/${TAG}_w8prof.log; exit 1; }
f=$(find gpurun_out/${TAG}_w8prof -name "*kernel_stats.csv" | head -1)
cp "$f" gpurun_out/${TAG}_w8_kernel_stats.csv
find gpurun_out/${TAG}_w8prof -name "*kernel_trace.csv" -size +20M -delete
python3 - "$f" <<'PY'
import csv, sys
for x in csv.DictReader(open(sys.argv[1])):
    print(f"{x['Name'][:70]:70s} n={x['Calls']:>5} avg_us={float(x['AverageNs'])/1000:9.1f} tot_ms={float(x['TotalDurationNs'])/1e6:9.2f} {float(x['Percentage']):6.2f}%")
PY
