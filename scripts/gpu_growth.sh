#!/bin/bash
# Segmented table growth on the GPU: growth tests, the headline bench with the
# table range on VMM (default) vs one hipMalloc (XFLOW_TABLE_VMM=0), the split
# cost per 1e8 keys, and an FM-8 table growing past half of HBM.  (The bench's
# table cannot grow -- 2^31 slots -- so it is one hipMalloc either way.)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread tests/test_table_growth.py > gpurun_out/growth_tests.log 2>&1 || { echo "growth tests failed"; tail -40 gpurun_out/growth_tests.log; exit 1; }
tail -1 gpurun_out/growth_tests.log
for v in 1 1; do
  XFLOW_TABLE_VMM=$v timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/growth_bench.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/growth_bench.log; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/growth_bench.log').read().strip().splitlines()[-1]); print('VMM=$v', round(d['value']/1e6,1), 'M samples/s', round(d['ms_per_step'],3), 'ms/step')"
done
timeout -k 10 300 python tools/table_ops_bench.py --grow-only --grow-log2 28 > gpurun_out/growth_ops.log 2>&1 || { echo "table_ops failed"; tail -20 gpurun_out/growth_ops.log; exit 1; }
tail -1 gpurun_out/growth_ops.log
timeout -k 10 400 python -u tools/table_grow_bench.py > gpurun_out/growth_hbm.log 2>&1 || { echo "grow bench failed"; tail -20 gpurun_out/growth_hbm.log; exit 1; }
grep -E '"start"|prefill_keys|summary' gpurun_out/growth_hbm.log
