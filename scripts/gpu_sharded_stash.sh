set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -x -q -m gpu --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest gpu failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
for i in 1 2; do
timeout -k 10 200 python bench.py --steps 30 --warmup 5 --sharded > gpurun_out/bs.log 2>&1 || { tail -20 gpurun_out/bs.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bs.log').read().strip().splitlines()[-1]); print('sharded', round(d['value']/1e6,1), d['ms_per_step'])"
XFLOW_LR_SLOT_GRADS=1 timeout -k 10 200 python bench.py --steps 30 --warmup 5 --sharded > gpurun_out/bs0.log 2>&1 || { tail -20 gpurun_out/bs0.log; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/bs0.log').read().strip().splitlines()[-1]); print('sharded-nostash', round(d['value']/1e6,1), d['ms_per_step'])"
done
