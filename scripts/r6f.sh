set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6f; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_determinism.py tests/test_csr_slices.py tests/test_plan_paths.py tests/test_engine_numerics.py tests/test_gpu_paths.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/t.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $O/t.log | tail -60; [ $rc -eq 0 ] || { tail -80 $O/t.log; exit $rc; }
TAG=r6f_bench bash scripts/gpu.sh bench "--model fm --fm-math standard|--model fm --fm-math standard --slices 64|--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9|"
timeout -k 10 300 python -u -m pytest tests/test_reader.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/reader.log 2>&1; rc=$?; grep -E "PASSED|FAILED|passed|failed" $O/reader.log | tail; [ $rc -eq 0 ] || { tail -40 $O/reader.log; exit $rc; }
for fmt in v2 packed; do
  timeout -k 10 400 python scripts/xfb_bench.py --rows 8388608 --epochs 4 --data criteo --format $fmt --dir /tmp/xfb_$fmt > $O/xfb_$fmt.log 2>&1 || { tail -20 $O/xfb_$fmt.log; exit 1; }
  grep '"path"' $O/xfb_$fmt.log | cut -c1-400
done
