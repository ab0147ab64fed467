set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6b; mkdir -p $O
timeout -k 10 60 ./build/ipc_probe > $O/ipc.log 2>&1; echo "ipc rc=$?" >> $O/ipc.log; cat $O/ipc.log
timeout -k 10 400 python -u -m pytest tests/test_async_ps_gpu.py -x -v --timeout 150 --timeout-method thread > $O/aps_gpu.log 2>&1; rc=$?; tail -15 $O/aps_gpu.log; [ $rc -eq 0 ] || exit $rc
bash scripts/gpu.sh smoke && bash scripts/gpu.sh bench ""
