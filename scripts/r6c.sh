set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6c; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_rccl_multiprocess.py -k csr -x -v --timeout 200 --timeout-method thread > $O/csr_rccl.log 2>&1; rc=$?; tail -12 $O/csr_rccl.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_bench_contract.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/bench_contract.log 2>&1; rc=$?; tail -14 $O/bench_contract.log; [ $rc -eq 0 ] || exit $rc
TAG=r6c_reh TLIM=240 bash scripts/async_rehearsal.sh 4 20 --slices 64
