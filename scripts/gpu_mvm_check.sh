#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -s -m gpu -k "mvm" tests/test_kernels_misc.py tests/test_engine_numerics.py > gpurun_out/mvmc_red.log 2>&1; r1=$?
tail -30 gpurun_out/mvmc_red.log
[ $r1 -le 1 ] || exit $r1
XFLOW_MVM_ATOMICS=1 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -s -m gpu -k "mvm" tests/test_kernels_misc.py tests/test_engine_numerics.py > gpurun_out/mvmc_atom.log 2>&1; r2=$?
tail -30 gpurun_out/mvmc_atom.log
exit $(( r1 > r2 ? r1 : r2 ))
