#!/bin/bash
# Host-side AddressSanitizer + UBSan run of the native trainer (CPU backend)
# over every model family, quirk mode and the reference-compat loaders.
# GPU sanitizers / xnack are not available on the MI355X pool; device code is
# covered by the kernel-vs-reference numerics tests instead.
set -e
ROOT=$(cd "$(dirname "$0")/.." && pwd)
B=${XFLOW_SAN_BUILD:-$ROOT/build/asan}
cmake -S "$ROOT" -B "$B" -DCMAKE_HIP_COMPILER=${ROCM_PATH:-/opt/rocm}/llvm/bin/clang++ \
      -DCMAKE_PREFIX_PATH=${ROCM_PATH:-/opt/rocm} -DXFLOW_HOST_SANITIZE=ON \
      -DCMAKE_BUILD_TYPE=RelWithDebInfo > "$B.cmake.log" 2>&1
cmake --build "$B" -j 8 --target xflow_lr > "$B.build.log" 2>&1
export ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1
export HIP_VISIBLE_DEVICES=
W=$(mktemp -d)
cd "$W"
D=$ROOT/data
for args in "0 3 --threads 8" "0 2 --threads 8 --serial-slices --sgd" "1 2 --threads 8" \
            "1 2 --threads 4 --fm-standard --keep-remainder" "2 2 --threads 8" \
            "2 2 --threads 8 --mvm-fixed --mvm-predict-compat" "0 1 --threads 3 --save $W/t.xftb"; do
  "$B/xflow_lr" "$D/small_train" "$D/small_test" $args > out.log 2>&1 || { cat out.log; exit 1; }
  grep -q "train end" out.log
done
"$B/xflow_lr" "$D/small_train" "$D/small_test" 0 0 --threads 3 --load "$W/t.xftb" > out.log 2>&1
echo "sanitize_host: clean"
rm -rf "$W"
