#!/bin/bash
# Sensitivity of the 20-step bench number to warmup (clock warm-up GEMM time,
# training warmup steps) on one box.
set -o pipefail
mkdir -p gpurun_out
run() { tag=$1; shift; timeout -k 10 300 python bench.py "$@" > gpurun_out/warm_$tag.log 2>&1 || { echo "$tag failed"; tail -5 gpurun_out/warm_$tag.log; exit 1; }; python3 -c "import json; d=json.loads(open('gpurun_out/warm_$tag.log').read().strip().splitlines()[-1]); print('$tag', round(d['value']/1e6,1), 'M', round(d['ms_per_step'],4), 'ms')"; }
for r in 1 2; do
run cw0 --steps 20 --warmup 5 --clock-warmup-s 0
run cw025 --steps 20 --warmup 5
run cw1 --steps 20 --warmup 5 --clock-warmup-s 1.0
run w50 --steps 20 --warmup 50
run s200 --steps 200 --warmup 5
done
