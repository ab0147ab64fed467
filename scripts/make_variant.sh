#!/bin/bash
# Snapshot the current in-tree build as variants/<name>/ (bench.py + the
# xflow_amd package with its built extension) for same-box A/B runs:
#   bash scripts/make_variant.sh base; <edit, rebuild>; bash scripts/make_variant.sh new
#   gpurun -- 'ABV="base new" bash scripts/gpu_abv.sh'
set -e
cd "$(dirname "$0")/.."
n=${1:?variant name}
rm -rf variants/$n
mkdir -p variants/$n
cp bench.py variants/$n/
cp -r xflow_amd variants/$n/ && rm -rf variants/$n/xflow_amd/__pycache__ variants/$n/xflow_amd/*/__pycache__
echo "variants/$n: $(ls variants/$n/xflow_amd/*.so)"
