#!/bin/bash
# Emulated 8-GPU step (tools/w8_emulate.py) of variants/<name>/ snapshots
# (scripts/make_variant.sh) under rocprofv3: per-rank device time per step
# (tools/w8_kernel_sum.py), same box.  ABV="base new" MODEL=lr REPS="1 2"
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-w8abv}
MODEL=${MODEL:-lr}
ROOT=$(pwd)
for rep in ${REPS:-1}; do
for v in $ABV; do
  d=$ROOT/gpurun_out/${TAG}_${MODEL}_${v}_$rep
  rm -rf $d
  mkdir -p variants/$v/tools && cp tools/w8_emulate.py variants/$v/tools/
  ( cd variants/$v && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 tools/w8_emulate.py --model $MODEL ${W8_ARGS:-} > $d.log 2>&1 ) || { echo "w8 $v failed"; tail -30 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  cp "$f" ${d}_kernel_stats.csv
  t=$(find $d -name "*kernel_trace.csv" | head -1)
  echo "== $MODEL $v rep $rep: $(grep -o '"ms_per_rank_step": [0-9.]*' $d.log)"
  python3 tools/w8_kernel_sum.py "$t" --world 8 | tee ${d}_per_rank_step.txt | head -${TOP:-8}
  find $d -name "*kernel_trace.csv" -size +20M -delete
done
done
