#!/bin/bash
# Emulated 8-GPU step (tools/w8_emulate.py) under rocprofv3, A/B of env
# variants: per-rank device time per step from the kernel stats
# (tools/w8_kernel_sum.py).  VARIANTS: '|'-separated "name:ENV=1 ENV2=1".
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
mkdir -p gpurun_out
TAG=${TAG:-w8ab}
MODEL=${MODEL:-lr}
VARIANTS=${VARIANTS:-"base:"}
IFS='|' read -ra VL <<< "$VARIANTS"
for rep in ${REPS:-1}; do
for v in "${VL[@]}"; do
  name=${v%%:*}; envs=${v#*:}
  d=gpurun_out/${TAG}_${MODEL}_${name}_$rep
  rm -rf $d
  ( for e in $envs; do export "$e"; done
    timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- \
      python3 tools/w8_emulate.py --model $MODEL ${W8_ARGS:-} > $d.log 2>&1 ) || { echo "w8 $name failed"; tail -30 $d.log; exit 1; }
  f=$(find $d -name "*kernel_stats.csv" | head -1)
  cp "$f" ${d}_kernel_stats.csv
  t=$(find $d -name "*kernel_trace.csv" | head -1)
  echo "== $MODEL $name rep $rep: $(grep -o '"ms_per_rank_step": [0-9.]*' $d.log)"
  python3 tools/w8_kernel_sum.py "$t" --world 8 | tee ${d}_per_rank_step.txt
  find $d -name "*kernel_trace.csv" -size +20M -delete
done
done
