#!/bin/bash
# PMC counter passes (one rocprofv3 run per counter group, kernel trace off)
# over a short bench run, or over PMC_CMD (e.g. "build/kbench").
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-pmc}
ARGS=${BENCH_ARGS:-"--steps 4 --warmup 2"}
CMD=${PMC_CMD:-"python3 bench.py $ARGS"}
GROUPS_DEFAULT=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_WAVES"
  "TCC_HIT_sum TCC_MISS_sum TCC_EA0_ATOMIC_sum"
  "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_VALU SQ_INSTS_SALU SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"
)
if [ -n "$PMC_GROUPS" ]; then IFS=';' read -ra GROUPS_LIST <<< "$PMC_GROUPS"; else GROUPS_LIST=("${GROUPS_DEFAULT[@]}"); fi
i=0
for grp in "${GROUPS_LIST[@]}"; do
  i=$((i + 1))
  timeout -k 10 300 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/${TAG}_$i -o run -- \
    $CMD > gpurun_out/${TAG}_$i.log 2>&1 || { echo "pmc pass $i failed"; tail -20 gpurun_out/${TAG}_$i.log; exit 1; }
done
python3 tools/pmc_summary.py gpurun_out/${TAG}_*
