#!/bin/bash
# PMC counters of selected kernels (KREGEX) of a bench.py run (ARGS), one
# rocprofv3 pass per counter group; per-kernel averages printed.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out
TAG=${TAG:-pmc}
ARGS=${ARGS:-"--model fm --v-dim 8 --fm-math standard"}
KREGEX=${KREGEX:-"k_fm_std_red|k_red_sum_vec|k_fm_std_fwd"}
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"
P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  d=gpurun_out/${TAG}_p$i
  timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "$KREGEX" --output-format csv -d $d -o run -- python3 bench.py --steps 3 --warmup 1 $ARGS > $d.log 2>&1 || { echo "pass $i failed"; tail -20 $d.log; exit 1; }
done
python3 - gpurun_out/${TAG}_p1 gpurun_out/${TAG}_p2 gpurun_out/${TAG}_p3 <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for d in sys.argv[1:]:
    for f in glob.glob(d + "/**/*counter_collection.csv", recursive=True):
        for r in csv.DictReader(open(f)):
            acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print("==", k)
    for c, v in sorted(cs.items()):
        print(f"   {c:24s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
