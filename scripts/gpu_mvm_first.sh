#!/bin/bash
# Per-call kernel durations of the MVM backward when every occurrence is live
# (first steps of FTRL with O(1) latent init), reduction path vs atomics.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for v in red atomics; do
  case $v in atomics*) export XFLOW_MVM_ATOMICS=1;; *) unset XFLOW_MVM_ATOMICS;; esac
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/prof_mvmf_$v -o run -- python3 bench.py --model mvm --v-dim 10 --v-init-scale 1.0 --steps 2 --warmup 1 > gpurun_out/prof_mvmf_$v.log 2>&1 || { tail -20 gpurun_out/prof_mvmf_$v.log; exit 1; }
  f=$(find gpurun_out/prof_mvmf_$v -name "*kernel_trace.csv" | head -1)
  python3 - "$f" "$v" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: int(r['Start_Timestamp']))
for r in rows:
    n = r['Kernel_Name']
    if any(k in n for k in ('k_mvm', 'k_red_', 'k_apply', 'k_dedup')):
        print(sys.argv[2], f"{(int(r['End_Timestamp'])-int(r['Start_Timestamp']))/1000:9.1f} us  {n[:60]}")
PY
  rm -f "$f"
done
