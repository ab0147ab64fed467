#!/bin/bash
# standard FM: scatter-free producer (default) vs dense region + k_red_scatter
# (XFLOW_FMSTD_SEG=0), same box, alternating; then the LR step's kernel stats
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r6s
mkdir -p $O
sum() { python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print(f"{sys.argv[2]:28s} {d['value']/1e6:8.1f} M samples/s {d['ms_per_step']:.4f} ms/step logloss {d['logloss']:.6f}")
PY
}
for r in 1 2; do
  for v in 1 0; do
    XFLOW_FMSTD_SEG=$v timeout -k 10 300 python bench.py --model fm --fm-math standard --steps 20 \
        --warmup 5 > $O/fms_$v.log 2>&1 && sum $O/fms_$v.log "r$r XFLOW_FMSTD_SEG=$v" || exit 1
  done
done
XFLOW_FMSTD_SEG=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/p0 -o run -- \
    python3 bench.py --model fm --fm-math standard --steps 20 --warmup 5 > $O/p0.log 2>&1 &&
TAG=r6s_lr bash scripts/gpu.sh prof "" &&
python3 tools/kstats.py $(find $O/p0 -name "*kernel_stats.csv" | head -1) 2>/dev/null | head -16 ||
head -16 $(find $O/p0 -name "*kernel_stats.csv" | head -1)
