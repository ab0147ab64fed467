#!/bin/bash
# The README performance table: one bench.py run per row on one box
# (--steps 20 --warmup 5, the driver's shape), one summary line each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-models}
mkdir -p "$O"
i=0
while IFS= read -r args; do
  i=$((i + 1))
  timeout -k 10 300 python bench.py --steps ${STEPS:-20} --warmup 5 $args > "$O/m$i.log" 2>&1 ||
      { echo "run '$args' failed"; tail -20 "$O/m$i.log"; exit 1; }
  python3 - "$O/m$i.log" "$args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
x = {k: round(d[k], 4) for k in ("logloss",) if k in d}
if "mvm_live" in d:
    x["mvm_live"] = d["mvm_live"]
print(f"{sys.argv[2] or '(default)':60s} {d['value']/1e6:7.1f} M samples/s {d['ms_per_step']:.4f} ms/step {x}")
PY
done <<'LIST'

--slices 8
--slices 64
--slices 256
--model fm
--model fm --slices 4
--model fm --slices 8
--model fm --slices 256
--model fm --fm-math standard
--model fm --fm-math standard --slices 8
--model fm --fm-math standard --slices 64
--model fm --fm-math standard --slices 256
--model mvm --v-dim 10
--model mvm --v-dim 10 --slices 8
--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9
--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --slices 4
--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --slices 64
--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --slices 256
--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --fields 18
LIST
