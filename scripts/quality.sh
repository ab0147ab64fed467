#!/bin/bash
# Bench-shape model quality: each configuration trains --warmup steps untimed,
# then reports the progressive train logloss of the next --steps steps next to
# the constant predictor's (the labels' base-rate entropy).  A model learns
# when its logloss is below the constant one.  ONLY=<regex>: just the matching
# rows; ROWS=<newline-separated argument lists>: these rows instead of the list.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-quality}
mkdir -p "$O"
W=${WARMUP:-300}
S=${STEPS:-100}
i=0
while IFS= read -r args; do
  [ -z "$args" ] && continue
  [ -n "$ONLY" ] && ! [[ "$args" =~ $ONLY ]] && continue
  i=$((i + 1))
  timeout -k 10 300 python bench.py --warmup $W --steps $S --clock-warmup-s 0 $args > "$O/q$i.log" 2>&1 ||
      { echo "run '$args' failed"; tail -20 "$O/q$i.log"; exit 1; }
  python3 - "$O/q$i.log" "$args" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
ll, c = d["logloss"], d["constant_logloss"]
print(f"{sys.argv[2]:70s} {d['value']/1e6:7.1f} M/s  logloss {ll:.4f}  constant {c:.4f}  "
      f"{'LEARNS' if ll < c else 'above constant'} ({100 * (c - ll) / c:+.1f} %)")
PY
done < <(if [ -n "$ROWS" ]; then printf '%s\n' "$ROWS"; else cat <<'LIST'
--model lr
--model lr --slices 256
--model fm --v-dim 8
--model fm --v-dim 8 --slices 8
--model fm --v-dim 8 --slices 256
--model fm --v-dim 8 --slices 256 --v-init-scale 1e-4
--model fm --v-dim 8 --fm-math standard
--model fm --v-dim 8 --fm-math standard --slices 256
--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9
--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --sgd-lr 10 --slices 256
--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --sgd-lr 1 --slices 256 --planted-bias 1.2
--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --sgd-lr 256 --planted-bias 1.2
--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --sgd-lr 4 --fields 18 --slices 64 --planted-bias 1.2
LIST
fi)
