#!/bin/bash
# One parametrised runner for every GPU-box job (run through gpurun):
#
#   bash scripts/gpu.sh head                      GPU tests + smoke + driver bench x2 + kernel profile
#   bash scripts/gpu.sh tests [pytest args]       GPU test suite (default: all of -m gpu)
#   bash scripts/gpu.sh smoke
#   bash scripts/gpu.sh bench "ARGS|ARGS|..."     bench.py per argument set, one summary line each
#   bash scripts/gpu.sh prof "ARGS"               rocprofv3 kernel stats + launch gaps of one bench
#   bash scripts/gpu.sh pmc "ARGS" "KREGEX"       three PMC passes over the kernels matching KREGEX
#   bash scripts/gpu.sh ab "V1 V2" "ARGS"         ABAB of variants/<V>/ snapshots (make_variant.sh)
#   bash scripts/gpu.sh shared "N..." "ARGS|..."  multi-process RCCL rehearsal, N ranks sharing GPU 0
#   bash scripts/gpu.sh kbench "ARGS"             tools/kbench.hip kernel experiments
#
# Outputs go to gpurun_out/$TAG/ (TAG defaults to the subcommand).  Every GPU
# step runs under its own time limit and the script stops at the first
# failure (no retries).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
cmd=${1:?subcommand}
shift
TAG=${TAG:-$cmd}
O=gpurun_out/$TAG
mkdir -p "$O"

summary() {  # last JSON line of a bench log -> one line
  python3 - "$1" "$2" <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
extra = {k: d[k] for k in ("logloss", "mvm_live", "bytes_moved_per_step", "host_waits", "mid_step_waits")
         if k in d}
print(f"{sys.argv[2]:40s} {d['value']/1e6:8.1f} M samples/s {d['ms_per_step']:.4f} ms/step", extra)
PY
}

kstats() {  # top kernels of a rocprofv3 kernel_stats.csv
  python3 - "$1" <<'PY'
import csv, sys
for x in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{x['Name'][:72]:72s} n={x['Calls']:>5} avg_us={float(x['AverageNs'])/1000:9.1f} {float(x['Percentage']):6.2f}%")
PY
}

run_tests() {  # [pytest args]: default the whole GPU suite (-x); with args, just those
  local sel=(tests -x)
  [ $# -gt 0 ] && sel=()
  timeout -k 10 900 python -u -m pytest "${sel[@]}" -q -m gpu --timeout 170 --timeout-method thread "$@" \
      > "$O/pytest_gpu.log" 2>&1 || { echo "pytest gpu failed"; tail -60 "$O/pytest_gpu.log"; exit 1; }
  tail -1 "$O/pytest_gpu.log"
}

run_smoke() {
  timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 ||
      { echo "smoke failed"; cat "$O/smoke.log"; exit 1; }
  tail -1 "$O/smoke.log"
}

run_bench() {  # "ARGS|ARGS|..."
  IFS='|' read -ra L <<< "${1:-}"
  [ ${#L[@]} -eq 0 ] && L=("")
  local i=0
  for a in "${L[@]}"; do
    i=$((i + 1))
    timeout -k 10 ${TLIM:-300} python bench.py --steps ${STEPS:-20} --warmup ${WARMUP:-5} $a \
        > "$O/bench_$i.log" 2>&1 || { echo "bench '$a' failed"; tail -30 "$O/bench_$i.log"; exit 1; }
    summary "$O/bench_$i.log" "${a:-(default)}"
  done
}

run_prof() {  # "ARGS"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$O/prof" -o run -- \
      python3 bench.py --steps ${STEPS:-20} --warmup 5 ${1:-} > "$O/prof.log" 2>&1 ||
      { echo "profile failed"; tail -20 "$O/prof.log"; exit 1; }
  local f t
  f=$(find "$O/prof" -name "*kernel_stats.csv" | head -1)
  cp "$f" "$O/kernel_stats.csv"
  kstats "$O/kernel_stats.csv"
  t=$(find "$O/prof" -name "*kernel_trace.csv" | head -1)
  python3 tools/trace_gaps.py "$t" --marker ${MARKER:-k_synth} --steps $(( ${STEPS:-20} - 2 )) > "$O/gaps.txt" &&
      head -24 "$O/gaps.txt"
  find "$O/prof" -name "*kernel_trace.csv" -size +20M -delete
}

run_pmc() {  # "ARGS" "KREGEX"
  local P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE"
  local P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_ANY"
  local P3="TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_WRREQ_sum"
  local i=0 P d
  for P in "$P1" "$P2" "$P3"; do
    i=$((i + 1))
    d=$O/p$i
    timeout -s KILL 150 rocprofv3 --pmc $P --kernel-include-regex "${2:-.}" --output-format csv -d $d -o run -- \
        python3 bench.py --steps 3 --warmup 1 ${1:-} > $d.log 2>&1 || { echo "pmc pass $i failed"; tail -20 $d.log; exit 1; }
  done
  python3 - "$O/p1" "$O/p2" "$O/p3" <<'PY'
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
}

run_pmcx() {  # "ARGS" "KREGEX" "COUNTERS" -- one extra PMC pass with the given counters
  local d=$O/px
  timeout -s KILL 150 rocprofv3 --pmc $3 --kernel-include-regex "${2:-.}" --output-format csv -d $d -o run -- \
      python3 bench.py --steps 3 --warmup 1 ${1:-} > $d.log 2>&1 || { echo "pmc pass failed"; tail -20 $d.log; exit 1; }
  python3 - "$d" <<'PY'
import csv, glob, sys, collections
acc = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        acc[r["Kernel_Name"][:60]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, cs in acc.items():
    print("==", k)
    for c, v in sorted(cs.items()):
        print(f"   {c:40s} {sum(v)/len(v):16.1f}  (n={len(v)})")
PY
}

run_ab() {  # "V1 V2 ..." "ARGS"
  local r v
  for r in $(seq 1 ${ROUNDS:-2}); do
    for v in $1; do
      (cd variants/$v && timeout -k 10 300 python bench.py --steps ${STEPS:-30} --warmup 5 ${2:-}) \
          > "$O/ab_$v.log" 2>&1 || { echo "variant $v failed"; tail -20 "$O/ab_$v.log"; exit 1; }
      summary "$O/ab_$v.log" "round $r [$v]"
    done
  done
}

run_shared() {  # "N..." "ARGS|ARGS|..."
  export XFLOW_SHARED_GPU=1 NCCL_DEBUG=${NCCL_DEBUG:-WARN}
  local n a log j=0
  IFS='|' read -ra L <<< "${2:-}"
  [ ${#L[@]} -eq 0 ] && L=("")
  for n in ${1:-2}; do
    for a in "${L[@]}"; do
      j=$((j + 1))
      log=$O/shared_n${n}_$j.log
      timeout -k 10 ${TLIM:-240} python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
          --master-addr 127.0.0.1 --master-port $((29611 + n)) bench.py --gpus $n \
          --steps ${STEPS:-5} --warmup 2 --batch ${BATCH:-65536} --log2-cap ${LOG2CAP:-26} $a \
          > $log 2>&1 || { echo "shared-GPU bench n=$n '$a' failed"; tail -40 $log; exit 1; }
      summary $log "n=$n ${a:-(default)}"
    done
  done
}

run_kbench() {
  if [ ! -x build/kbench ] || [ -n "$REBUILD" ]; then
    /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -ffp-contract=off \
      -Icsrc/include -Icsrc/hip tools/kbench.hip csrc/hip/kernels_table.hip \
      csrc/hip/kernels_model.hip csrc/hip/kernels_synth.hip -o build/kbench || exit 1
  fi
  timeout -k 10 300 build/kbench ${1:-} > "$O/kbench.log" 2>&1 || { echo "kbench failed"; tail -20 "$O/kbench.log"; exit 1; }
  cat "$O/kbench.log"
}

case $cmd in
  head) run_tests && run_smoke && run_bench "" && run_bench "" && run_prof "" ;;
  tests) run_tests "$@" ;;
  smoke) run_smoke ;;
  bench) run_bench "${1:-}" ;;
  prof) run_prof "${1:-}" ;;
  pmc) run_pmc "${1:-}" "${2:-.}" ;;
  pmcx) run_pmcx "${1:-}" "${2:-.}" "${3:?counters}" ;;
  ab) run_ab "${1:?variants}" "${2:-}" ;;
  shared) run_shared "${1:-2}" "${2:-}" ;;
  kbench) run_kbench "${1:-}" ;;
  *) echo "unknown subcommand $cmd"; exit 2 ;;
esac
