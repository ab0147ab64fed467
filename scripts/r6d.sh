set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r6d; mkdir -p $O
timeout -k 10 120 rocprofv3 -L > $O/counters.txt 2>&1; echo "list rc=$?"; wc -l $O/counters.txt
TAG=r6d_bubble bash scripts/csr_bubble.sh || exit 1
TAG=r6d_pmc bash scripts/gpu.sh pmc "" "k_dedup_insert|k_lr|k_pull_lr16|k_red_sum|k_red_scatter|k_apply_lr16|k_synth|k_compact_write"
