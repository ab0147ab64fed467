set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
TAG=r6g_quality bash scripts/quality.sh &&
TAG=r6g_pmc bash scripts/gpu.sh pmc "--model fm --fm-math standard" "k_fm_std_red|k_red_sum_vec"
