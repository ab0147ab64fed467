#!/bin/bash
# PMC of the final column-walk producers: standard FM (k_fm_std_red) and LR (k_lr)
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${P:-r6w}_fms bash scripts/gpu.sh pmc "--model fm --fm-math standard" "k_fm_std_red|k_red_sum_vec" &&
TAG=${P:-r6w}_lr bash scripts/gpu.sh pmc "" "k_lr|k_red_sum|k_red_scatter"
