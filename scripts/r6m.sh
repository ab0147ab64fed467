#!/bin/bash
# 39-field MVM quality at a 74 % CTR after 2000 untimed steps, two rates each
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
M="--model mvm --v-dim 10 --optimizer sgd --sgd-v-init 0.9 --planted-bias 1.2"
TAG=r6m_quality WARMUP=2000 ROWS="$M --sgd-lr 0.25 --slices 256
$M --sgd-lr 1 --slices 256
$M --sgd-lr 64
$M --sgd-lr 256" bash scripts/quality.sh
