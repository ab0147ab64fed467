set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
K="k_dedup_insert|k_lr|k_pull_lr16|k_red_sum|k_red_scatter|k_apply_lr16|k_synth|k_compact_write"
TAG=r6e_pmc4 bash scripts/gpu.sh pmcx "" "$K" "GRBM_UTCL2_BUSY GRBM_TA_BUSY TA_TA_BUSY_sum TCP_UTCL1_TRANSLATION_MISS_sum TCP_UTCL1_TRANSLATION_HIT_sum TCP_UTCL1_STALL_MULTI_MISS_sum TCP_PENDING_STALL_CYCLES_sum TCC_EA0_RDREQ_DRAM_sum TCC_EA0_WRREQ_DRAM_sum TCC_TAG_STALL_sum TCC_EA0_RDREQ_DRAM_CREDIT_STALL_sum" &&
TAG=r6e_bubble bash scripts/csr_bubble.sh
