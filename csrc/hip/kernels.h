// xflow-amd: host launchers of the gfx950 kernels (implemented in *.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "xflow/backend.h"

namespace xflow {
namespace hip {

// kernels_table.hip
void launch_dedup(const u64* keys, int64_t nnz, ScratchView s, DedupOut o, hipStream_t st);
void launch_scratch_reset(ScratchView s, const u32* pos, const int64_t* n_dev, int64_t n_max,
                          hipStream_t st);
void launch_table_pull(const PullArgs& a, hipStream_t st);
void launch_table_apply(const ApplyArgs& a, hipStream_t st);
void launch_gather_grads(const GatherGradArgs& a, hipStream_t st);
void launch_owner_group(const OwnerGroupArgs& a, hipStream_t st);
void launch_bucket(const BucketArgs& a, hipStream_t st);
void launch_remap_pos(u32* pos, int64_t nnz, const u32* inv, u32 none, hipStream_t st);
void launch_partition_counts(const ScratchView& s, const u32* chunk_offsets,
                             const int64_t* n_uniq, int64_t* counts, int64_t seq, hipStream_t st);
void launch_scatter_rows(const float* src, float* dst, const u32* map, const int64_t* n_dev,
                         int64_t n_max, int width, float* zero_out, int zero_width,
                         hipStream_t st);
void launch_gather_rows(const float* src, float* dst, const u32* map, const int64_t* n_dev,
                        int64_t n_max, int width, bool zero_src, hipStream_t st);
void launch_gather_u32(const u32* src, u32* dst, const u32* map, const int64_t* n_dev,
                       int64_t n_max, bool zero_src, hipStream_t st);
void launch_scatter_u32(const u32* src, u32* dst, const u32* map, const int64_t* n_dev,
                        int64_t n_max, hipStream_t st);
void launch_fill_u64(u64* p, u64 v, size_t n, hipStream_t st);
// CSR exchange: exclusive scan (out[n] = total; tiles: n_max / 4096 + 2 words)
void launch_scan_u32(const u32* in, u32* out, const int64_t* n_dev, int64_t n_max, u32* tiles,
                     hipStream_t st);
void launch_csr_pack(const u32* off, const u32* cnt, const void* src, const u32* doff,
                     const int64_t* n_dev, int64_t n_max, void* dst, int entry_bytes,
                     hipStream_t st);
void launch_csr_totals(const int64_t* counts, int world, bool encoded, const u32* doff,
                       int64_t* totals, hipStream_t st);
void launch_upload_small(void* dst, const void* src, size_t bytes, hipStream_t st);
void launch_download_small(void* host_dst, const void* src, size_t bytes, hipStream_t st);
void launch_snapshot(HostSnap* dst, const u32* mon, unsigned long long seq, hipStream_t st);
void launch_table_clear(const TableView& t, hipStream_t st);
void launch_table_export(const TableView& t, u64* keys_out, u32* words_out, int64_t max_rows,
                         unsigned long long* counter, hipStream_t st);
void launch_table_import(const TableView& t, const u64* keys, const u32* words, int64_t n,
                         hipStream_t st);
void launch_table_prefill(const TableView& t, int64_t n, u64 seed, hipStream_t st);
// growth: split segments [s0, s0 + k) (marks: (k << seg_log2) / 64 words of scratch)
void launch_table_split(const TableView& t, u64 s0, u64 k, u64* marks, hipStream_t st);
void launch_table_nonzero(const TableView& t, const OptSpec& o, unsigned long long* counter,
                          hipStream_t st);

// kernels_layout.hip
void launch_unpack_block(const UnpackArgs& a, hipStream_t st);
void launch_field_major(const void* src, void* dst, int64_t rows, int F, int elem_bytes, bool widen,
                        hipStream_t st);

// kernels_model.hip
void launch_forward_backward(const FwdArgs& a, hipStream_t st);
void launch_slice_masks(const BatchView& b, const u32* pos, u32* tmask, hipStream_t st);

// kernels_parse.hip
void launch_parse_text(const TextParseArgs& a, hipStream_t st);

// kernels_eval.hip
void launch_eval_metrics(const float* pctr, const float* labels, int64_t n, EvalMetrics* out,
                         hipStream_t st);

// kernels_synth.hip
void launch_synth(const SynthArgs& a, hipStream_t st);

}  // namespace hip
}  // namespace xflow
