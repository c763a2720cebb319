// C ABI of the gfx950 kernel launchers (implemented in *.hip, used by binding.cpp).
// Every launcher is asynchronous on the given stream, allocates nothing and never
// synchronises, so callers may capture it into a hipGraph.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

extern "C" {
// sampling.hip
hipError_t eh_rng_advance(int64_t* state, int64_t inc, hipStream_t s);
hipError_t eh_sample_neighbor(const int64_t* indptr, const int32_t* nbr, const float* cumw, int64_t num_rows,
                              int num_types, uint32_t type_mask, const void* nodes, int nodes_is64, int64_t n,
                              int count, int32_t default_row, const int64_t* rng, uint64_t stream_id, int32_t* out,
                              float* out_w, int32_t* out_t, hipStream_t s);
hipError_t eh_alias_sample(const float* prob, const int32_t* alias, const int32_t* rows, int64_t pop, int64_t count,
                           const int64_t* rng, uint64_t stream_id, int32_t* out, hipStream_t s);
hipError_t eh_random_walk(const int64_t* indptr, const int32_t* nbr, const float* cumw, int64_t num_rows,
                          int num_types, const uint32_t* step_masks, const int32_t* starts, int64_t n, int walk_len,
                          int32_t default_row, const int64_t* rng, uint64_t stream_id, float p, float q, int32_t* out,
                          hipStream_t s);
hipError_t eh_synth_degree(int64_t n, float avg_deg, int max_deg, uint64_t seed, int64_t* deg, hipStream_t s);
hipError_t eh_synth_fill(int64_t n, const int64_t* indptr, uint64_t seed, int32_t* nbr, float* cumw, hipStream_t s);

// sage.hip
hipError_t eh_sage_fwd(const void* x, int D, const int32_t* self_idx, const int32_t* nbr_idx, int F,
                       int include_self, float inv_cnt, const void* W, const float* bias, int H, int64_t M, void* out,
                       void* a_save, int relu, hipStream_t s);
hipError_t eh_linear_fwd(const void* A, int K, const void* W, const float* bias, int H, int64_t M, void* out,
                         int relu, hipStream_t s);
hipError_t eh_sage_bwd_scatter(const void* dA, int D, const int32_t* self_idx, const int32_t* nbr_idx, int F,
                               int include_self, float inv_cnt, int64_t M, int disjoint, float* dx, hipStream_t s);
hipError_t eh_relu_bwd(void* g, const void* y, int64_t n, hipStream_t s);

// mp.hip
hipError_t eh_gather_sum(const void* x, int is_bf16, int64_t n_rows, int64_t row_bytes, const int64_t* idx, int64_t n,
                         int F, float* out, hipStream_t s);
hipError_t eh_gather_rows(const void* x, int64_t n_rows, int64_t row_bytes, const void* idx, int idx_is64, int64_t n,
                          void* out, hipStream_t s);
hipError_t eh_segment_reduce_wave(const void* src, int is_bf16, int D, const int64_t* indptr, const int64_t* perm,
                                  int64_t S, int op, void* out, hipStream_t s);
hipError_t eh_segment_reduce(const void* src, int is_bf16, int D, const int64_t* indptr, const int64_t* perm,
                             int64_t S, int op, float empty_val, void* out, int64_t* argmax, hipStream_t s);
hipError_t eh_index_add_rows(const void* src, int is_bf16, int D, const int64_t* idx, int64_t n, float* out,
                             int64_t n_out, hipStream_t s);
hipError_t eh_max_bwd(const void* gout, int is_bf16, const int64_t* argmax, int64_t S, int D, void* gsrc,
                      hipStream_t s);
hipError_t eh_edge_softmax(const void* logits, int is_bf16, int H, const int64_t* indptr, const int64_t* perm,
                           int64_t S, void* out, hipStream_t s);
hipError_t eh_edge_softmax_bwd(const void* p, const void* g, int is_bf16, int H, const int64_t* indptr,
                               const int64_t* perm, int64_t S, void* gin, hipStream_t s);
hipError_t eh_spmm_csr(const int64_t* indptr, const int64_t* col, const float* w, const void* x, int is_bf16, int D,
                       int64_t S, void* out, hipStream_t s);
}

extern "C" {
// gat.hip (K5: fused multi-head GAT edge-softmax + aggregation)
int eh_gat_supported(int H, int C, int is_bf16);
// order / corder: optional visiting order of the CSR / CSC rows (nullptr = identity);
// a_src (optional, [H*C]): al = <h, a_src> per head, recomputed from each gathered row
// instead of read from al (h must then be the same rows al was computed from)
hipError_t eh_gat_fwd(const int64_t* indptr, const int32_t* col, const int32_t* order, int64_t S, const void* h,
                      int is_bf16, const float* al, const float* ar, int H, int C, float slope, void* out, float* lse,
                      const float* a_src, hipStream_t s);
// attention terms al/ar = <z, a_src/a_dst> per head, and their backward (dz += ..., da += ...)
hipError_t eh_gat_att_fwd(const void* z, int is_bf16, int64_t N, int H, int C, const float* a_src,
                          const float* a_dst, float* al, float* ar, hipStream_t s);
// da_src / da_dst: per-block partial slabs [eh_gat_att_bwd_blocks(...)][H*C] (caller sums them)
int eh_gat_att_bwd_blocks(int64_t N, int H, int C, int is_bf16);
hipError_t eh_gat_att_bwd(const void* z, int is_bf16, int64_t N, int H, int C, const float* a_src, const float* a_dst,
                          const float* dal, const float* dar, void* dz, float* da_src, float* da_dst, hipStream_t s);
// stat: scratch of S*H*4 floats (packed (ar, lse, Dv) per row and head)
hipError_t eh_gat_bwd(const int64_t* indptr, const int32_t* col, const int32_t* order, int64_t S,
                      const int64_t* cindptr, const int32_t* crow, const int32_t* corder, int64_t N, const void* h,
                      int is_bf16, const float* al, const float* ar, int H, int C, float slope, const void* out,
                      const void* dout, const float* lse, float* stat, void* dh, float* dal, float* dar,
                      const float* a_src, hipStream_t s);

// rgcn.hip (K6: relation-grouped MFMA GEMM)
size_t eh_rel_gemm_lds(int K, int N, int mode, int tm);
int eh_rel_gemm_tile();      // edges per message-GEMM tile (tiles: <= this many edges of one relation)
int eh_rel_gemm_dw_chunk();
hipError_t eh_rel_weight_bf16(const float* W, int64_t R, int N, int K, void* wb, void* wt, hipStream_t s);  // edges per dW chunk (chunks: <= this many edges of one relation)
hipError_t eh_rel_gemm(const void* A, int K, const int32_t* a_idx, const int32_t* trel, const int32_t* tstart,
                       const int32_t* tlen, int n_tiles, const void* B, int N, const float* scale,
                       const int32_t* o_idx, int mode, int tm, void* Y, hipStream_t s);
hipError_t eh_rel_gemm_dw(const void* G, int N, const int32_t* g_idx, const void* X, int K, const int32_t* x_idx,
                          const float* scale, const int32_t* crel, const int32_t* cstart, const int32_t* clen,
                          const int32_t* csolo, int n_chunks, float* dW, int accum, hipStream_t s,
                          const int32_t* cslot = nullptr, float* part = nullptr, const int32_t* mrel = nullptr,
                          const int32_t* mrp = nullptr, int n_multi = 0);

// embed.hip (K10 knowledge-graph scores, K11 skip-gram sigmoid-CE)
hipError_t eh_sgns_fwd(const void* emb, const void* pos, const void* neg, int is_bf16, int64_t B, int P, int K, int D,
                       float* logits, float* loss_rows, hipStream_t s);
hipError_t eh_sgns_bwd(const void* emb, const void* pos, const void* neg, int is_bf16, int64_t B, int P, int K, int D,
                       const float* logits, float gscale, void* demb, void* dpos, void* dneg, hipStream_t s);
hipError_t eh_sgns_fwd_idx(const void* T, const int64_t* tmap, int64_t nTm, const int64_t* tinv, int64_t nT,
                           const void* C, const int64_t* cmap, int64_t nCm, const int64_t* cinv, int64_t nC,
                           int64_t P, int K, int D,
                           float gscale, float* coef, float* loss_rows, int rows_bf16, hipStream_t s);
hipError_t eh_gather_f32_bf16(const float* x, int64_t n_rows, int D, const int64_t* idx, int64_t n, void* out,
                              hipStream_t s);
hipError_t eh_occ_count_scan(const int64_t* inv, int64_t n, int64_t n_u, int* cnt, int64_t* ptr, void* temp,
                             size_t* temp_bytes, hipStream_t s);
hipError_t eh_occ_fill(const int64_t* inv, int64_t n, const int64_t* ptr, int* cursor, int* list, hipStream_t s);
hipError_t eh_sgns_update(int side, int64_t n_u, const int64_t* ptr, const int* list, const float* coef, int64_t P,
                          int K, int D, const void* src, int src_bf16, int64_t n_src, const int64_t* smap,
                          int64_t n_smap, const int64_t* sinv, void* gout, int gout_bf16, float* table, float* m,
                          float* v, const int64_t* rows, int64_t n_rows, int64_t* step, int inc_step, float lr,
                          float b1, float b2, float eps, int kind, hipStream_t s);
hipError_t eh_kg_fwd(const float* ent, const float* rel, const int64_t* src, const int64_t* dst, const int64_t* ridx,
                     const int64_t* neg, int64_t B, int K, int D, int kind, int corrupt, int normalize,
                     float* pos_score, float* neg_score, hipStream_t s);
hipError_t eh_kg_bwd(const float* ent, const float* rel, const int64_t* src, const int64_t* dst, const int64_t* ridx,
                     const int64_t* neg, int64_t B, int K, int D, int kind, int corrupt, int normalize,
                     const float* gpos, const float* gneg, float* dent, float* drel, int occ, hipStream_t s);

hipError_t eh_kg_step(const float* ent, const float* rel, const int64_t* pool, int64_t P, const int64_t* t_src,
                      const int64_t* t_dst, const int64_t* t_rel, int64_t num_ent, const int64_t* step, uint64_t seed,
                      int64_t B, int K, int D, int kind, int normalize, float margin, int64_t* o_src, int64_t* o_dst,
                      int64_t* o_ridx, int64_t* o_neg, float* coef, float* part, float* loss, float* dent,
                      float* drel, int* nparts_out, float* drel_rep, int rep, int64_t num_rel, hipStream_t s,
                      float* occ_e = nullptr, float* occ_r = nullptr, int64_t* key_e = nullptr,
                      int64_t* key_r = nullptr);
hipError_t eh_det_segsum(const float* src, int D, const int64_t* ptr, const int* perm, int64_t S, float* out,
                         hipStream_t s);
hipError_t eh_det_occ(const int64_t* keys, int64_t n, int64_t S, int* cnt, int64_t* ptr, int* work, int* perm,
                      void* temp, size_t* temp_bytes, hipStream_t s);
hipError_t eh_cast_bf16(const float* x, int64_t n, void* out, hipStream_t s);
hipError_t eh_zero(void* x, int64_t bytes, hipStream_t s);
int eh_bce_parts(int64_t n);
hipError_t eh_bce_f1_fwd(const float* x, const float* labels, const int64_t* rows, int64_t B, int C, float* part,
                         float* loss, int64_t* counts, hipStream_t s);
hipError_t eh_bce_bwd(const float* x, const float* labels, const int64_t* rows, int64_t B, int C, const float* g,
                      float* dx, hipStream_t s);
hipError_t eh_drop_rows(const float* x, int64_t n, int d, float p, uint64_t seed, const int64_t* step, uint64_t salt,
                        float* x0, float* keep, hipStream_t s);

// pair.hip (fused sigmoid cross-entropy of the unsupervised pair objective)
hipError_t eh_pair_fwd(const float* es, const float* ec, int B, int K, int E, float inv_n, float* logits, float* part,
                       float* loss, float* mrr, hipStream_t s);
hipError_t eh_pair_bwd(const float* es, const float* ec, int B, int K, int E, float inv_n, const float* logits,
                       const float* dloss, float* des, float* dec, hipStream_t s);

// gemm.hip (tiled MFMA GEMM with fused epilogues and split-K)
hipError_t eh_gemm(const void* A, const void* B, void* C, const float* bias, const void* rmask, float* part,
                   int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int a_t,
                   int b_t, int a_bf16, int b_bf16, int c_bf16, int r_bf16, int relu, int splits, float alpha,
                   const void* addend, int64_t ld_add, int add_bf16, const float* rscale, hipStream_t s);

hipError_t eh_gemm_tn(const void* A, const void* B, void* C, float* part, int64_t M, int64_t N, int64_t K, int64_t lda,
                      int64_t ldb, int64_t ldc, int a_bf16, int b_bf16, int c_bf16, int splits, float alpha,
                      const void* addend, int64_t ld_add, int add_bf16, const float* rscale, hipStream_t s);

// route.hip (owner routing of the fixed-capacity all-to-all exchanges)
int64_t eh_route_chunks(int64_t n);
hipError_t eh_route_by_owner(const int64_t* ids, int64_t n, int W, int64_t C, int self_rank, int32_t* cnt,
                             int64_t* pos, int64_t* send, int32_t* overflow, hipStream_t s);

// unique.hip (K8: hash unique, first-occurrence order)
hipError_t eh_unique_init(void* keys, int32_t* minpos, int64_t cap, hipStream_t s);
hipError_t eh_unique_insert(const int64_t* x, int64_t n, void* keys, int32_t* minpos, int64_t cap, int32_t* slot,
                            int skip_neg, hipStream_t s);
hipError_t eh_unique_mark(int64_t n, const int32_t* slot, const int32_t* minpos, int32_t* flag, hipStream_t s);
hipError_t eh_unique_finalize(const int64_t* x, int64_t n, const int32_t* slot, const int32_t* minpos,
                              const int32_t* flag, const int32_t* pos, int64_t* inv, int64_t* uniq, int64_t offset, hipStream_t s);

// flow.hip (device full-neighbourhood expansion, capacity-padded)
hipError_t eh_flow_degree(const int64_t* indptr, int64_t num_rows, int num_types, uint32_t mask, const int64_t* rows,
                          int64_t n, int64_t* deg, hipStream_t s);
hipError_t eh_flow_expand(const int64_t* indptr, const int32_t* nbr, int64_t num_rows, int num_types, uint32_t mask,
                          const int64_t* rows, int64_t n, const int64_t* offs, int64_t cap, int64_t* out_nbr,
                          int64_t* out_src, int32_t* overflow, hipStream_t s);
hipError_t eh_seg_count(const int64_t* idx, int64_t n, int64_t size, int64_t* cnt, hipStream_t s);
hipError_t eh_sage_block(const int64_t* inv, const int64_t* uniq, const int64_t* cnt, const int64_t* last_idx,
                         int64_t cap_prev, int64_t f, int64_t cap_n, int self_loops, int64_t* new_n_id,
                         int64_t* res_n_id, int64_t* edge_index, int64_t* counts, int64_t* last_new, int64_t* cnt_new,
                         hipStream_t s);
hipError_t eh_sage_place(const int64_t* inv, const int64_t* last_idx, int64_t cap_prev, int64_t f, int self_loops,
                         const int64_t* indptr, int64_t* perm, hipStream_t s);
hipError_t eh_gcn_norm_weight(const int64_t* dst, const int64_t* src, int64_t E, const int64_t* c0, int64_t n0,
                              const int64_t* c1, int64_t n1, float* w, hipStream_t s);
hipError_t eh_flow_block(const int64_t* src, const int64_t* offs, const int64_t* uniq, const int64_t* inv,
                         const int64_t* cnt, const int64_t* last_idx, const int64_t* n_targets, int64_t cap_e,
                         int64_t cap_prev, int64_t cap_n, int self_loops, int64_t* new_n_id, int64_t* res_n_id,
                         int64_t* edge_index, int64_t* perm, int64_t* indptr, int64_t* counts, int64_t* last_new,
                         int64_t* cnt_new, int32_t* overflow, hipStream_t s);

// optim.hip
hipError_t eh_flat_optim(float* p, const float* g, float* m, float* v, int64_t n, int64_t* step, float lr, float b1,
                         float b2, float eps, float wd, float grad_scale, int kind, hipStream_t s);
// ticket (int32 [1], zero-initialised; null: a separate step-increment launch): the last block
// advances the step; wd2 replaces wd on the elements [w0, w1)
hipError_t eh_flat_optim2(float* p, const float* g, float* m, float* v, int64_t n, int64_t* step, int32_t* ticket,
                          float lr, float b1, float b2, float eps, float wd, float wd2, int64_t w0, int64_t w1,
                          float grad_scale, int kind, hipStream_t s);
hipError_t eh_sparse_optim(float* table, float* m, float* v, const int64_t* rows, const void* grads, int grads_bf16,
                           int64_t n, int D, int64_t n_rows, int64_t* step, float lr, float b1, float b2, float eps,
                           int kind, hipStream_t s);
}

extern "C" {
// xgmi_ar.hip: two-shot all-reduce over xGMI peer memory (IPC-mapped uncached buffers)
int eh_xar_max_ranks();
int eh_xar_max_blocks();
int eh_xar_vec_per_thread();
hipError_t eh_xar_alloc(int64_t cap, void** sig, void** data);
hipError_t eh_xar_run(void* const* sigs, void* const* bufs, int world, int rank, void* data, int is_bf16, int64_t n,
                      int64_t cap, int blocks, uint32_t* epoch, int* err, long long timeout, hipStream_t s);
}
