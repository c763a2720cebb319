// Argument blocks of the fused GraphSAGE tree-step kernels (sage_tree.hip), shared by
// the kernels and the host binding (binding_tree.cpp).  Plain C++ (no device code):
// the binding TU is compiled by g++.
//
// Mini-batch layout ("slotted tree"): level 0 = B roots; every row of level k-1 owns a
// group of P_k = 2^logP_k slots at level k: slots 0..F_k-1 are its F_k sampled
// neighbours, slot F_k is the row itself, the rest are padding (node -1, zero rows).
// The rows of a sibling group are contiguous and power-of-two aligned, so the tree
// mean of a layer is a block-local epilogue and the backward routing of a row is
// row >> logP (no index tensors, no atomics).
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace euler_hip {

constexpr int kTrMaxProbs = 6;
constexpr int kTrMaxSegs = 8;
constexpr int kTrHeadRows = 16;  // roots per block of the head kernel
constexpr int kTrHeadSampleRows = 256;  // target rows per sampler block of the head launch

struct TrGraph {
  const int64_t* indptr;    // [N*T + 1]
  const int32_t* nbr;       // [E] neighbour rows
  const float* cumw;        // [E] per-segment inclusive prefix sums of edge weights
  int64_t num_rows;
  int32_t num_types;
  const float* prob;        // root alias table over `pop` candidates
  const int32_t* alias;
  const int32_t* root_rows;  // optional candidate -> row map (node-type subsets)
  int64_t pop;
};

// sampling chain above the target rows of layer 0 (levels 1 and 2 at most)
struct TrTree {
  const int64_t* rng;  // device (seed, counter)
  const int32_t* root_in;  // optional: the roots are given (root t = root_in[t], -1 = padding)
                           // instead of drawn from the alias table (towers of pair models)
  int32_t F1, F2;      // fanouts of hops 1 and 2
  int32_t logP1, logP2;
  uint32_t m1, m2;     // edge-type masks of hops 1 and 2
  // root_in == nullptr: root_mode 0 = alias draw t (stream kTrStreamRoot); 1 = the context
  // tower of a pair model: t < pair_B -> one out-neighbour (pair_mask, stream kTrStreamPos)
  // of the source root t (alias draw t, recomputed), -1 when it has none; t >= pair_B -> an
  // alias draw of the negative stream (kTrStreamNeg)
  int32_t root_mode, pair_B;
  uint32_t pair_mask;
  int32_t stream_off;  // added to the hop / leaf Philox streams (the two towers of a pair
                       // model draw independent neighbourhoods)
};

// mini-batch sampler: the node of every target row of layer 0 (level lv of the tree,
// root -> hop chain) and its FL leaf draws; run one step ahead of the forward on a
// forked stream (sampling depends on nothing the step computes)
struct TrSampleArgs {
  TrGraph g;
  TrTree tr;
  int64_t M;             // target rows (slots of level lv)
  int32_t lv;            // level of the target rows
  int32_t FL;            // leaf fanout (hop lv + 1)
  uint32_t mL;           // leaf edge-type mask
  int32_t hopL;          // leaf hop number (Philox stream)
  int32_t* roots;        // [B] sampled roots (written by the root's self-chain row)
  int32_t* nodes;        // [M] node of every target row
  int32_t* leaf;         // [M][FL] leaf samples
};

// fc and out_fc combined: there is no nonlinearity between them, so the head computes
// logits = h Wc^T + bc and the logits' gradient to h as dlog Wc with Wc = Wout Wfc [C][H]
// and bc = Wout bfc [C] (two dependent GEMM phases fewer on the head's critical path; emb
// and demb, needed only by the fc / out_fc weight gradients, are computed off it).  Wc is
// rebuilt every step from the fp32 masters by extra blocks of the first forward launch.
struct TrCombArgs {
  const float* wout;  // [C][E] fp32 (flat parameters), for bc
  const float* bfc;   // [E]
  const uint16_t* wout_sh;  // fm [C][E] bf16 shadow (the optimizer's)
  const uint16_t* wfcT_sh;  // fm [H][E] bf16 shadow of Wfc^T
  int32_t C, E, H;
  uint16_t* Wc;       // fm [C][H] bf16
  uint16_t* WcT;      // fm [H][C] bf16
  float* bc;          // [C]
};

// one fused SAGE layer: mode 0 = gather (sampled ids) + GEMM + tree-mean epilogue (layer 0),
// mode 1 = gather only, writing [x_self | mean x_nbr] rows (1-hop models),
// mode 2 = rows + GEMM + tree-mean epilogue (inner layers of 3-hop models)
struct TrFwdArgs {
  const void* x;         // modes 0/1: feature table [N][D] (bf16 or fp32); mode 2: A rows bf16 [M][2D]
  int32_t D;             // input width (padded, % 16 == 0)
  int64_t M;             // target rows
  int32_t FL;            // leaf fanout (hop lv + 1)
  int32_t include_self;
  float inv_leaf;        // 1 / (FL + include_self)
  const int32_t* nodes;  // modes 0/1: [M] node of every target row (sampler output)
  const int32_t* leaf;   // modes 0/1: [M][FL] leaf samples
  const uint16_t* W;     // fm bf16 [H][2D]
  int32_t H;             // output width (% 64 == 0)
  uint16_t* a_kt;        // [M/32][2D][32] A operand of dW (optional)
  uint32_t* mask;        // [M/32][H] ReLU bits (optional)
  uint16_t* a_next;      // modes 0/2: [M >> logPg][2H] parent A rows; mode 1: [M][2D]
  int32_t logPg, Fg;     // sibling groups of the target rows: size 2^logPg, Fg neighbour slots
  float inv_grp;         // 1 / (Fg + include_self)
  int64_t* step;         // optimizer step counter (block 0 increments it)
  int64_t* rng;          // (seed, counter): block 0 advances the counter (the batch is consumed)
  const int32_t* roots_in;  // modes 0/1: [B] the batch's roots (sampler output) ...
  int32_t* roots_cur;       // ... copied here for the head (the sampler may refill roots_in)
  int32_t B;
  long long* prof;       // optional per-block phase stamps [grid][8]
  TrCombArgs comb;       // modes 0/1, ncomb != 0: wave 0 of every block builds tiles of the head's Wc
  int32_t ncomb;
  uint16_t* a_rows;      // pipelined step: [M][2D] row-major A rows ([self | mean]) written by the
                         // gather blocks of the previous optimizer launch, read by the GEMM-only
                         // forward (mode 3)
};

// head: last SAGE conv + fc + out_fc + sigmoid-CE + backward down to dA, kTrHeadRows roots / block
struct TrHeadArgs {
  const uint16_t* A;     // [B][Hin2] bf16 rows [self | mean]
  int32_t Hin2, H, E, C, C_real;
  const uint16_t *W, *WT, *Wfc, *WfcT, *Wout, *WoutT;  // fm shadows
  const uint16_t *Wc, *WcT;  // fm Wout Wfc and its transpose (TrCombArgs)
  const float* bfc;      // [E]
  const float* bc;       // [C] Wout bfc
  const int32_t* roots;  // [B] (the forward's copy of the batch's roots)
  const void* labels;    // mode 0: int16 [N] class ids, 1: int32 [N], 2: bf16 [N][C] dense
  int32_t label_mode;
  float inv_scale;       // 1 / (B * C_real)
  uint16_t *A_kt, *h_kt, *emb_kt, *dlog_kt, *demb_kt, *g_kt;
  float* dA;             // [B][Hin2] fp32 (nullptr: no lower layer)
  float* dbfc_part;      // [B/kTrHeadRows][E] per-block fc-bias gradient (reduced by tr_opt)
  float* head_part;      // [B/kTrHeadRows][4] per-block loss, tp, fp, fn (reduced by tr_opt)
  long long* prof;       // optional per-block phase stamps [B/16][8]
  TrSampleArgs smp;      // the next step's sampler, run by extra blocks of the launch on the
  int32_t nsample;       // CUs the head leaves idle (0: none)
};

// pair head (unsupervised GraphSAGE, models/sage_tower.py): for kTrHeadRows sources per
// block and their 1 + K context rows (positive, K negatives) the last conv + fc of both
// towers, the pair logits + sigmoid CE + reciprocal rank, and the backward to dA1 of both
// towers; weight-gradient operands in kt layout for tr_dw, per-block bias / loss partials
// for tr_opt.  Tower s = source (R = B rows), c = context (R = B (1 + K): B positives, then
// the B x K negatives source-major).
struct TrPairTower {
  const uint16_t* A1;        // [R][2H0] bf16 rows [self | mean] (layer 0 of the tower)
  const uint16_t *W1, *W1T;  // fm [H1][2H0] and its transpose
  const uint16_t *Wfc, *WfcT;  // fm [E][H1] and its transpose
  const float* bfc;          // [E] fp32 master
  uint16_t *A1_kt, *h_kt, *de_kt, *g_kt;  // kt [R][2H0], [R][H1], [R][E], [R][H1]
  float* dA1;                // [R][2H0] fp32
  float* dbfc_part;          // [nblk][E]
};
struct TrPairHeadArgs {
  TrPairTower s, c;
  int32_t B, K, H0x2, H1, E;
  float inv_n;       // 1 / (B (1 + K))
  float* head_part;  // [nblk][4]: loss, reciprocal-rank sum, 0, 0
};

// inner-layer backward (3-hop): dA_out = route(dA_parent, mask) @ W  (fp32 rows)
struct TrBwdArgs {
  const float* dA;       // parent gradient [M >> logPg][2Hk]
  const uint32_t* mask;  // [M/32][Hk]
  const uint16_t* WT;    // fm [K2out][Hk]
  int32_t Hk, K2out;
  int64_t M;
  int32_t logPg, Fg, include_self;
  float inv;
  float* dA_out;         // [M][K2out]
};

// split-K dW = G^T X for one weight; route problems build G from the parent gradient
struct TrDwProb {
  const uint16_t* G;     // kt [M/32][P][32] (non-route)
  const uint16_t* X;     // kt [M/32][Q][32]
  float* part;           // [S][P][Q]
  int32_t P, Q, MB, kps, S, tiles_q, ntiles, wg0;
  const float* dA;       // route: [M >> logPg][2P]
  const uint32_t* mask;  // route: [M/32][P]
  int32_t route, logPg, Fg, include_self;
  float inv;
};
struct TrDwProbs {
  TrDwProb p[kTrMaxProbs];
  int32_t n;
};

// flat parameter buffer segments: gradient = sum of S partials [S][n] (split-K slabs of a
// dW problem, or the head's per-block fc-bias sums).  Weight matrices (cols > 0, rows % 8
// == 0, cols % 32 == 0) are processed in 8 x 32 tiles, one per block, so their bf16
// shadows (fm [rows][cols] and the transpose fm [cols][rows]) are written as 16-B rows;
// vectors (cols == 0) in 256-element blocks.
struct TrSeg {
  int64_t off, n;
  const float* part;
  int32_t S;
  int32_t rows, cols;  // cols == 0: vector segment
  int32_t blk0;        // first block of the segment
  uint16_t* sh;        // optional fm [rows][cols]
  uint16_t* shT;       // optional fm [cols][rows]
  int32_t sgrp;        // vector segments: slab groups per element (1 or 4; tr_seg_prepare)
};
// vector segments with many split-K slabs (the fc bias: one slab per head block) spread each
// element's slab sum over 4 threads (256 / 4 elements per block): one round of 16 loads in
// flight per thread instead of S / 16 dependent rounds, which made the bias block the tail
// of the optimizer launch.  Returns the segment's block count.
inline int tr_seg_groups(const TrSeg& s) { return s.cols == 0 && s.S > 16 ? 4 : 1; }
inline int tr_seg_blocks(const TrSeg& s) {
  if (s.cols > 0) return (s.rows / 8) * (s.cols / 32);
  const int64_t per = 256 / tr_seg_groups(s);
  return static_cast<int>((s.n + per - 1) / per);
}
inline int tr_seg_prepare(TrSeg& s) {
  s.sgrp = tr_seg_groups(s);
  return tr_seg_blocks(s);
}
struct TrOptArgs {
  float *p, *g, *m, *v;
  uint16_t* g16;  // optional bf16 gradient (data parallel: the all-reduce moves half the bytes);
                  // mode 0 writes it instead of g, mode 1 reads it
  int64_t n;
  TrSeg seg[kTrMaxSegs];
  int32_t nseg;
  int32_t nblk;  // blocks of the parameter part of the grid
  const int64_t* step;
  float lr, b1, b2, eps, wd, grad_scale;
  int32_t kind;  // 0 adam, 1 adagrad, 2 sgd, 3 momentum
  const float* head_part;  // [nhead][4] per-block loss / tp / fp / fn of the head
  int32_t nhead;
  float* loss_acc;         // loss of the last forward (written by the reduce)
  uint32_t* counts;        // tp, fp, fn since the last reset (accumulated by the reduce)
  float* loss_out;         // loss of the last optimizer step
  float* stat_f;           // optional: += the head's second statistic (pair models: reciprocal
                           // ranks) instead of the tp / fp / fn counts
  TrSampleArgs smp;        // the next step's sampler, run by extra blocks (modes 1/2)
  int32_t nsample;         // sampler blocks (0: none)
  TrFwdArgs gat;           // the next step's layer-0 gather (pipelined step), run by extra blocks:
  int32_t ngather;         //   32-row tiles -> gat.a_kt (dW operand) and gat.a_rows (0: none)
  int32_t gat_fp32;        //   feature table dtype
  int32_t gather_first;    //   gather tiles before the parameter / sampler blocks in the grid
  int32_t opt_tpb;         //   with gather tiles: parameter tiles per block (fewer, longer blocks)
};

// one launch for every dW of the step: routed problems first (their blocks, S % 8 == 0),
// then the stored-G problems grouped
struct TrDwLaunch {
  TrDwProbs plain;
  TrDwProb route[2];
  int32_t nroute;
  int32_t rwg[3];       // block prefix of the routed problems
  int32_t route_impl;   // 0: G^T tile built once per block in LDS; 1: built per wave in registers
  long long* prof;      // optional [route blocks][8] wall-clock stamps (diagnostics)
};

}  // namespace euler_hip

extern "C" {
// feat_fp32: feature table dtype (modes 0/1); bm: rows per block (32, 64 or 128)
hipError_t eh_tr_sample(const euler_hip::TrSampleArgs* a, hipStream_t s);
// mode 3: GEMM-only layer 0 of the pipelined step (a->a_rows from the gather blocks of the
// previous tr_opt launch; fwd2 shapes only)
hipError_t eh_tr_fwd(const euler_hip::TrFwdArgs* a, int mode, int feat_fp32, int bm, hipStream_t s);
size_t eh_tr_gather32_lds(int D, int FL);
hipError_t eh_tr_head(const euler_hip::TrHeadArgs* a, int64_t B, hipStream_t s);
hipError_t eh_tr_bwd(const euler_hip::TrBwdArgs* a, hipStream_t s);
// fills S / tiles / wg0 of every problem from P, Q, MB, kps before launching
hipError_t eh_tr_dw(euler_hip::TrDwLaunch* p, hipStream_t s);
// mode 0: split-K reduce into g; 1: optimizer from g; 2: both fused (single process);
// 3: shadows only (after an external parameter write).  Modes 1/2 also run a->nsample
// sampler blocks.
hipError_t eh_tr_opt(const euler_hip::TrOptArgs* a, int mode, hipStream_t s);
size_t eh_tr_fwd_lds(int D, int H, int bm, int FL, int mode);
size_t eh_tr_fwd2_lds(int D, int FL);
size_t eh_tr_head_lds(int Hin2, int H, int E, int C, int label_mode);
size_t eh_tr_pair_head_lds(int K, int H0x2, int H1, int E);
hipError_t eh_tr_pair_head(const euler_hip::TrPairHeadArgs* a, hipStream_t s);
}
