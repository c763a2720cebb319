// Argument blocks of the fused GCN training step (gcn.hip), shared by the kernels and the
// host binding (binding_gcn.cpp).  Plain C++ (no device code).
//
// The step (models/gcn_trainer.py GcnTrainer) trains SupervisedGCN-shaped models — L = 1
// or 2 GCNConv layers over the full-neighbourhood flow (reference
// tf_euler/python/dataflow/gcn_dataflow.py:26-48, convolution/gcn_conv.py:26-54), fc,
// out_fc, sigmoid cross-entropy (mp_utils/base.py:24-47) — in a fixed sequence of launches
// captured into one hipGraph:
//
//   per hop h (targets -> the next node set), three launches:
//     expand  degree + look-back scan of the targets' edge offsets, the neighbour list,
//             one returning atomicAdd per edge on its node's counter (the edge that sees 0
//             claims the node: its count and, when unplaced, its new set position)
//     mark    claims -> look-back scan -> new set positions (node -> position table,
//             stamped with the step's epoch: no table is ever cleared)
//     place   every edge's source position; each claimer adds its node's final count to
//             the in-block source degree (GCN norm) and resets the counter
//   layer     (L = 2) the outer conv: edge-parallel weighted aggregation into LDS, MFMA
//             linear + ReLU -> h1, the aggregate kept for dW
//   head      the last conv + fc + out_fc + loss + the whole row-local backward + the
//             weight-gradient partials of its rows + d(agg) of the roots (L = 2)
//   dw        (L = 2) d(W0) partials, one GEMM row per hop-0 edge: w_e (mask[s] . d agg[t])
//             against the kept aggregate of s (d(h1) is never formed)
//   reduce    the partials into the flat fp32 gradient, loss / F1 counts, epoch + 1
// then the flat optimizer (optim.hip).
//
// Node sets are nested (S_1 ⊂ S_2) and ordered targets-first: S_{h+1} = [S_h, new
// neighbours in the edge order of their claims], so a node keeps its position once placed
// (which of a node's edges claims it is a race: the order of the new nodes is not fixed
// across runs; every per-target sum still runs over the same edges in edge order).  Hop
// 0's targets are the B roots as drawn (repeats kept); S_1 starts with the distinct roots.
// Sets are permutations of the reference's unique([neighbours, targets]) sets, and every
// per-target sum runs over the same edges, so the loss equals the generic device path's.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace euler_hip {

constexpr int kGcnMaxHops = 2;
constexpr int kGcnHeadRows = 16;   // roots per head block
constexpr int kGcnTileRows = 64;   // targets per layer block
constexpr int kGcnDwRows = 128;    // rows of S_1 per dw block (4 chunks of 32)
constexpr int kGcnExpandT = 64;    // most targets per expand block
// targets per expand block for a hop of cap_t targets: a power of two in [4, 64] near
// cap_t / 1024, so the launch has >= ~128 blocks (expand's edges spread over the chip)
__host__ __device__ inline int gcn_expand_tile(int64_t cap_t) {
  int te = 4;
  while (te < kGcnExpandT && static_cast<int64_t>(te) * 2 * 1024 <= cap_t) te *= 2;
  return te;
}
constexpr int kGcnMaxStage = 4;    // weight images staged per step
constexpr int kGcnStageBlocks = 64;// extra blocks of hop 0's expand launch that stage them

// one fp32 weight [rows][cols] -> a padded bf16 image [rowsp][ld] in global memory
struct GcnStageW {
  const float* w;
  int32_t rows, cols, rowsp, ld;
  uint16_t* img;
};

struct GcnGraph {
  const int64_t* indptr;  // [N*T + 1]
  const int32_t* nbr;     // [E]
  const float* cumw;      // [E] per-(row, type) cumulative edge weights (layer-wise draws)
  int64_t num_rows;
  int32_t num_types;
};

struct GcnHop {
  GcnGraph g;
  uint32_t mask;           // edge types of this hop
  int32_t h;               // hop index
  int32_t self_loops;      // 1: one (t, t) edge per target (counted in the source degrees)
  int32_t* roots;          // hop 0: [B] the drawn roots (expand writes them); nullptr for h >= 1
  int32_t B;
  int32_t* set;            // cumulative node set [cap_set] (ids by position)
  int32_t* cnt;            // [kGcnMaxHops + 1] device counts (cnt[0] = B)
  int64_t cap_t;           // target capacity
  int64_t cap_e;           // edge capacity
  int64_t cap_n;           // capacity of S_{h+1}
  int32_t* off;            // [cap_t + 1] exclusive edge offsets per target
  int32_t* enode;          // [cap_e] neighbour node of every edge
  int32_t* etgt;           // [cap_e] target index of every edge
  int32_t* esrc;           // [cap_e] source position (-1: padding)
  int32_t* deg_s;          // [cap_n] in-block source counts (self loops included)
  int32_t* rself;          // hop 0: [B] the set position of each root (its self-loop source)
  // hop 0: the roots are drawn by this launch (Walker alias table over root_rows, Philox
  // (rng[0], rng[1] << 8 ^ 1, t): the same draw as sampling.hip alias_sample_kernel)
  const float* prob;
  const int32_t* alias;
  const int32_t* root_rows;  // nullable: draw rows directly
  int64_t pop;
  const int64_t* rng;
  uint64_t* first;         // [N] epoch-keyed first occurrence of a root (hop 0)
  int32_t* cntw;           // [N] per-node edge counters of the running hop (zero between hops:
                           //     each node's counter claimer resets it in place)
  uint8_t* eflag;          // [cap_e] bit 0: the edge took its node's counter first (the
                           //     counter claimer), bit 1: ... and the node is not yet placed
  int32_t* tag;            // [N] epoch of a node's placement
  int32_t* pos;            // [N] position of a placed node
  uint64_t* scan_deg;      // look-back words of the degree scan [expand blocks]
  uint64_t* scan_flag;     // look-back words of the first-occurrence scan [mark blocks]
  const int32_t* stamp;    // [1] step epoch (the reduce launch advances it)
  int32_t* overflow;       // [1] |= 1 when an edge or set capacity is exceeded
  int32_t* err;            // [1] |= 2 when a look-back wait timed out
  GcnStageW st[kGcnMaxStage];  // hop 0: weight images staged by extra blocks of expand
  int32_t nst;
  // FastGCN / AdaptiveGCN layer filter (nullptr: the full neighbourhood): an edge is kept
  // iff its neighbour's lflag entry holds this step's epoch (gcn_layer_draw stamps the layer)
  const int32_t* lflag;
  int32_t roots_given;     // hop 0: the roots were drawn by the layer-wise draw (read, not drawn)
};

// The per-hop layer of the layer-sampled flows, stamped with the step's epoch in lflag:
//   kind 0 (FastGCN, reference tf_euler/python/dataflow/fast_dataflow.py:25-57): count rows
//     drawn from a node-type sampler's alias table on Philox (rng[0], rng[1] << 8 ^ stream,
//     i) — sample_node(count, stream) of the generic DeviceLayerFlow;
//   kind 1 (AdaptiveGCN, layerwise_dataflow.py:26-71, sampleLNB): one block draws the B
//     roots (the root alias table, stream 1, written to roots: hop 0's expand reads them),
//     their out-weights under the hop's mask, a double prefix sum, count picks of a root in
//     proportion (uniforms from two 16-bit draws on streams 40 + h and 140 + h) and one
//     weighted neighbour of each (stream 30 + h) — DeviceLayerFlow's "layer" hop.
struct GcnLayerDraw {
  int32_t kind;
  const float* prob;         // kind 0: the layer sampler; kind 1: the root sampler
  const int32_t* alias;
  const int32_t* root_rows;  // nullable
  int64_t pop;
  const int64_t* rng;
  uint64_t stream;           // kind 0: the draw; kind 1: the neighbour draw (30 + h)
  int64_t count;
  int32_t* lflag;
  const int32_t* stamp;
  // kind 1
  GcnGraph g;
  uint32_t mask;
  int32_t B;
  int32_t* roots;
  uint64_t stream_u;         // 40 + h (the second 16 bits on stream_u + 100)
};
constexpr int kGcnLayerMaxRoots = 4096;  // kind 1: the roots' prefix sums live in LDS

// one conv layer's weights (fp32 masters, unpadded [out][in])
struct GcnLin {
  const float* w;
  int32_t out, in;   // real sizes
  int32_t outp, inp; // padded (multiples of 32)
};

// edge-parallel aggregation source of a block: source rows either feature rows by node id
// (x = feature table [N][ld], via set[]) or bf16 rows by set position (x = h rows [cap][ld])
struct GcnAggSrc {
  const void* x;
  int32_t x_fp32;      // feature table dtype (by-id source only)
  int32_t by_id;       // 1: row = set[src]; 0: row = src
  const int32_t* set;
  int32_t ld;          // row stride (elements)
  int32_t cols;        // real columns read (<= ld)
};

struct GcnLayerArgs {  // the outer conv (L = 2): targets S_1, sources S_2
  GcnAggSrc src;
  const int32_t* enode; // hop 1 neighbour node ids (by-id source rows)
  const int32_t* off;   // hop 1
  const int32_t* etgt;
  const int32_t* esrc;
  const int32_t* deg_s;
  const int32_t* cnt;   // device counts; targets = cnt[1]
  int64_t cap_t;
  int32_t self_loops;
  GcnLin lin;
  const uint16_t* wimg; // staged bf16 image of lin.w [outp][img_ld(inp)]
  uint16_t* h_out;      // [cap_t][lin.outp] bf16 relu(agg W^T)
  uint16_t* agg_out;    // [cap_t][lin.inp] bf16 aggregate (dW operand)
};

struct GcnHeadArgs {  // targets: the B roots; sources: S_1
  GcnAggSrc src;
  const int32_t* enode; // hop 0 neighbour node ids (L = 1: by-id source rows)
  const int32_t* off;   // hop 0
  const int32_t* etgt;
  const int32_t* esrc;
  const int32_t* deg_s;
  const int32_t* rself;
  const int32_t* roots;
  int32_t B;
  int32_t self_loops;
  GcnLin lin;           // the last conv
  const uint16_t* wl_img;    // staged bf16 images: last conv [outp][img_ld(inp)],
  const uint16_t* wfc_img;   //   fc [Ep][img_ld(outp)],
  const uint16_t* wout_img;  //   out [Cp][144]
  const float* wfc;     // [E][H] fp32
  const float* bfc;     // [E]
  const float* wout;    // [C][E] fp32 (no bias: reference out_fc)
  int32_t E, Ep, C, Cp;
  const float* labels;  // [N][C] dense multi-label targets
  float inv_scale;      // 1 / (B C)
  float* dagg;          // L = 2: [B][lin.inp] fp32 d(agg) of the roots, gcn_dw's input (nullptr: L = 1)
  float* dbg_agg;       // diagnostics (nullptr in the step): [B][KP] the roots' fp32 aggregates
  int64_t* ostep_inc;   // fused optimizer step: block 0 advances the optimizer's step count
                        // (the reduce launch then reads it; no ticket over its ~2K blocks)
  float* part_w;        // [nblk][outp][inp]   d(last conv)
  float* part_fc;       // [nblk][Ep][outp]    d(fc W)
  float* part_bfc;      // [nblk][Ep]
  float* part_out;      // [nblk][Cp][Ep]      d(out_fc W)
  float* part_stat;     // [nblk][4] loss, tp, fp, fn
  long long* prof;      // optional [nblk][16] wall-clock stamps of the phases (diagnostics)
};

struct GcnDwArgs {  // d(W0) over hop 0's edges + self loops (L = 2)
  const float* dagg;    // [B][lin.outp] fp32 d(agg) of the roots (the head writes it)
  const uint16_t* h;    // [cap_1][lin.outp] bf16 relu output (its sign = the ReLU mask)
  const uint16_t* agg;  // [cap_1][lin.inp] bf16
  const int32_t* off;   // hop 0 [cap_t + 1]
  const int32_t* etgt;
  const int32_t* esrc;
  const int32_t* rself;
  const int32_t* deg_s;
  int64_t cap_t, cap_e;  // hop 0
  int32_t B, self_loops;
  GcnLin lin;
  float* part;          // [nblk][outp][inp]
};

constexpr int kGcnMaxSegs = 6;
struct GcnRedSeg {
  float* grad;          // flat gradient view [rows][cols]
  const float* part;    // [S][...] slabs
  int32_t rows, cols;   // real (unpadded) sizes; rows = 1 for vectors
  int32_t prs;          // partial row stride
  int64_t slab;         // elements per slab
  int32_t S;
  int32_t blk0;         // first block of the segment
  float *p, *m, *v;     // fused optimizer: the parameter and its slots, laid out as grad
};
struct GcnReduceArgs {
  GcnRedSeg seg[kGcnMaxSegs];
  int32_t nseg, nblk;
  const float* part_stat;  // [nstat][4]
  int32_t nstat;
  float* loss_out;         // [1]
  int64_t* counts;         // [3] tp, fp, fn (accumulated)
  int32_t* stamp;          // [1] += 1 (block 0, after every read of this step)
  int64_t* rng;            // [2] (seed, counter): counter += 1 (the step's draws are consumed)
  // the flat optimizer folded into this launch (one process: no gradient all-reduce between
  // the reduce and the update): every element is updated where its gradient is summed, at
  // the optimizer's step count the head launch of this step already advanced (a ticket
  // over this launch's ~2K blocks would serialise on one word: ~18 us)
  int32_t fuse_opt, okind;
  const int64_t* ostep;
  float lr, b1, b2, eps, wd, grad_scale;
};

}  // namespace euler_hip

extern "C" {
hipError_t eh_gcn_expand(const euler_hip::GcnHop* a, hipStream_t s);
hipError_t eh_gcn_layer_draw(const euler_hip::GcnLayerDraw* a, hipStream_t s);
hipError_t eh_gcn_mark(const euler_hip::GcnHop* a, hipStream_t s);
hipError_t eh_gcn_place(const euler_hip::GcnHop* a, hipStream_t s);
int64_t eh_gcn_expand_blocks(int64_t cap_t);
int64_t eh_gcn_mark_blocks(const euler_hip::GcnHop* a);
hipError_t eh_gcn_layer(const euler_hip::GcnLayerArgs* a, hipStream_t s);
hipError_t eh_gcn_head(const euler_hip::GcnHeadArgs* a, hipStream_t s);
size_t eh_gcn_head_lds(const euler_hip::GcnHeadArgs* a);
size_t eh_gcn_layer_lds(const euler_hip::GcnLayerArgs* a);
hipError_t eh_gcn_dw(const euler_hip::GcnDwArgs* a, int64_t nblk, hipStream_t s);
hipError_t eh_gcn_reduce(const euler_hip::GcnReduceArgs* a, hipStream_t s);
}
