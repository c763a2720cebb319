// Fused GraphSAGE training step on gfx950 for 1-3 hop models (SURVEY §2.7 K1/K2/K3/K11/
// K12/K13, §7.3) — the kernels behind euler_amd.models.sage_trainer.SageTrainer, which
// NodeEstimator(device_graph=True) and bench.py run.
//
// Model (reference examples/graphsage/graphsage.py:56-67, mp_utils/base_gnn.py:75-92,
// mp_utils/base.py:24-47, convolution/sage_conv.py:33-44):
//   h_k   = relu([h_{k-1}[self] | mean_nbr h_{k-1}] @ W_k^T)     k = 0 .. L-1
//   emb   = h_{L-1} @ Wfc^T + bfc ;  logits = emb @ Wout^T
//   loss  = mean(sigmoid_ce(logits, label))
// Mini-batch = the reference SageDataFlow (sample every node of the previous hops again,
// sage_dataflow.py:35-50) without dedup, in the slotted tree layout of tree_args.h.
//
// A 2-hop step is four launches:
//   tr_fwd  (mode 0)  roots + hop 1 + hop 2 sampling (Philox, on the HBM CSR), gather of
//                     the leaf feature rows, mean, MFMA GEMM + ReLU, and the tree mean of
//                     the next layer as the epilogue -> A1 rows, A0 (kt), ReLU bits
//   tr_head           last conv + fc + out_fc + loss + backward to dA1
//   tr_dw             grouped split-K dW of every weight; the outer layer's G operand is
//                     routed from dA1 through the tree inside the kernel (never stored)
//   tr_opt   (mode 2) split-K reduce + Adam/Adagrad/SGD/momentum + bf16 weight shadows
// (3 hops add one tr_fwd mode 2 and one tr_bwd; 1 hop uses tr_fwd mode 1).
#include <algorithm>
#include <cstdlib>

#include "hip/tile.h"
#include "hip/tree_args.h"

namespace euler_hip {

constexpr uint64_t kTrStreamRoot = 1, kTrStreamPos = 2, kTrStreamNeg = 3, kTrStreamHop = 16;
constexpr int kTrBN = 256;  // output columns per GEMM chunk (4 waves x 64)

__device__ __forceinline__ uint4_t tr_rand(const int64_t* rng, uint64_t stream, uint64_t idx) {
  return Philox::gen(static_cast<uint64_t>(rng[0]), (static_cast<uint64_t>(rng[1]) << 8) ^ stream, idx);
}

// Walker alias draw of root t (reference sample_node: weighted, per node type)
__device__ __forceinline__ int32_t tr_root(const TrGraph& g, const int64_t* rng, int64_t t,
                                           uint64_t stream = kTrStreamRoot) {
  const uint4_t r = tr_rand(rng, stream, static_cast<uint64_t>(t));
  const uint64_t x = (static_cast<uint64_t>(r[0]) << 32) | r[1];
  int64_t k = static_cast<int64_t>(__umul64hi(x, static_cast<uint64_t>(g.pop)));
  if (k >= g.pop) k = g.pop - 1;
  const int64_t pick = (u01(r[2]) < g.prob[k]) ? k : static_cast<int64_t>(g.alias[k]);
  return g.root_rows ? g.root_rows[pick] : static_cast<int32_t>(pick);
}

// one weighted with-replacement neighbour draw (reference node.cc:98-161: pick an edge
// type group by its weight sum, then binary-search the group); -1 when there is none
__device__ int32_t tr_neighbor(const TrGraph& g, int32_t row, uint32_t mask, uint4_t r) {
  if (row < 0 || row >= g.num_rows) return -1;
  const int64_t base = static_cast<int64_t>(row) * g.num_types;
  int64_t lo = 0, hi = 0;
  float total = 0.f;
  if (g.num_types == 1) {
    if (!(mask & 1u)) return -1;
    lo = g.indptr[base];
    hi = g.indptr[base + 1];
    total = hi > lo ? g.cumw[hi - 1] : 0.f;
  } else {
    float tot = 0.f;
    for (int t = 0; t < g.num_types; ++t) {
      if (!((mask >> t) & 1u)) continue;
      const int64_t a = g.indptr[base + t], b = g.indptr[base + t + 1];
      if (b > a) tot += g.cumw[b - 1];
    }
    if (!(tot > 0.f)) return -1;
    float u = u01(r[0]) * tot;
    for (int t = 0; t < g.num_types; ++t) {
      if (!((mask >> t) & 1u)) continue;
      const int64_t a = g.indptr[base + t], b = g.indptr[base + t + 1];
      if (b <= a) continue;
      const float gw = g.cumw[b - 1];
      lo = a;
      hi = b;
      total = gw;
      if (u < gw) break;
      u -= gw;
    }
  }
  if (hi <= lo || !(total > 0.f)) return -1;
  const float u = u01(r[1]) * total;
  int64_t a = lo, b = hi - 1;
  while (a < b) {
    const int64_t m = (a + b) >> 1;
    if (g.cumw[m] > u) b = m;
    else a = m + 1;
  }
  return g.nbr[a];
}

// slot j of the group of `parent` (whose own slot index is parent_slot) at hop `hop`
__device__ __forceinline__ int32_t tr_hop(const TrGraph& g, const int64_t* rng, int32_t parent, int j, int F,
                                          uint32_t mask, int hop, int64_t parent_slot, int stream_off = 0) {
  if (j < F)
    return parent >= 0 ? tr_neighbor(g, parent, mask,
                                     tr_rand(rng, kTrStreamHop + hop + stream_off,
                                             static_cast<uint64_t>(parent_slot * F + j)))
                       : -1;
  return j == F ? parent : -1;
}

// root t of a tree (see TrTree::root_mode): given, an alias draw, or a pair model's context
// root (the source root's positive neighbour, or a negative draw)
__device__ __forceinline__ int32_t tr_tree_root(const TrGraph& g, const TrTree& tr, int64_t t) {
  if (tr.root_in) return tr.root_in[t];
  if (tr.root_mode == 0) return tr_root(g, tr.rng, t);
  if (t < tr.pair_B) {
    const int32_t src = tr_root(g, tr.rng, t);
    return src >= 0 ? tr_neighbor(g, src, tr.pair_mask, tr_rand(tr.rng, kTrStreamPos, static_cast<uint64_t>(t)))
                    : -1;
  }
  return tr_root(g, tr.rng, t, kTrStreamNeg);
}

// node of slot s at level lv (0..2); *root = index of its root, *self_chain = the slot is
// the root itself (every digit is the self slot)
__device__ int32_t tr_slot_node(const TrGraph& g, const TrTree& tr, int64_t s, int lv, int64_t* root,
                                bool* self_chain) {
  int64_t i0 = s, i1 = 0, i2 = 0;
  if (lv == 1) {
    i1 = s;
    i0 = s >> tr.logP1;
  } else if (lv == 2) {
    i2 = s;
    i1 = s >> tr.logP2;
    i0 = i1 >> tr.logP1;
  }
  int32_t node = tr_tree_root(g, tr, i0);
  bool sc = true;
  if (lv >= 1) {
    const int j = static_cast<int>(i1 & ((int64_t(1) << tr.logP1) - 1));
    sc = j == tr.F1;
    node = tr_hop(g, tr.rng, node, j, tr.F1, tr.m1, 1, i0, tr.stream_off);
  }
  if (lv >= 2) {
    const int j = static_cast<int>(i2 & ((int64_t(1) << tr.logP2) - 1));
    sc = sc && j == tr.F2;
    node = tr_hop(g, tr.rng, node, j, tr.F2, tr.m2, 2, i1, tr.stream_off);
  }
  *root = i0;
  *self_chain = sc;
  return node;
}

__device__ __forceinline__ float bf_lo(uint32_t v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(uint32_t v) { return __uint_as_float(v & 0xffff0000u); }

// 8 consecutive feature columns of one row, bf16 or fp32 storage
template <typename FT>
struct Feat8;
template <>
struct Feat8<bf16_t> {
  static constexpr int kInFlight = 10;  // rows in flight per thread and item
  uint4_t v;
  __device__ __forceinline__ void load(const bf16_t* p) { v = *reinterpret_cast<const uint4_t*>(p); }
  __device__ __forceinline__ void zero() { v = uint4_t{0u, 0u, 0u, 0u}; }
  __device__ __forceinline__ void add_to(float* acc) const { acc_bf16x8(acc, v); }
  __device__ __forceinline__ void add_scaled_to(float* acc, float w) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[2 * i] += w * bf_lo(v[i]);
      acc[2 * i + 1] += w * bf_hi(v[i]);
    }
  }
  // keep = false: the row was a padding id (-1) loaded from row 0; contributes zero
  __device__ __forceinline__ void keep(bool k) {
#pragma unroll
    for (int i = 0; i < 4; ++i) v[i] = k ? v[i] : 0u;
  }
  __device__ __forceinline__ uint4_t bf16() const { return v; }
};
template <>
struct Feat8<float> {
  static constexpr int kInFlight = 5;
  float4_t a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = *reinterpret_cast<const float4_t*>(p);
    b = *reinterpret_cast<const float4_t*>(p + 4);
  }
  __device__ __forceinline__ void zero() { a = b = float4_t{0.f, 0.f, 0.f, 0.f}; }
  __device__ __forceinline__ void add_to(float* acc) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i] += a[i];
      acc[4 + i] += b[i];
    }
  }
  __device__ __forceinline__ void add_scaled_to(float* acc, float w) const {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      acc[i] += w * a[i];
      acc[4 + i] += w * b[i];
    }
  }
  __device__ __forceinline__ void keep(bool k) {
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      a[i] = k ? a[i] : 0.f;
      b[i] = k ? b[i] : 0.f;
    }
  }
  __device__ __forceinline__ uint4_t bf16() const {
    float t[8] = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return pack_bf16x8(t);
  }
};

// ----------------------------------------------------------------------------
// combination tiles, computed by wave 0 of the forward launch's tile blocks before their
// own work (the MFMA units are idle during the gather): Wc = Wout Wfc as 16 x 16 MFMA
// tiles of the bf16 fm shadows (an fm fragment of Wout [C][E] is also a valid A fragment:
// lane l holds row l & 15, k 8(l >> 4)..+7), all E/32 fragment pairs of a tile in
// flight; bc = Wout bfc in fp32 from the masters (one row per block).  No extra blocks:
// extra blocks would push tile blocks past the resident slots into a second round.
// ----------------------------------------------------------------------------
__device__ __forceinline__ void tr_comb_wave(const TrCombArgs& c, int first, int stride, int lane) {
  const int tcols = c.H >> 4, ntiles = (c.C >> 4) * tcols;
  for (int t = first; t < ntiles; t += stride) {
    const int c0 = (t / tcols) * 16, h0 = (t % tcols) * 16;
    float4_t acc = float4_t{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < c.E; k0 += 128) {  // 4 fragment pairs in flight (register budget of the host kernel)
      uint4_t av[4], bv[4];
#pragma unroll
      for (int s = 0; s < 4; ++s) {
        const int k = k0 + s * 32 < c.E ? k0 + s * 32 : 0;
        av[s] = fm_frag(c.wout_sh, c0, k, c.E, lane);
        bv[s] = fm_frag(c.wfcT_sh, h0, k, c.E, lane);
      }
#pragma unroll
      for (int s = 0; s < 4; ++s)
        if (k0 + s * 32 < c.E) acc = mfma16(av[s], bv[s], acc);
    }
    const int h = h0 + (lane & 15);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = c0 + (lane >> 4) * 4 + j;
      c.Wc[fm_off(r, h, c.H)] = f2bf(acc[j]);
      c.WcT[fm_off(h, r, c.C)] = f2bf(acc[j]);
    }
  }
  // bc = Wout bfc in fp32: one row per block (rows strided over the blocks like the tiles),
  // the wave's lanes split E and reduce by shuffles.  (One row per lane with a serial loop
  // over E made block 0 a 25 us straggler: 256 dependent-issue global loads per lane.)
  for (int r = first; r < c.C; r += stride) {
    const float* w = c.wout + static_cast<int64_t>(r) * c.E;
    float b = 0.f;
    for (int e = lane; e < c.E; e += 64) b += w[e] * c.bfc[e];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) b += __shfl_xor(b, o, 64);
    if (lane == 0) c.bc[r] = b;
  }
}

// ----------------------------------------------------------------------------
// tr_sample: target-row nodes (root -> hop chain) and their leaf draws, BM rows per block
// ----------------------------------------------------------------------------
constexpr int kTrSampleRows = 64;

// one sampler block of NT threads: NT / 4 target rows (root -> hop chain by the first
// NT / 4 threads, then every thread draws leaves)
template <int NT>
__device__ __forceinline__ void tr_sample_block(const TrSampleArgs& a, int blk, int32_t* node_s) {
  constexpr int R = NT / 4;
  const int64_t row0 = static_cast<int64_t>(blk) * R;
  if (threadIdx.x < R) {
    const int64_t s = row0 + threadIdx.x;
    int32_t node = -1;
    if (s < a.M) {
      int64_t root;
      bool sc;
      node = tr_slot_node(a.g, a.tr, s, a.lv, &root, &sc);
      if (sc) a.roots[root] = node;
      a.nodes[s] = node;
    }
    node_s[threadIdx.x] = node;
  }
  __syncthreads();
  for (int it = threadIdx.x; it < R * a.FL; it += NT) {
    const int r = it / a.FL, k = it - r * a.FL;
    const int64_t s = row0 + r;
    if (s >= a.M) break;
    const int32_t node = node_s[r];
    a.leaf[s * a.FL + k] =
        node >= 0 ? tr_neighbor(a.g, node, a.mL,
                                tr_rand(a.tr.rng, kTrStreamHop + a.hopL + a.tr.stream_off,
                                        static_cast<uint64_t>(s * a.FL + k)))
                  : -1;
  }
}

__global__ __launch_bounds__(256) void tr_sample_kernel(TrSampleArgs a) {
  __shared__ int32_t node_s[kTrSampleRows];
  tr_sample_block<256>(a, blockIdx.x, node_s);
}

// ----------------------------------------------------------------------------
// tr_fwd: one SAGE layer over BM target rows per block (see TrFwdArgs)
// ----------------------------------------------------------------------------
#ifndef TR_FWD_WAVES
#define TR_FWD_WAVES 4
#endif
#ifndef TR_FWD_BPF
#define TR_FWD_BPF 2
#endif
template <typename FT, int BM, int MODE>
__global__ __launch_bounds__(256, (BM == 32 ? TR_FWD_WAVES : 2)) void tr_fwd_kernel(TrFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  constexpr bool kGather = MODE != 2;
  const int tb = static_cast<int>(blockIdx.x), ntb = static_cast<int>(gridDim.x);
  if (a.ncomb && threadIdx.x < 64) tr_comb_wave(a.comb, tb, ntb, threadIdx.x);  // the head's Wc
  const int D = a.D;
  const int K2 = 2 * D;
  const int ldsw = K2 + 8;
  const int tile = xcd_remap(tb, ntb);
  const int64_t row0 = static_cast<int64_t>(tile) * BM;
  const int H = a.H;
  const bool alias_out = H <= kTrBN && kTrBN <= K2;
  // LDS: [BM][ldsw] A tile | [BM][kTrBN + 8] output tile (modes 0/2, unless it aliases the
  // A tile) | node ids [BM] + leaf ids [BM][FL] (modes 0/1); must match eh_tr_fwd_lds
  const bool own_otile = MODE != 1 && !alias_out;
  bf16_t* otile = own_otile ? lds + BM * ldsw : lds;
  int32_t* node_s = reinterpret_cast<int32_t*>(lds + BM * ldsw + (own_otile ? BM * (kTrBN + 8) : 0));
  int32_t* leaf_s = node_s + BM;

#define TF_STAMP(k) \
  if (a.prof && threadIdx.x == 0) a.prof[tb * 8 + (k)] = static_cast<long long>(wall_clock64())
  TF_STAMP(0);
  constexpr int FN = 4;
  constexpr int kBP = TR_FWD_BPF;  // k-steps of weight fragments in flight
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const bf16_t* W = a.W;
  uint4_t bq[kBP][FN];
  if constexpr (kGather) {
    // ---- the sampled ids of the block (sampler output, one step ahead): coalesced
    if (tb == 0 && threadIdx.x == 0) {
      if (a.step) a.step[0] += 1;
      a.rng[1] += 1;  // this batch is consumed: the sampler draws the next counter
    }
    for (int i = tb * 256 + threadIdx.x; i < a.B; i += ntb * 256) a.roots_cur[i] = a.roots_in[i];
    if (threadIdx.x < BM) node_s[threadIdx.x] = row0 + threadIdx.x < a.M ? a.nodes[row0 + threadIdx.x] : -1;
    for (int it = threadIdx.x; it < BM * a.FL; it += 256)
      leaf_s[it] = row0 * a.FL + it < a.M * a.FL ? a.leaf[row0 * a.FL + it] : -1;
    __syncthreads();
    TF_STAMP(1);
    // ---- gather + mean: item = (row, 8-column chunk); two items per thread with every
    // leaf load of both in flight
    const FT* x = static_cast<const FT*>(a.x);
    const int cpr = D >> 3;
    const int nitems = BM * cpr;
    constexpr int G = Feat8<FT>::kInFlight;
    for (int it = threadIdx.x; it < nitems; it += 512) {
      const int itb = it + 256;
      const bool hb = itb < nitems;
      const int ra = it / cpr, ca = it - ra * cpr;
      const int rb = hb ? itb / cpr : ra, cb = hb ? itb - rb * cpr : ca;
      const int32_t na = node_s[ra], nb = hb ? node_s[rb] : -1;
      // branch-free loads: a padding id (-1) reads row 0 and is zeroed at use, so no
      // divergent branch forces the compiler to wait on each load (vmcnt(0))
      Feat8<FT> sa, sb;
      float acc_a[8], acc_b[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) acc_a[i] = acc_b[i] = 0.f;
      sa.load(x + static_cast<int64_t>(na > 0 ? na : 0) * D + ca * 8);
      sb.load(x + static_cast<int64_t>(nb > 0 ? nb : 0) * D + cb * 8);
      for (int k = 0; k < a.FL; k += G) {
        int32_t ja[G], jb[G];
        Feat8<FT> va[G], vb[G];
#pragma unroll
        for (int u = 0; u < G; ++u) {
          ja[u] = (k + u < a.FL) ? leaf_s[ra * a.FL + k + u] : -1;
          jb[u] = (hb && k + u < a.FL) ? leaf_s[rb * a.FL + k + u] : -1;
        }
        // unconditional: slots past FL (ids -1) re-read the L2-resident row 0
#pragma unroll
        for (int u = 0; u < G; ++u) {
          va[u].load(x + static_cast<int64_t>(ja[u] > 0 ? ja[u] : 0) * D + ca * 8);
          vb[u].load(x + static_cast<int64_t>(jb[u] > 0 ? jb[u] : 0) * D + cb * 8);
        }
#pragma unroll
        for (int u = 0; u < G; ++u) {
          va[u].keep(ja[u] >= 0);
          vb[u].keep(jb[u] >= 0);
          va[u].add_to(acc_a);
          vb[u].add_to(acc_b);
        }
      }
      sa.keep(na >= 0);
      sb.keep(nb >= 0);
      if (a.include_self) {
        sa.add_to(acc_a);
        sb.add_to(acc_b);
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        acc_a[i] *= a.inv_leaf;
        acc_b[i] *= a.inv_leaf;
      }
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        if (h == 1 && !hb) break;
        const int r = h ? rb : ra, c = h ? cb : ca;
        const uint4_t selfv = h ? sb.bf16() : sa.bf16(), meanv = pack_bf16x8(h ? acc_b : acc_a);
        const int64_t grow = row0 + r;
        if constexpr (MODE == 1) {
          if (grow < a.M) {
            *reinterpret_cast<uint4_t*>(a.a_next + grow * K2 + c * 8) = selfv;
            *reinterpret_cast<uint4_t*>(a.a_next + grow * K2 + D + c * 8) = meanv;
          }
        } else {
          *reinterpret_cast<uint4_t*>(lds + r * ldsw + c * 8) = selfv;
          *reinterpret_cast<uint4_t*>(lds + r * ldsw + D + c * 8) = meanv;
        }
      }
    }
    if constexpr (MODE == 1) return;
  } else {
    // ---- rows: BM rows of A [M][K2] (bf16) into the tile
    const bf16_t* A = static_cast<const bf16_t*>(a.x);
    const int cpr = K2 >> 3;
    for (int it = threadIdx.x; it < BM * cpr; it += 256) {
      const int r = it / cpr, c = it - r * cpr;
      const int64_t grow = row0 + r;
      const uint4_t v = grow < a.M ? *reinterpret_cast<const uint4_t*>(A + grow * K2 + c * 8) : uint4_t{0u, 0u, 0u, 0u};
      *reinterpret_cast<uint4_t*>(lds + r * ldsw + c * 8) = v;
    }
  }
  // the GEMM's first kBP k-steps of B fragments (weights: L2-resident) load behind the kt
  // pass; the loop below keeps kBP steps in flight (a weight-fragment load from L2 takes
  // longer than one step's MFMAs, so one step ahead leaves the chain latency-bound)
  if constexpr (MODE != 1) {
    if (wave * 64 < a.H) {
#pragma unroll
      for (int q = 0; q < kBP; ++q)
#pragma unroll
        for (int n = 0; n < FN; ++n) bq[q][n] = fm_frag(W, wave * 64 + n * 16, q * 32 < K2 ? q * 32 : 0, K2, lane);
    }
  }
  __syncthreads();
  TF_STAMP(2);

  // ---- A tile -> kt layout (dW operand): item = (column pair, 8-row chunk q), column
  // pairs fastest so a wave's 4-byte LDS reads cover consecutive banks
  if (a.a_kt) {
    constexpr int CH = BM / 8;
    const int np = K2 >> 1;
    for (int it = threadIdx.x; it < np * CH; it += 256) {
      const int q = it / np;
      const int n = (it - q * np) * 2;
      const int64_t gr = row0 + q * 8;
      if (gr >= a.M) continue;
      uint32_t w[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) w[i] = *reinterpret_cast<const uint32_t*>(lds + (q * 8 + i) * ldsw + n);
      uint4_t lo, hi;
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        lo[i] = (w[2 * i] & 0xffffu) | (w[2 * i + 1] << 16);
        hi[i] = (w[2 * i] >> 16) | (w[2 * i + 1] & 0xffff0000u);
      }
      *reinterpret_cast<uint4_t*>(a.a_kt + kt_off(gr, n, K2)) = lo;
      *reinterpret_cast<uint4_t*>(a.a_kt + kt_off(gr, n + 1, K2)) = hi;
    }
  }

  TF_STAMP(3);
  // ---- MFMA GEMM out of LDS; wave w owns 64-column slab w of each 256-column chunk
  constexpr int FM = BM / 16;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  const int ldo = kTrBN + 8;
  for (int cchunk = 0; cchunk < H; cchunk += kTrBN) {
    const int cb = cchunk + wave * 64;
    float4_t acc[FM][FN];
    tl_zero(acc);
    if (cb < H) {
      if (cchunk > 0) {
#pragma unroll
        for (int q = 0; q < kBP; ++q)
#pragma unroll
          for (int n = 0; n < FN; ++n) bq[q][n] = fm_frag(W, cb + n * 16, q * 32 < K2 ? q * 32 : 0, K2, lane);
      }
      // kBP steps per iteration, ring slot q holds step k0 + 32 q; after its MFMAs the slot
      // is refilled with step k0 + 32 (q + kBP) (clamped to a valid fragment past the end)
      for (int k0 = 0; k0 < K2; k0 += 32 * kBP) {
#pragma unroll
        for (int q = 0; q < kBP; ++q) {
          const int ks = k0 + 32 * q;
          if (ks >= K2) break;  // uniform
          uint4_t av[FM];
#pragma unroll
          for (int m = 0; m < FM; ++m)
            av[m] = *reinterpret_cast<const uint4_t*>(lds + (m * 16 + lr) * ldsw + ks + lk);
#pragma unroll
          for (int m = 0; m < FM; ++m)
#pragma unroll
            for (int n = 0; n < FN; ++n) acc[m][n] = mfma16(av[m], bq[q][n], acc[m][n]);
          const int kn = ks + 32 * kBP;
#pragma unroll
          for (int n = 0; n < FN; ++n) bq[q][n] = fm_frag(W, cb + n * 16, kn < K2 ? kn : 0, K2, lane);
        }
      }
    }
    if (alias_out) __syncthreads();  // every wave is done reading the A tile
    if (cb < H) {
#pragma unroll
      for (int m = 0; m < FM; ++m)
#pragma unroll
        for (int n = 0; n < FN; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = m * 16 + (lane >> 4) * 4 + j;
            otile[row * ldo + wave * 64 + n * 16 + lr] = f2bf(fmaxf(acc[m][n][j], 0.f));
          }
    }
    __syncthreads();
    TF_STAMP(4);
    const int ncols = (H - cchunk) < kTrBN ? (H - cchunk) : kTrBN;
    // tree-mean epilogue: A_next[parent] = [h[self slot] | mean_{j < Fg} h[j]] for every
    // sibling group of the block (item = (group, column pair), 4-byte stores)
    {
      const int groups = BM >> a.logPg;
      const int pairs = ncols >> 1;
      for (int it = threadIdx.x; it < groups * pairs; it += 256) {
        const int gi = it / pairs;
        const int c = (it - gi * pairs) * 2;
        const int base = gi << a.logPg;
        if (row0 + base >= a.M) continue;
        const uint32_t selfp = *reinterpret_cast<const uint32_t*>(otile + (base + a.Fg) * ldo + c);
        float s0 = 0.f, s1 = 0.f;
        for (int j = 0; j < a.Fg; ++j) {
          const uint32_t v = *reinterpret_cast<const uint32_t*>(otile + (base + j) * ldo + c);
          s0 += bf_lo(v);
          s1 += bf_hi(v);
        }
        if (a.include_self) {
          s0 += bf_lo(selfp);
          s1 += bf_hi(selfp);
        }
        const int64_t parent = (row0 >> a.logPg) + gi;
        bf16_t* dst = a.a_next + parent * 2 * H + cchunk + c;
        *reinterpret_cast<uint32_t*>(dst) = selfp;
        *reinterpret_cast<uint32_t*>(dst + H) = pack_bf16x2(s0 * a.inv_grp, s1 * a.inv_grp);
      }
    }
    // ReLU bits for the backward: word (32-row block, column) has bit i set iff row i > 0
    if (a.mask) {
      constexpr int KBB = BM / 32;
      for (int it = threadIdx.x; it < KBB * ncols; it += 256) {
        const int kbl = it / ncols, n = it - kbl * ncols;
        const int64_t gr = row0 + kbl * 32;
        if (gr >= a.M) continue;
        uint32_t bits = 0;
#pragma unroll
        for (int i = 0; i < 32; ++i) bits |= (bf_pos(otile[(kbl * 32 + i) * ldo + n]) ? 1u : 0u) << i;
        a.mask[(gr >> 5) * H + cchunk + n] = bits;
      }
    }
    __syncthreads();
  }
  TF_STAMP(5);
#undef TF_STAMP
}

// ----------------------------------------------------------------------------
// tr_fwd2: layer 0 (mode 0) with 64 target rows and 8 waves per block.  Versus
// tr_fwd_kernel<BM=32> (4 waves, each 64 columns x 32 rows):
//   * every wave multiplies all 64 rows by its 32 columns, so a weight fragment fetched
//     from L2 serves 64 rows instead of 32 (the GEMM phase was bound by re-fetching W
//     per 32 rows: 800 blocks x 128 KB);
//   * the A tile has no padding; 16-B chunk c of row r lives at chunk c ^ (r & 15), so
//     each ds_read_b128 lane group ({0-3,12-15,20-27}, ...: rows 0-15 x k-quarters 0/1
//     or 2/3) touches 16 distinct 16-B bank slots (the padded layout put two lanes of a
//     group on one slot: a 2-way conflict on every fragment read);
//   * the ReLU'd output goes to LDS transposed ([column][row], row stride 68 bf16 =
//     34 dwords): one 8-byte store per lane per MFMA tile instead of four 2-byte ones,
//     and the tree-mean / ReLU-bit epilogue reads whole 4-row words (ds_read_b64), all
//     bank-conflict-free (34c mod 64 is distinct for the 32 lanes of a half-wave).
// Needs D % 64 == 0 (A rows of a multiple of 16 chunks), M % 64 == 0 and sibling groups
// of at most 64 rows (else tr_fwd_kernel).
// ----------------------------------------------------------------------------
constexpr int kF2Rows = 64, kF2Threads = 512, kF2Ldt = kF2Rows + 4;
// F2_ALIAS=1: the output tile aliases the A tile (one region of max(A, O) bytes, a barrier
// between the last A read and the first O write): ~38 KB of LDS per block instead of ~70 KB
#ifndef F2_ALIAS
#define F2_ALIAS 1
#endif
#ifndef F2_SKIP_PAD
#define F2_SKIP_PAD 1
#endif
// k-steps of weight fragments in flight in the GEMM (2 per wave = 16 VGPRs, 4 = 32)
#ifndef F2_WPF
#define F2_WPF 4
#endif

__device__ __forceinline__ int f2_chunk(int r, int c) { return c ^ (r & 15); }

// gather + mean of BM target rows into the swizzled LDS tile At [BM][2D] (see tr_fwd2):
// item = (used row, 8-column chunk), two items per thread, every leaf load of both in
// flight; padding ids (-1) read row 0 and are zeroed at use; only the Fg + 1 used slots of
// each sibling group are gathered (F2_SKIP_PAD), the unused slots' rows are zero-filled.
template <typename FT, int BM, int NT>
__device__ __forceinline__ void f2_gather(const TrFwdArgs& a, bf16_t* At, const int32_t* node_s,
                                          const int32_t* leaf_s, int tid) {
  const int D = a.D, K2 = 2 * D;
  const FT* x = static_cast<const FT*>(a.x);
  const int cpr = D >> 3;
  const int P = 1 << a.logPg, U = F2_SKIP_PAD ? a.Fg + 1 : P;
  const int nitems = (BM >> a.logPg) * U * cpr;
  constexpr int G = Feat8<FT>::kInFlight;
  if (F2_SKIP_PAD && U < P) {
    const int pad = P - U, nch = K2 >> 3;
    for (int it = tid; it < (BM >> a.logPg) * pad * nch; it += NT) {
      const int q = it / nch, c = it - q * nch;
      const int r = (q / pad) * P + U + q % pad;
      *reinterpret_cast<uint4_t*>(At + r * K2 + f2_chunk(r, c) * 8) = uint4_t{0u, 0u, 0u, 0u};
    }
  }
  for (int it = tid; it < nitems; it += 2 * NT) {
    const int itb = it + NT;
    const bool hb = itb < nitems;
    const int qa = it / cpr, ca = it - qa * cpr;
    const int qb = hb ? itb / cpr : qa, cb = hb ? itb - qb * cpr : ca;
    const int ra = (qa / U) * P + qa % U, rb = (qb / U) * P + qb % U;
    const int32_t na = node_s[ra], nb = hb ? node_s[rb] : -1;
    Feat8<FT> sa, sb;
    float acc_a[8], acc_b[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc_a[i] = acc_b[i] = 0.f;
    sa.load(x + static_cast<int64_t>(na > 0 ? na : 0) * D + ca * 8);
    sb.load(x + static_cast<int64_t>(nb > 0 ? nb : 0) * D + cb * 8);
    for (int k = 0; k < a.FL; k += G) {
      int32_t ja[G], jb[G];
      Feat8<FT> va[G], vb[G];
#pragma unroll
      for (int u = 0; u < G; ++u) {
        ja[u] = (k + u < a.FL) ? leaf_s[ra * a.FL + k + u] : -1;
        jb[u] = (hb && k + u < a.FL) ? leaf_s[rb * a.FL + k + u] : -1;
      }
#pragma unroll
      for (int u = 0; u < G; ++u) {
        va[u].load(x + static_cast<int64_t>(ja[u] > 0 ? ja[u] : 0) * D + ca * 8);
        vb[u].load(x + static_cast<int64_t>(jb[u] > 0 ? jb[u] : 0) * D + cb * 8);
      }
#pragma unroll
      for (int u = 0; u < G; ++u) {
        va[u].keep(ja[u] >= 0);
        vb[u].keep(jb[u] >= 0);
        va[u].add_to(acc_a);
        vb[u].add_to(acc_b);
      }
    }
    sa.keep(na >= 0);
    sb.keep(nb >= 0);
    if (a.include_self) {
      sa.add_to(acc_a);
      sb.add_to(acc_b);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      acc_a[i] *= a.inv_leaf;
      acc_b[i] *= a.inv_leaf;
    }
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      if (h == 1 && !hb) break;
      const int r = h ? rb : ra, c = h ? cb : ca;
      *reinterpret_cast<uint4_t*>(At + r * K2 + f2_chunk(r, c) * 8) = h ? sb.bf16() : sa.bf16();
      *reinterpret_cast<uint4_t*>(At + r * K2 + f2_chunk(r, cpr + c) * 8) = pack_bf16x8(h ? acc_b : acc_a);
    }
  }
}

// the A tile -> kt layout (dW operand): item = (column pair, 8-row chunk), column pairs
// fastest: a half-wave's 4-byte reads cover 128 contiguous (permuted) bytes of a row
template <int BM, int NT>
__device__ __forceinline__ void f2_kt(const TrFwdArgs& a, int64_t row0, const bf16_t* At, int tid) {
  const int K2 = 2 * a.D;
  const int np = K2 >> 1;
  for (int it = tid; it < np * (BM / 8); it += NT) {
    const int q = it / np;
    const int n = (it - q * np) * 2;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int r = q * 8 + i;
      w[i] = *reinterpret_cast<const uint32_t*>(At + r * K2 + f2_chunk(r, n >> 3) * 8 + (n & 7));
    }
    uint4_t lo, hi;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = (w[2 * i] & 0xffffu) | (w[2 * i + 1] << 16);
      hi[i] = (w[2 * i] >> 16) | (w[2 * i + 1] & 0xffff0000u);
    }
    *reinterpret_cast<uint4_t*>(a.a_kt + kt_off(row0 + q * 8, n, K2)) = lo;
    *reinterpret_cast<uint4_t*>(a.a_kt + kt_off(row0 + q * 8, n + 1, K2)) = hi;
  }
}

// one 32-row gather tile of the pipelined step (extra blocks of the optimizer launch, 256
// threads): ids -> gather + mean -> LDS -> kt copy (dW operand) + row-major A rows (the
// GEMM-only forward's input).  LDS: A tile [32][2D] + ids (eh_tr_gather32_lds).
constexpr int kG32Rows = 32, kG32Threads = 256;

template <typename FT>
__device__ __forceinline__ void tr_gather32_tile(const TrFwdArgs& a, int tile, bf16_t* lds) {
  constexpr int BM = kG32Rows, NT = kG32Threads;
  const int K2 = 2 * a.D, tid = threadIdx.x;
  const int64_t row0 = static_cast<int64_t>(tile) * BM;
  bf16_t* At = lds;
  int32_t* node_s = reinterpret_cast<int32_t*>(lds + BM * K2);
  int32_t* leaf_s = node_s + BM;
  if (tid < BM) node_s[tid] = a.nodes[row0 + tid];
  for (int it = tid; it < BM * a.FL; it += NT) leaf_s[it] = a.leaf[row0 * a.FL + it];
  __syncthreads();
  f2_gather<FT, BM, NT>(a, At, node_s, leaf_s, tid);
  __syncthreads();
  f2_kt<BM, NT>(a, row0, At, tid);
  const int cpr2 = K2 >> 3;
  for (int it = tid; it < BM * cpr2; it += NT) {
    const int r = it / cpr2, c = it - r * cpr2;
    *reinterpret_cast<uint4_t*>(a.a_rows + (row0 + r) * K2 + c * 8) =
        *reinterpret_cast<const uint4_t*>(At + r * K2 + f2_chunk(r, c) * 8);
  }
}

// GO = 1 (pipelined step, mode 3): the gather already ran in the previous launch (gather
// blocks of tr_opt, tr_gather32_tile): the A tile is loaded from a.a_rows and the kt copy
// for dW exists; only the GEMM, the tree mean, the ReLU bits and the head's Wc remain.
template <typename FT, int GO>
__global__ __launch_bounds__(kF2Threads, 4) void tr_fwd2_kernel(TrFwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  constexpr int BM = kF2Rows, NT = kF2Threads;
  const int tb = static_cast<int>(blockIdx.x), ntb = static_cast<int>(gridDim.x);
  const int D = a.D, K2 = 2 * D, H = a.H;
  const int tile = xcd_remap(tb, ntb);
  const int64_t row0 = static_cast<int64_t>(tile) * BM;
  // LDS: A tile [BM][K2] (swizzled) | output tile [kTrBN][kF2Ldt] (transposed) | ids
  bf16_t* At = lds;
#if F2_ALIAS
  bf16_t* Ot = lds;
  int32_t* node_s = reinterpret_cast<int32_t*>(lds + (BM * K2 > kTrBN * kF2Ldt ? BM * K2 : kTrBN * kF2Ldt));
#else
  bf16_t* Ot = lds + BM * K2;
  int32_t* node_s = reinterpret_cast<int32_t*>(Ot + kTrBN * kF2Ldt);
#endif
  int32_t* leaf_s = node_s + BM;
#define F2_STAMP(k) \
  if (a.prof && threadIdx.x == 0) a.prof[tb * 8 + (k)] = static_cast<long long>(wall_clock64())
  F2_STAMP(0);
  if (a.prof && threadIdx.x == 0) a.prof[tb * 8 + 6] = static_cast<long long>(__smid());  // XCC / SE / CU
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lg = lane >> 4;
  if (tb == 0 && tid == 0) {
    if (a.step) a.step[0] += 1;
    a.rng[1] += 1;  // this batch is consumed: the sampler draws the next counter
  }
  for (int i = tb * NT + tid; i < a.B; i += ntb * NT) a.roots_cur[i] = a.roots_in[i];
  if constexpr (GO) {
    // A rows [64][K2] (row-major, 16-byte chunks) -> the swizzled LDS tile
    const int cpr2 = K2 >> 3;
    for (int it = tid; it < BM * cpr2; it += NT) {
      const int r = it / cpr2, c = it - r * cpr2;
      *reinterpret_cast<uint4_t*>(At + r * K2 + f2_chunk(r, c) * 8) =
          *reinterpret_cast<const uint4_t*>(a.a_rows + (row0 + r) * K2 + c * 8);
    }
  } else {
    if (tid < BM) node_s[tid] = a.nodes[row0 + tid];
    for (int it = tid; it < BM * a.FL; it += NT) leaf_s[it] = a.leaf[row0 * a.FL + it];
    __syncthreads();
  }
  F2_STAMP(1);
  // ---- gather + mean: item = (used row, 8-column chunk); two items per thread, every leaf
  // load of both in flight; padding ids (-1) read row 0 and are zeroed at use.  Only the
  // Fg + 1 used slots of each sibling group are items (F2_SKIP_PAD; at fanout 25, 26 of
  // every 32 rows): the unused slots' A rows are zero-filled instead of gathered.
  if constexpr (!GO) f2_gather<FT, BM, NT>(a, At, node_s, leaf_s, tid);
  // the head's Wc tiles (wave 0, after the gather: its registers are free again)
  if (a.ncomb && wave == 0) tr_comb_wave(a.comb, tb, ntb, lane);
  // the first WPF k-steps of this wave's weight fragments load behind the kt pass (not
  // earlier: held through the gather they would push its 20 row loads in flight to spill)
  const bf16_t* W = a.W;
  constexpr int WPF = F2_WPF;
  uint4_t bq[WPF][2];
  if (wave * 32 < H) {
#pragma unroll
    for (int q = 0; q < WPF; ++q)
#pragma unroll
      for (int n = 0; n < 2; ++n) bq[q][n] = fm_frag(W, wave * 32 + n * 16, q * 32 < K2 ? q * 32 : 0, K2, lane);
  }
  __syncthreads();
  F2_STAMP(2);
  // ---- A tile -> kt layout (dW operand): item = (column pair, 8-row chunk), column pairs
  // fastest: a half-wave's 4-byte reads cover 128 contiguous (permuted) bytes of a row
  if constexpr (!GO) f2_kt<BM, NT>(a, row0, At, tid);
  F2_STAMP(3);
  // ---- MFMA GEMM out of LDS: wave w owns columns w*32..+31 of each 256-column chunk, all
  // 64 rows; two k-steps of weight fragments in flight
  constexpr int FM = BM / 16, FN = 2;
  for (int cchunk = 0; cchunk < H; cchunk += kTrBN) {
    const int cb = cchunk + wave * 32;
    float4_t acc[FM][FN];
    tl_zero(acc);
    if (cb < H) {
      if (cchunk > 0) {
#pragma unroll
        for (int q = 0; q < WPF; ++q)
#pragma unroll
          for (int n = 0; n < FN; ++n) bq[q][n] = fm_frag(W, cb + n * 16, q * 32 < K2 ? q * 32 : 0, K2, lane);
      }
      for (int k0 = 0; k0 < K2; k0 += 32 * WPF) {
#pragma unroll
        for (int q = 0; q < WPF; ++q) {
          const int ks = k0 + 32 * q;
          if (ks >= K2) break;  // uniform
          uint4_t av[FM];
          const int phys = f2_chunk(lr, (ks >> 3) + lg) * 8;
#pragma unroll
          for (int m = 0; m < FM; ++m) av[m] = *reinterpret_cast<const uint4_t*>(At + (m * 16 + lr) * K2 + phys);
#pragma unroll
          for (int m = 0; m < FM; ++m)
#pragma unroll
            for (int n = 0; n < FN; ++n) acc[m][n] = mfma16(av[m], bq[q][n], acc[m][n]);
          const int kn = ks + 32 * WPF;
#pragma unroll
          for (int n = 0; n < FN; ++n) bq[q][n] = fm_frag(W, cb + n * 16, kn < K2 ? kn : 0, K2, lane);
        }
      }
    }
#if F2_ALIAS
    __syncthreads();  // every wave is done reading the A tile the output tile overwrites
#endif
    if (cb < H) {
      // ReLU -> transposed output tile: 4 consecutive rows of one column per 8-byte store
#pragma unroll
      for (int m = 0; m < FM; ++m)
#pragma unroll
        for (int n = 0; n < FN; ++n) {
          tl_uint2 v;
          v[0] = pack_bf16x2(fmaxf(acc[m][n][0], 0.f), fmaxf(acc[m][n][1], 0.f));
          v[1] = pack_bf16x2(fmaxf(acc[m][n][2], 0.f), fmaxf(acc[m][n][3], 0.f));
          *reinterpret_cast<tl_uint2*>(Ot + (wave * 32 + n * 16 + lr) * kF2Ldt + m * 16 + lg * 4) = v;
        }
    }
    __syncthreads();
    F2_STAMP(4);
    const int ncols = (H - cchunk) < kTrBN ? (H - cchunk) : kTrBN;
    // tree-mean epilogue: item = (sibling group, column); the group's rows are contiguous
    // in the column's LDS row: 8-byte reads of 4 rows
    {
      const int P = 1 << a.logPg;
      const int groups = BM >> a.logPg;
      for (int it = tid; it < groups * ncols; it += NT) {
        const int gi = it / ncols, c = it - gi * ncols;
        const bf16_t* col = Ot + c * kF2Ldt + (gi << a.logPg);
        float s = 0.f, self = 0.f;
        for (int r4 = 0; r4 < P; r4 += 4) {
          const tl_uint2 v = *reinterpret_cast<const tl_uint2*>(col + r4);
          const float e[4] = {bf_lo(v[0]), bf_hi(v[0]), bf_lo(v[1]), bf_hi(v[1])};
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int r = r4 + j;
            s += r < a.Fg ? e[j] : 0.f;
            self = r == a.Fg ? e[j] : self;
          }
        }
        if (a.include_self) s += self;
        const int64_t parent = (row0 >> a.logPg) + gi;
        bf16_t* dst = a.a_next + parent * 2 * H + cchunk + c;
        dst[0] = f2bf(self);
        dst[H] = f2bf(s * a.inv_grp);
      }
    }
    // ReLU bits for the backward: word (32-row block, column) has bit i set iff row i > 0
    if (a.mask) {
      for (int it = tid; it < (BM / 32) * ncols; it += NT) {
        const int kbl = it / ncols, c = it - kbl * ncols;
        const bf16_t* col = Ot + c * kF2Ldt + kbl * 32;
        uint32_t bits = 0;
#pragma unroll
        for (int r4 = 0; r4 < 32; r4 += 4) {
          const tl_uint2 v = *reinterpret_cast<const tl_uint2*>(col + r4);
          bits |= (bf_pos(static_cast<bf16_t>(v[0] & 0xffffu)) ? 1u : 0u) << r4;
          bits |= (bf_pos(static_cast<bf16_t>(v[0] >> 16)) ? 1u : 0u) << (r4 + 1);
          bits |= (bf_pos(static_cast<bf16_t>(v[1] & 0xffffu)) ? 1u : 0u) << (r4 + 2);
          bits |= (bf_pos(static_cast<bf16_t>(v[1] >> 16)) ? 1u : 0u) << (r4 + 3);
        }
        a.mask[((row0 >> 5) + kbl) * H + cchunk + c] = bits;
      }
    }
    __syncthreads();
  }
  F2_STAMP(5);
#undef F2_STAMP
}

// ----------------------------------------------------------------------------
// tr_bwd (3-hop inner layer): G rows routed from the parent gradient through the tree
// and the ReLU bits, then dA_out = G @ W (fp32 rows)
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void tr_bwd_kernel(TrBwdArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  constexpr int BM = 32;
  const int Hk = a.Hk, K2 = a.K2out;
  const int ldg = Hk + 8;
  const int64_t row0 = static_cast<int64_t>(xcd_remap(blockIdx.x, gridDim.x)) * BM;
  const int Pm = (1 << a.logPg) - 1;
  for (int it = threadIdx.x; it < BM * Hk; it += 256) {
    const int r = it / Hk, n = it - r * Hk;
    const int64_t row = row0 + r;
    float v = 0.f;
    if (row < a.M && ((a.mask[(row >> 5) * Hk + n] >> (row & 31)) & 1u)) {
      const int64_t t = row >> a.logPg;
      const int j = static_cast<int>(row & Pm);
      const float dn = a.dA[t * 2 * Hk + Hk + n] * a.inv;
      if (j < a.Fg) v = dn;
      else if (j == a.Fg) v = a.dA[t * 2 * Hk + n] + (a.include_self ? dn : 0.f);
    }
    lds[r * ldg + n] = f2bf(v);
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  constexpr int FM = BM / 16, FN = 4;
  for (int cchunk = 0; cchunk < K2; cchunk += kTrBN) {
    const int cb = cchunk + wave * 64;
    if (cb >= K2) continue;
    float4_t acc[FM][FN];
    tl_zero(acc);
    for (int k0 = 0; k0 < Hk; k0 += 32) {
      uint4_t b[FN], av[FM];
#pragma unroll
      for (int n = 0; n < FN; ++n) b[n] = fm_frag(a.WT, cb + n * 16, k0, Hk, lane);
#pragma unroll
      for (int m = 0; m < FM; ++m) av[m] = *reinterpret_cast<const uint4_t*>(lds + (m * 16 + lr) * ldg + k0 + lk);
#pragma unroll
      for (int m = 0; m < FM; ++m)
#pragma unroll
        for (int n = 0; n < FN; ++n) acc[m][n] = mfma16(av[m], b[n], acc[m][n]);
    }
#pragma unroll
    for (int m = 0; m < FM; ++m)
#pragma unroll
      for (int n = 0; n < FN; ++n)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t row = row0 + m * 16 + (lane >> 4) * 4 + j;
          if (row < a.M) a.dA_out[row * K2 + cb + n * 16 + lr] = acc[m][n][j];
        }
  }
}

// ----------------------------------------------------------------------------
// tr_head: kTrHeadRows roots per block, 16 waves; wave w owns 16-column slabs w, w+16, ...
// ----------------------------------------------------------------------------
constexpr int HB = kTrHeadRows;
constexpr int HFM = HB / 16;
constexpr int HNW = 16;
constexpr int TR_KC = 8;  // k steps (x32) per B chunk

// Head LDS tiles: rows padded by 16 bf16 (stride = 2 mod 4 16-B slots), so every
// ds_read_b128 lane group of an MFMA A-fragment read (rows 0-15 of two k-quarters:
// {0-3,12-15,20-27}, ...) lands on 16 distinct bank slots (2r + kq mod 16); the old
// +8 padding (stride 1 mod 16) put two lanes of every group on one slot.  Per-lane
// addresses stay base + constant, so the k loop folds them into the load offsets.
__device__ __forceinline__ int sw_off(int r, int col, int ld) { return r * ld + col; }

// the routed dW's G^T tile [64 p][32 k] (4 chunks per row, no padding): chunk c of row r
// at c ^ ((r >> 2) & 2) — conflict-free for the fragment reads and for 8-lane store groups
// that cover two whole rows (rows sharing a slot quad get distinct masks)
__device__ __forceinline__ int rt_off(int r, int col) { return r * 32 + ((((col >> 3) ^ ((r >> 2) & 2))) << 3) + (col & 7); }

__device__ __forceinline__ void tr_prefetch(const bf16_t* __restrict__ Bf, int col0, int N, int K, int lane,
                                            uint4_t (&b)[TR_KC]) {
  const int c = col0 < N ? col0 : 0;  // branch-free: out-of-range fragments are loaded but unused
#pragma unroll
  for (int s = 0; s < TR_KC; ++s) b[s] = fm_frag(Bf, c, s * 32 < K ? s * 32 : 0, K, lane);
}

__device__ __forceinline__ void tr_mfma_chunk(const bf16_t* A, int lda, int kc, int K, const uint4_t (&b)[TR_KC],
                                              float4_t (&acc)[HFM][1], int lane) {
  const int lr = lane & 15, lk = (lane >> 4) * 8;
#pragma unroll
  for (int s = 0; s < TR_KC; ++s) {
    if (kc + s * 32 < K) {
      uint4_t av[HFM];
#pragma unroll
      for (int m = 0; m < HFM; ++m) av[m] = *reinterpret_cast<const uint4_t*>(A + sw_off(m * 16 + lr, kc + s * 32 + lk, lda));
#pragma unroll
      for (int m = 0; m < HFM; ++m) acc[m][0] = mfma16(av[m], b[s], acc[m][0]);
    }
  }
}

// acc += A_lds[rows][0:K] @ Bf[col0 .. col0+15][0:K]^T; the first chunk was prefetched
__device__ __forceinline__ void tr_gemm(const bf16_t* A, int lda, const bf16_t* __restrict__ Bf, int col0, int K,
                                        float4_t (&acc)[HFM][1], int lane, const uint4_t (&pre)[TR_KC]) {
  tr_mfma_chunk(A, lda, 0, K, pre, acc, lane);
  for (int kc = 32 * TR_KC; kc < K; kc += 32 * TR_KC) {
    uint4_t b[TR_KC];
#pragma unroll
    for (int s = 0; s < TR_KC; ++s) b[s] = fm_frag(Bf, col0, kc + s * 32 < K ? kc + s * 32 : 0, K, lane);
    tr_mfma_chunk(A, lda, kc, K, b, acc, lane);
  }
}

// tile rows -> kt layout: item = (column pair, 8-row chunk), column pairs fastest (4-byte
// LDS reads over consecutive banks), two 16-byte kt chunks per item
__device__ __forceinline__ void tr_lds_to_kt(const bf16_t* tile, int ld, int N, int64_t r0, bf16_t* kt) {
  const int np = N >> 1;
  for (int it = threadIdx.x; it < np * (HB / 8); it += HNW * 64) {
    const int q = it / np, n = (it - q * np) * 2;
    uint32_t w[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) w[i] = *reinterpret_cast<const uint32_t*>(tile + sw_off(q * 8 + i, n, ld));
    uint4_t lo, hi;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      lo[i] = (w[2 * i] & 0xffffu) | (w[2 * i + 1] << 16);
      hi[i] = (w[2 * i] >> 16) | (w[2 * i + 1] & 0xffff0000u);
    }
    *reinterpret_cast<uint4_t*>(kt + kt_off(r0 + q * 8, n, N)) = lo;
    *reinterpret_cast<uint4_t*>(kt + kt_off(r0 + q * 8, n + 1, N)) = hi;
  }
}

__device__ __forceinline__ int tr_head_ld(int w) { return w + 16; }  // see sw_off

// Phases (a barrier between each; every wave takes tile jobs j = wave, wave + 16, ...):
//   P0  h = relu(A W^T)                                  [A tile + A_kt, h_kt]
//   P1  logits = h Wc^T + bc -> loss, F1 counts, dlogits   (C/16 jobs, critical path)
//       emb = h Wfc^T + bfc -> emb_kt                      (fills the idle waves)
//   P2  g = (dlogits Wc) * relu'(h) -> g_kt                (H/16 jobs, critical path)
//       demb = dlogits Wout -> demb_kt, fc-bias partials   (E/16 jobs)
//       remaining emb jobs
//   P3  dA = g W (fp32 rows for the layer below)
// fc and out_fc enter the critical path only through Wc = Wout Wfc (TrCombArgs): the
// reference model has no nonlinearity between them, so logits and their gradient to h are
// the same products with two dependent GEMM phases fewer.
__global__ __launch_bounds__(HNW * 64) void tr_head_kernel(TrHeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int nhb = static_cast<int>(gridDim.x) - a.nsample;
  if (static_cast<int>(blockIdx.x) >= nhb) {  // the next step's sampler on the CUs the head leaves idle
    tr_sample_block<HNW * 64>(a.smp, blockIdx.x - nhb, reinterpret_cast<int32_t*>(lds));
    return;
  }
#define TR_STAMP(k) \
  if (a.prof && threadIdx.x == 0) a.prof[blockIdx.x * 8 + (k)] = static_cast<long long>(wall_clock64())
  TR_STAMP(0);
  const int Hin2 = a.Hin2, H = a.H, E = a.E, C = a.C;
  const int lda = tr_head_ld(Hin2), ldh = tr_head_ld(H), ldc = tr_head_ld(C);
  bf16_t* Aa = lds;            // [HB][lda]  A rows
  bf16_t* Ah = Aa + HB * lda;  // [HB][ldh]  h (post-ReLU)
  bf16_t* Gb = Ah + HB * ldh;  // [HB][ldh]  g
  bf16_t* Dl = Gb + HB * ldh;  // [HB][ldc]  dlogits
  bf16_t* Ly = Dl + HB * ldc;  // [HB][C]    dense labels (label_mode 2)
  __shared__ int lab_s[HB];
  __shared__ float red_s[HNW][4];
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * HB;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  constexpr int NT = HNW * 64;

  if (a.label_mode < 2) {
    if (threadIdx.x < HB) {
      const int32_t root = a.roots[r0 + threadIdx.x];
      lab_s[threadIdx.x] = a.label_mode == 0 ? static_cast<int>(static_cast<const int16_t*>(a.labels)[root])
                                             : static_cast<const int32_t*>(a.labels)[root];
    }
  } else {
    const bf16_t* L = static_cast<const bf16_t*>(a.labels);
    const int cpl = C >> 3;
    for (int it = threadIdx.x; it < HB * cpl; it += NT) {
      const int r = it / cpl, c = it - r * cpl;
      const int64_t root = a.roots[r0 + r];
      *reinterpret_cast<uint4_t*>(Ly + r * C + c * 8) = *reinterpret_cast<const uint4_t*>(L + root * C + c * 8);
    }
  }
  // job lists of P1 / P2: (B operand, its K, output column)
  const int nl = C >> 4, ne = E >> 4, nh = H >> 4;
  const int ne1 = (HNW - nl) > 0 ? ((HNW - nl) < ne ? (HNW - nl) : ne) : 0;  // emb jobs beside the logits
  const int n1 = nl + ne1, n2 = nh + ne + (ne - ne1);
  auto job1 = [&](int j, const bf16_t*& Bf, int& cc) {
    if (j < nl) {
      Bf = a.Wc;
      cc = j * 16;
    } else {
      Bf = a.Wfc;
      cc = (j - nl) * 16;
    }
  };
  auto job2 = [&](int j, const bf16_t*& Bf, int& cc, int& K) {
    if (j < nh) {
      Bf = a.WcT;
      cc = j * 16;
      K = C;
    } else if (j < nh + ne) {
      Bf = a.WoutT;
      cc = (j - nh) * 16;
      K = C;
    } else {
      Bf = a.Wfc;
      cc = (ne1 + j - nh - ne) * 16;
      K = H;
    }
  };

  // P0: A tile -> LDS (+ A_kt); h = relu(A @ W^T)
  uint4_t pre[TR_KC];
  tr_prefetch(a.W, wave * 16, H, Hin2, lane, pre);
  const int cpa = Hin2 >> 3;
  for (int it = threadIdx.x; it < HB * cpa; it += NT) {
    const int r = it / cpa, c = it - r * cpa;
    *reinterpret_cast<uint4_t*>(Aa + sw_off(r, c * 8, lda)) =
        *reinterpret_cast<const uint4_t*>(a.A + (r0 + r) * Hin2 + c * 8);
  }
  __syncthreads();
  TR_STAMP(1);
  tr_lds_to_kt(Aa, lda, Hin2, r0, a.A_kt);
  for (int cc = wave * 16; cc < H; cc += HNW * 16) {
    float4_t acc[HFM][1];
    tl_zero(acc);
    tr_gemm(Aa, lda, a.W, cc, Hin2, acc, lane, pre);
    if (cc + HNW * 16 < H) tr_prefetch(a.W, cc + HNW * 16, H, Hin2, lane, pre);
#pragma unroll
    for (int m = 0; m < HFM; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) Ah[sw_off(m * 16 + lg * 4 + j, cc + lr, ldh)] = f2bf(fmaxf(acc[m][0][j], 0.f));
  }
  if (wave < n1) {
    const bf16_t* Bf;
    int cc;
    job1(wave, Bf, cc);
    tr_prefetch(Bf, cc, 1 << 30, H, lane, pre);
  }
  __syncthreads();
  TR_STAMP(2);
  tr_lds_to_kt(Ah, ldh, H, r0, a.h_kt);

  // P1: logits (+ loss, dlogits, F1 counts; padded label columns excluded) and emb
  float lsum = 0.f;
  int tp = 0, fp = 0, fn = 0;
  for (int j = wave; j < n1; j += HNW) {
    const bf16_t* Bf;
    int cc;
    job1(j, Bf, cc);
    float4_t acc[HFM][1];
    tl_zero(acc);
    tr_gemm(Ah, ldh, Bf, cc, H, acc, lane, pre);
    const int col = cc + lr;
    if (j < nl) {
      const bool valid = col < a.C_real;
      const float bias = a.bc[col];
#pragma unroll
      for (int m = 0; m < HFM; ++m) {
        float d[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int row = m * 16 + lg * 4 + jj;
          const float xv = acc[m][0][jj] + bias;
          const float y = a.label_mode < 2 ? ((lab_s[row] == col) ? 1.f : 0.f) : bf2f(Ly[row * C + col]);
          const float p = 1.f / (1.f + __expf(-xv));
          if (valid) {
            lsum += fmaxf(xv, 0.f) - xv * y + log1pf(__expf(-fabsf(xv)));
            const bool pred = xv >= 0.f, pos = y > 0.5f;
            tp += pred && pos;
            fp += pred && !pos;
            fn += !pred && pos;
          }
          d[jj] = valid ? bf2f(f2bf((p - y) * a.inv_scale)) : 0.f;
          Dl[sw_off(row, col, ldc)] = f2bf(d[jj]);
        }
        kt_store4(a.dlog_kt, r0 + m * 16 + lg * 4, col, C, d[0], d[1], d[2], d[3]);
      }
    } else {
      const float b = a.bfc[col];
#pragma unroll
      for (int m = 0; m < HFM; ++m)
        kt_store4(a.emb_kt, r0 + m * 16 + lg * 4, col, E, acc[m][0][0] + b, acc[m][0][1] + b, acc[m][0][2] + b,
                  acc[m][0][3] + b);
    }
    if (j + HNW < n1) {  // (after the epilogue: the loss math keeps no prefetch registers live)
      const bf16_t* Bn;
      int cn;
      job1(j + HNW, Bn, cn);
      tr_prefetch(Bn, cn, 1 << 30, H, lane, pre);
    }
  }
  {
    lsum = wave_sum(lsum);
    tp = wave_sum_i(tp);
    fp = wave_sum_i(fp);
    fn = wave_sum_i(fn);
    if (lane == 0) {
      red_s[wave][0] = lsum;
      red_s[wave][1] = static_cast<float>(tp);
      red_s[wave][2] = static_cast<float>(fp);
      red_s[wave][3] = static_cast<float>(fn);
    }
  }
  if (wave < n2) {
    const bf16_t* Bf;
    int cc, K;
    job2(wave, Bf, cc, K);
    tr_prefetch(Bf, cc, 1 << 30, K, lane, pre);
  }
  __syncthreads();
  TR_STAMP(3);
  if (threadIdx.x < 4) {  // per-block sums, plain stores (no contended atomics)
    float v = 0.f;
#pragma unroll
    for (int w = 0; w < HNW; ++w) v += red_s[w][threadIdx.x];
    a.head_part[blockIdx.x * 4 + threadIdx.x] = threadIdx.x == 0 ? v * a.inv_scale : v;
  }

  // P2: g = (dlogits Wc) * relu'(h); demb = dlogits Wout (+ fc-bias column sums); emb rest
  for (int j = wave; j < n2; j += HNW) {
    const bf16_t* Bf;
    int cc, K;
    job2(j, Bf, cc, K);
    float4_t acc[HFM][1];
    tl_zero(acc);
    tr_gemm(j < nh + ne ? Dl : Ah, j < nh + ne ? ldc : ldh, Bf, cc, K, acc, lane, pre);
    const int col = cc + lr;
    if (j < nh) {
#pragma unroll
      for (int m = 0; m < HFM; ++m) {
        float e[4];
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int row = m * 16 + lg * 4 + jj;
          e[jj] = bf2f(f2bf(bf_pos(Ah[sw_off(row, col, ldh)]) ? acc[m][0][jj] : 0.f));
          Gb[sw_off(row, col, ldh)] = f2bf(e[jj]);
        }
        kt_store4(a.g_kt, r0 + m * 16 + lg * 4, col, H, e[0], e[1], e[2], e[3]);
      }
    } else if (j < nh + ne) {
      float cs = 0.f;
#pragma unroll
      for (int m = 0; m < HFM; ++m) {
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) cs += acc[m][0][jj];
        kt_store4(a.demb_kt, r0 + m * 16 + lg * 4, col, E, acc[m][0][0], acc[m][0][1], acc[m][0][2], acc[m][0][3]);
      }
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      if (lg == 0) a.dbfc_part[static_cast<int64_t>(blockIdx.x) * E + col] = cs;
    } else {
      const float b = a.bfc[col];
#pragma unroll
      for (int m = 0; m < HFM; ++m)
        kt_store4(a.emb_kt, r0 + m * 16 + lg * 4, col, E, acc[m][0][0] + b, acc[m][0][1] + b, acc[m][0][2] + b,
                  acc[m][0][3] + b);
    }
    if (j + HNW < n2) {
      const bf16_t* Bn;
      int cn, Kn;
      job2(j + HNW, Bn, cn, Kn);
      tr_prefetch(Bn, cn, 1 << 30, Kn, lane, pre);
    }
  }
  if (a.dA) tr_prefetch(a.WT, wave * 16, Hin2, H, lane, pre);
  __syncthreads();
  TR_STAMP(4);

  // P3: dA = g @ W (fp32 rows) for the layer below
  if (a.dA) {
    for (int cc = wave * 16; cc < Hin2; cc += HNW * 16) {
      float4_t acc[HFM][1];
      tl_zero(acc);
      tr_gemm(Gb, ldh, a.WT, cc, H, acc, lane, pre);
      if (cc + HNW * 16 < Hin2) tr_prefetch(a.WT, cc + HNW * 16, Hin2, H, lane, pre);
#pragma unroll
      for (int m = 0; m < HFM; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) a.dA[(r0 + m * 16 + lg * 4 + j) * Hin2 + cc + lr] = acc[m][0][j];
    }
  }
  TR_STAMP(5);
#undef TR_STAMP
}

// ----------------------------------------------------------------------------
// tr_pair_head: the head of the unsupervised GraphSAGE step (see TrPairHeadArgs; reference
// examples/graphsage/graphsage.py:70-98, tf_euler/python/mp_utils/base.py:49-91).  Block b:
// sources 16b..16b+15 and their context rows, 2 + K row tiles of 16 in LDS (tile 0: the
// sources, tile 1: their positives, tiles 2..: their negatives, source-major), 16 waves;
// every phase deals its (tile, 16-column slab) jobs round-robin over the waves, each one
// tr_gemm (A rows from LDS, the tile's tower's B fragments from L2):
//   P1 h1 = relu(A1 W1^T)                   -> H   (+ A1_kt, h_kt for the dW GEMMs)
//   P2 e  = h1 Wfc^T + bfc                  -> Ef  (fp32, over the dead A1 tile)
//   P3 wave i = source i: logits <e_i, e_ctx>, softplus CE, reciprocal rank, de (fp32)
//                                           -> D (bf16, + de_kt), bias / loss partials
//   P4 g  = (de Wfc) * relu'(h1)            -> G   (over the dead Ef) (+ g_kt)
//   P5 dA1 = g W1                           (fp32 rows: the routed layer-0 dW reads them)
// ----------------------------------------------------------------------------
__device__ __forceinline__ const TrPairTower& pr_tower(const TrPairHeadArgs& a, int t) { return t == 0 ? a.s : a.c; }

// first row of tile t in its tower
__device__ __forceinline__ int64_t pr_row0(const TrPairHeadArgs& a, int b, int t) {
  if (t <= 1) return static_cast<int64_t>(b) * 16;
  return static_cast<int64_t>(a.B) + static_cast<int64_t>(b) * 16 * a.K + 16 * (t - 2);
}

__global__ __launch_bounds__(HNW * 64) void tr_pair_head_kernel(TrPairHeadArgs a) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int b = blockIdx.x;
  const int NTILE = 2 + a.K, rows = 16 * NTILE;
  const int H0x2 = a.H0x2, H1 = a.H1, E = a.E;
  const int lda = tr_head_ld(H0x2), ldh = tr_head_ld(H1), lde = tr_head_ld(E);
  const int abytes = rows * lda * 2, ebytes = rows * E * 4, gbytes = rows * ldh * 2;
  const int region = ((abytes > ebytes ? abytes : ebytes) > gbytes ? (abytes > ebytes ? abytes : ebytes) : gbytes);
  bf16_t* Aa = lds;                                                   // P1 input
  float* Ef = reinterpret_cast<float*>(lds);                          // P2 -> P3 (over Aa)
  bf16_t* Gg = lds;                                                   // P4 -> P5 (over Ef)
  bf16_t* Hh = lds + region / 2;                                      // h1
  bf16_t* Dd = Hh + rows * ldh;                                       // de
  float* ps = reinterpret_cast<float*>(Dd + rows * lde);              // [2][16][E] bias partials
  __shared__ float red_s[HNW][2];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  constexpr int NT = HNW * 64;

  // A1 rows of every tile -> LDS (+ the kt copies for dW1)
  const int cpa = H0x2 >> 3;
  for (int it = threadIdx.x; it < rows * cpa; it += NT) {
    const int r = it / cpa, c = it - r * cpa;
    const int t = r >> 4;
    const TrPairTower& tw = pr_tower(a, t);
    *reinterpret_cast<uint4_t*>(Aa + sw_off(r, c * 8, lda)) =
        *reinterpret_cast<const uint4_t*>(tw.A1 + (pr_row0(a, b, t) + (r & 15)) * H0x2 + c * 8);
  }
  __syncthreads();
  for (int t = 0; t < NTILE; ++t) tr_lds_to_kt(Aa + 16 * t * lda, lda, H0x2, pr_row0(a, b, t), pr_tower(a, t).A1_kt);

  uint4_t pre[TR_KC];
  // P1: h1 = relu(A1 W1^T)
  {
    const int nc = H1 >> 4, nj = NTILE * nc;
    if (wave < nj) tr_prefetch(pr_tower(a, wave / nc).W1, (wave % nc) * 16, H1, H0x2, lane, pre);
    for (int j = wave; j < nj; j += HNW) {
      const int t = j / nc, cs = (j - t * nc) * 16;
      float4_t acc[HFM][1];
      tl_zero(acc);
      tr_gemm(Aa + 16 * t * lda, lda, pr_tower(a, t).W1, cs, H0x2, acc, lane, pre);
      if (j + HNW < nj) tr_prefetch(pr_tower(a, (j + HNW) / nc).W1, ((j + HNW) % nc) * 16, H1, H0x2, lane, pre);
      float v[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        v[jj] = fmaxf(acc[0][0][jj], 0.f);
        Hh[sw_off(16 * t + lg * 4 + jj, cs + lr, ldh)] = f2bf(v[jj]);
      }
      kt_store4(pr_tower(a, t).h_kt, pr_row0(a, b, t) + lg * 4, cs + lr, H1, bf2f(f2bf(v[0])), bf2f(f2bf(v[1])),
                bf2f(f2bf(v[2])), bf2f(f2bf(v[3])));
    }
  }
  __syncthreads();  // A1 dead from here (Ef takes its place)
  // P2: e = h1 Wfc^T + bfc (fp32)
  {
    const int nc = E >> 4, nj = NTILE * nc;
    if (wave < nj) tr_prefetch(pr_tower(a, wave / nc).Wfc, (wave % nc) * 16, E, H1, lane, pre);
    for (int j = wave; j < nj; j += HNW) {
      const int t = j / nc, cs = (j - t * nc) * 16;
      float4_t acc[HFM][1];
      tl_zero(acc);
      tr_gemm(Hh + 16 * t * ldh, ldh, pr_tower(a, t).Wfc, cs, H1, acc, lane, pre);
      if (j + HNW < nj) tr_prefetch(pr_tower(a, (j + HNW) / nc).Wfc, ((j + HNW) % nc) * 16, E, H1, lane, pre);
      const float bias = pr_tower(a, t).bfc[cs + lr];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) Ef[(16 * t + lg * 4 + jj) * E + cs + lr] = acc[0][0][jj] + bias;
    }
  }
  __syncthreads();
  // P3: wave i = source i of the block
  {
    // logits / gradients of the 1 + K <= 16 pairs in registers (fully unrolled: constant
    // indices, no scratch)
    const int i = wave;
    const int K = a.K;
    float l[16], g[16];
    const float* es = Ef + i * E;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      l[k] = 0.f;
      if (k > K) continue;
      const int row = k == 0 ? 16 + i : 32 + i * K + (k - 1);
      float d = 0.f;
      for (int c = lane; c < E; c += 64) d += es[c] * Ef[row * E + c];
      l[k] = wave_sum(d);
    }
    float loss = 0.f, gsum = 0.f;
    int beat = 0;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      g[k] = 0.f;
      if (k > K) continue;
      const float x = l[k];
      loss += fmaxf(x, 0.f) + log1pf(__expf(-fabsf(x))) - (k == 0 ? x : 0.f);
      g[k] = (1.f / (1.f + __expf(-x)) - (k == 0 ? 1.f : 0.f)) * a.inv_n;
      gsum += g[k];
      if (k > 0 && x >= l[0]) ++beat;
    }
    if (lane == 0) {
      red_s[i][0] = loss * a.inv_n;
      red_s[i][1] = 1.f / static_cast<float>(1 + beat);
    }
    for (int c = lane; c < E; c += 64) {
      const float ev = es[c];
      float de = 0.f;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (k > K) continue;
        const int row = k == 0 ? 16 + i : 32 + i * K + (k - 1);
        de += g[k] * Ef[row * E + c];
        Dd[sw_off(row, c, lde)] = f2bf(g[k] * ev);
      }
      Dd[sw_off(i, c, lde)] = f2bf(de);
      ps[i * E + c] = de;                 // source-tower bias gradient share
      ps[(16 + i) * E + c] = gsum * ev;   // context-tower share: sum_k g_k e_i
    }
  }
  __syncthreads();  // Ef dead from here (G takes its place)
  for (int t = 0; t < NTILE; ++t) tr_lds_to_kt(Dd + 16 * t * lde, lde, E, pr_row0(a, b, t), pr_tower(a, t).de_kt);
  for (int c = threadIdx.x; c < 2 * E; c += NT) {  // per-block bias partials, fixed order
    const int tw = c >= E, col = c - tw * E;
    float v = 0.f;
    for (int w = 0; w < 16; ++w) v += ps[(tw * 16 + w) * E + col];
    (tw ? a.c : a.s).dbfc_part[static_cast<int64_t>(b) * E + col] = v;
  }
  if (threadIdx.x < 4) {
    float v = 0.f;
    if (threadIdx.x < 2)
      for (int w = 0; w < 16; ++w) v += red_s[w][threadIdx.x];
    a.head_part[b * 4 + threadIdx.x] = v;
  }
  // P4: g = (de Wfc) * relu'(h1)
  {
    const int nc = H1 >> 4, nj = NTILE * nc;
    if (wave < nj) tr_prefetch(pr_tower(a, wave / nc).WfcT, (wave % nc) * 16, H1, E, lane, pre);
    for (int j = wave; j < nj; j += HNW) {
      const int t = j / nc, cs = (j - t * nc) * 16;
      float4_t acc[HFM][1];
      tl_zero(acc);
      tr_gemm(Dd + 16 * t * lde, lde, pr_tower(a, t).WfcT, cs, E, acc, lane, pre);
      if (j + HNW < nj) tr_prefetch(pr_tower(a, (j + HNW) / nc).WfcT, ((j + HNW) % nc) * 16, H1, E, lane, pre);
      float v[4];
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int row = 16 * t + lg * 4 + jj;
        v[jj] = bf2f(f2bf(bf_pos(Hh[sw_off(row, cs + lr, ldh)]) ? acc[0][0][jj] : 0.f));
        Gg[sw_off(row, cs + lr, ldh)] = f2bf(v[jj]);
      }
      kt_store4(pr_tower(a, t).g_kt, pr_row0(a, b, t) + lg * 4, cs + lr, H1, v[0], v[1], v[2], v[3]);
    }
  }
  __syncthreads();
  // P5: dA1 = g W1 (fp32 rows)
  {
    const int nc = H0x2 >> 4, nj = NTILE * nc;
    if (wave < nj) tr_prefetch(pr_tower(a, wave / nc).W1T, (wave % nc) * 16, H0x2, H1, lane, pre);
    for (int j = wave; j < nj; j += HNW) {
      const int t = j / nc, cs = (j - t * nc) * 16;
      float4_t acc[HFM][1];
      tl_zero(acc);
      tr_gemm(Gg + 16 * t * ldh, ldh, pr_tower(a, t).W1T, cs, H1, acc, lane, pre);
      if (j + HNW < nj) tr_prefetch(pr_tower(a, (j + HNW) / nc).W1T, ((j + HNW) % nc) * 16, H0x2, H1, lane, pre);
      float* out = pr_tower(a, t).dA1;
      const int64_t r0 = pr_row0(a, b, t);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) out[(r0 + lg * 4 + jj) * H0x2 + cs + lr] = acc[0][0][jj];
    }
  }
}

// ----------------------------------------------------------------------------
// tr_dw: grouped split-K weight gradients, part[s][p][q] = sum_{m in split s} G[m][p] X[m][q];
// 64x64 tiles, 4 waves of 32x32
// ----------------------------------------------------------------------------
// raw operands of a route problem's G^T fragment (rows mb*32 + lk .. +7, column p): the
// ReLU bits and the parent's self / neighbour gradients
struct RouteRaw {
  uint32_t bits;
  float ds, dn;
};

__device__ __forceinline__ RouteRaw tr_route_load(const TrDwProb& pr, int mb, int p, int lk) {
  const int64_t m0 = static_cast<int64_t>(mb) * 32 + lk;
  const float* row = pr.dA + (m0 >> pr.logPg) * 2 * pr.P;
  RouteRaw r;
  r.bits = pr.mask[static_cast<int64_t>(mb) * pr.P + p] >> lk;
  r.ds = row[p];
  r.dn = row[pr.P + p];
  return r;
}

// G[m][p] for the 8 rows: neighbour slots (j < Fg) get dn / (Fg + self), the self slot
// ds (+ the neighbour share with self loops), padding 0, all masked by the ReLU bits
__device__ __forceinline__ uint4_t tr_route_frag(const TrDwProb& pr, const RouteRaw& r, int mb, int lk) {
  const int j0 = static_cast<int>((static_cast<int64_t>(mb) * 32 + lk) & ((int64_t(1) << pr.logPg) - 1));
  const float dn = r.dn * pr.inv;
  const float ds = r.ds + (pr.include_self ? dn : 0.f);
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    const int j = j0 + i;
    const float val = j < pr.Fg ? dn : (j == pr.Fg ? ds : 0.f);
    v[i] = ((r.bits >> i) & 1u) ? val : 0.f;
  }
  return pack_bf16x8(v);
}

// the same fragment with a handful of instructions (the select chain above costs ~77 VALU
// per fragment and made the routed dW issue-bound): which of the 8 rows are neighbour /
// self slots is two 8-bit masks of j0, the ReLU bits pick rows, and `lut` (256 entries,
// LDS) spreads an 8-bit row set into the 0xffff halves of 4 words; the values are the
// bf16 pair of dn (resp. ds), rounded exactly like pack_bf16x8.
__device__ __forceinline__ uint4_t tr_route_frag_lut(const TrDwProb& pr, const RouteRaw& r, int mb, int lk,
                                                     const uint4_t* lut) {
  const int j0 = static_cast<int>((static_cast<int64_t>(mb) * 32 + lk) & ((int64_t(1) << pr.logPg) - 1));
  const int dF = pr.Fg - j0;
  const uint32_t nm = dF >= 8 ? 0xffu : (dF <= 0 ? 0u : ((1u << dF) - 1u));
  const uint32_t sm = (dF >= 0 && dF < 8) ? (1u << dF) : 0u;
  const uint32_t b8 = r.bits & 0xffu;
  const float dn = r.dn * pr.inv;
  const float ds = r.ds + (pr.include_self ? dn : 0.f);
  const uint32_t DN = pack_bf16x2(dn, dn), DS = pack_bf16x2(ds, ds);
  const uint4_t mN = lut[b8 & nm], mS = lut[b8 & sm];
  uint4_t out;
#pragma unroll
  for (int i = 0; i < 4; ++i) out[i] = (DN & mN[i]) | (DS & mS[i]);
  return out;
}

// lut[b] word i = (bit 2i of b ? 0x0000ffff : 0) | (bit 2i + 1 ? 0xffff0000 : 0); one entry
// per thread of a 256-thread block (the caller synchronises before the first use)
__device__ __forceinline__ void tr_spread_lut_init(uint4_t* lut) {
  if (threadIdx.x < 256) {
    const uint32_t b = threadIdx.x;
    uint4_t w;
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = (((b >> (2 * i)) & 1u) ? 0x0000ffffu : 0u) | (((b >> (2 * i + 1)) & 1u) ? 0xffff0000u : 0u);
    lut[b] = w;
  }
}

// ----------------------------------------------------------------------------
// tr_dw_route: split-K dW of a layer whose output gradient is routed from the parent
// rows (the tree mean's backward). Workgroup tile 64 p x 128 q; per stage of kRKB
// k-blocks every thread builds one G^T fragment lane per k-block (p = tid & 63, 8 rows)
// into LDS, so each routed element is built once per q tile; wave w multiplies all 64 p
// rows by its 32 q columns with X fragments loaded straight from the kt layout, one
// stage (kRKB k-blocks) ahead.
// ----------------------------------------------------------------------------
#ifndef TR_RKB
#define TR_RKB 8
#endif
// kRKB k-blocks per stage; the double-buffered G tile takes 2 * kRKB * 4 KiB of LDS.
// G^T tile [64 p][32 rows], 16-B chunks swizzled (rt_off, 4 chunks per row): the MFMA
// fragment reads and the builder's stores (lanes 4i..4i+3 = the 4 chunks of p-row i, so
// an 8-lane store group covers two whole rows) are bank-conflict-free
constexpr int kRP = 64, kRQ = 128, kRKB = TR_RKB, kRLd = 32;

struct RouteStage {
  RouteRaw r[kRKB];
  uint4_t x[kRKB][2];
};

typedef bf16_t RouteLds[2][kRKB][kRP * kRLd];

#define RT_STAMP(k) \
  if (prof && threadIdx.x == 0) prof[static_cast<int64_t>(b) * 8 + (k)] = static_cast<long long>(wall_clock64())
__device__ __forceinline__ void tr_dw_route_body(const TrDwProb& pr, int b, RouteLds& gs, const uint4_t* lut,
                                                 long long* prof) {
  RT_STAMP(0);
  // XCD-aware: the tiles of one split (which read the same X rows) share b % 8
  const int j = b >> 3;
  const int tile = j % pr.ntiles;
  const int s = (j / pr.ntiles) * 8 + (b & 7);
  const int tp = tile / pr.tiles_q, tq = tile - tp * pr.tiles_q;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  const int bpl = tid >> 2, blk = (tid & 3) * 8;  // builder: column p = bpl, rows blk..+7
  const int bp = tp * kRP + bpl;
  const int wq = tq * kRQ + wave * 32;                           // MFMA: columns wq..+31, all 64 rows
  const int64_t Q = pr.Q;
  const bool qok = wq < Q;  // uniform
  const int mb0 = s * pr.kps;
  const int mb1 = (mb0 + pr.kps) < pr.MB ? (mb0 + pr.kps) : pr.MB;
  float4_t acc[4][2];
  tl_zero(acc);
  if (mb0 < mb1) {
    auto load = [&](RouteStage& st, int mbs) {
#pragma unroll
      for (int u = 0; u < kRKB; ++u) {
        const int mb = (mbs + u) < mb1 ? (mbs + u) : (mb1 - 1);  // clamped: always a valid row
        st.r[u] = tr_route_load(pr, mb, bp, blk);
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const int q = qok ? wq + f * 16 + lr : lr;
          st.x[u][f] = *reinterpret_cast<const uint4_t*>(pr.X + ((static_cast<int64_t>(mb) * Q + q) * 32 + lk));
        }
      }
    };
    auto build = [&](const RouteStage& st, int buf, int mbs) {
#pragma unroll
      for (int u = 0; u < kRKB; ++u) {
        const uint4_t fr = (mbs + u) < mb1 ? tr_route_frag_lut(pr, st.r[u], mbs + u, blk, lut) : uint4_t{0u, 0u, 0u, 0u};
        *reinterpret_cast<uint4_t*>(&gs[buf][u][rt_off(bpl, blk)]) = fr;
      }
    };
    auto compute = [&](const RouteStage& st, int buf, int mbs) {
      if (!qok) return;
#pragma unroll
      for (int u = 0; u < kRKB; ++u) {
        if (mbs + u >= mb1) break;  // uniform
        uint4_t a[4];
#pragma unroll
        for (int fm = 0; fm < 4; ++fm)
          a[fm] = *reinterpret_cast<const uint4_t*>(&gs[buf][u][rt_off(fm * 16 + lr, lk)]);
#pragma unroll
        for (int fn = 0; fn < 2; ++fn)
#pragma unroll
          for (int fm = 0; fm < 4; ++fm) acc[fm][fn] = mfma16(a[fm], st.x[u][fn], acc[fm][fn]);
      }
    };
    RouteStage A, B;
    load(A, mb0);
    int it = 0;
    for (int mbs = mb0; mbs < mb1; mbs += 2 * kRKB) {
      build(A, 0, mbs);
      load(B, mbs + kRKB);
      __syncthreads();
      compute(A, 0, mbs);
      if (mbs + kRKB < mb1) {
        build(B, 1, mbs + kRKB);
        load(A, mbs + 2 * kRKB);
        __syncthreads();
        compute(B, 1, mbs + kRKB);
      }
      ++it;
      if (it < 6) RT_STAMP(it);
    }
  }
  RT_STAMP(7);
  if (!qok) return;
  float* out = pr.part + static_cast<int64_t>(s) * pr.P * Q;
  const int p0 = tp * kRP;
#pragma unroll
  for (int fm = 0; fm < 4; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        out[(p0 + fm * 16 + (lane >> 4) * 4 + jj) * Q + wq + fn * 16 + lr] = acc[fm][fn][jj];
}

// ----------------------------------------------------------------------------
// tr_dw_route_reg: the routed dW without the LDS G tile or any barrier.  Every wave builds
// the G^T fragments of all 64 p rows of the tile in registers (p = p0 + 16 fm + lr, rows
// lk..lk+7 of the k-block) from the ReLU bits and the parent's dA row (4x redundant across
// the block's waves, served by L1) and multiplies them by its own 32 X columns; k-block
// groups of kRG double-buffered in registers like the plain body, so the next group's
// loads are in flight behind this group's build + MFMAs.
// ----------------------------------------------------------------------------
constexpr int kRG = 4;
__device__ __forceinline__ void tr_dw_route_reg_body(const TrDwProb& pr, int b, const uint4_t* lut, long long* prof) {
  RT_STAMP(0);
  const int j = b >> 3;
  const int tile = j % pr.ntiles;
  const int s = (j / pr.ntiles) * 8 + (b & 7);
  const int tp = tile / pr.tiles_q, tq = tile - tp * pr.tiles_q;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  const int p0 = tp * kRP;
  const int wq = tq * kRQ + wave * 32;
  const int64_t Q = pr.Q, P = pr.P;
  if (wq >= Q) return;  // no barriers in this body
  const int mb0 = s * pr.kps;
  const int mb1 = (mb0 + pr.kps) < pr.MB ? (mb0 + pr.kps) : pr.MB;
  float4_t acc[4][2];
  tl_zero(acc);
  struct Grp {
    uint4_t x[kRG][2];
    RouteRaw r[kRG][4];
  };
  auto load = [&](Grp& g, int mbs) {
#pragma unroll
    for (int u = 0; u < kRG; ++u) {
      const int mb = (mbs + u) < mb1 ? (mbs + u) : (mb1 - 1);
#pragma unroll
      for (int f = 0; f < 2; ++f)
        g.x[u][f] = *reinterpret_cast<const uint4_t*>(pr.X + ((static_cast<int64_t>(mb) * Q + wq + f * 16 + lr) * 32 + lk));
#pragma unroll
      for (int fm = 0; fm < 4; ++fm) g.r[u][fm] = tr_route_load(pr, mb, p0 + fm * 16 + lr, lk);
    }
  };
  auto compute = [&](const Grp& g, int mbs) {
#pragma unroll
    for (int u = 0; u < kRG; ++u) {
      if (mbs + u >= mb1) break;  // uniform
#pragma unroll
      for (int fm = 0; fm < 4; ++fm) {
        const uint4_t a = tr_route_frag_lut(pr, g.r[u][fm], mbs + u, lk, lut);
#pragma unroll
        for (int fn = 0; fn < 2; ++fn) acc[fm][fn] = mfma16(a, g.x[u][fn], acc[fm][fn]);
      }
    }
  };
  if (mb0 < mb1) {
    Grp A, B;
    load(A, mb0);
    int it = 0;
    for (int mbs = mb0; mbs < mb1; mbs += 2 * kRG) {
      load(B, mbs + kRG);
      compute(A, mbs);
      if (mbs + kRG >= mb1) break;
      load(A, mbs + 2 * kRG);
      compute(B, mbs + kRG);
      ++it;
      if (it < 6 && (it & 1) == 0) RT_STAMP(it >> 1);
    }
  }
  (void)P;
  float* out = pr.part + static_cast<int64_t>(s) * pr.P * Q;
#pragma unroll
  for (int fm = 0; fm < 4; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj)
        out[(p0 + fm * 16 + (lane >> 4) * 4 + jj) * Q + wq + fn * 16 + lr] = acc[fm][fn][jj];
  RT_STAMP(7);
}
#undef RT_STAMP

// ----------------------------------------------------------------------------
// tr_dw: grouped split-K dW of the problems with stored G operands (kt layout),
// part[s][p][q] = sum_{m in split s} G[m][p] X[m][q]; 64x64 tiles, 4 waves of 32x32,
// k-block groups double-buffered in registers (unrolled ping-pong: no register copies)
// ----------------------------------------------------------------------------
__device__ __forceinline__ void tr_dw_plain_body(const TrDwProbs& probs, int b, int nwg) {
  const int id = xcd_remap(b, nwg);
  // constant indices only (no dynamic indexing of kernel arguments)
  TrDwProb pr = probs.p[0];
#pragma unroll
  for (int i = 1; i < kTrMaxProbs; ++i)
    if (probs.n > i && id >= probs.p[i].wg0) pr = probs.p[i];
  const int local = id - pr.wg0;
  const int s = local / pr.ntiles;
  const int tile = local - s * pr.ntiles;
  const int tp = tile / pr.tiles_q, tq = tile - (tile / pr.tiles_q) * pr.tiles_q;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  const int p0 = tp * 64 + (wave >> 1) * 32;
  const int q0 = tq * 64 + (wave & 1) * 32;
  const int mb0 = s * pr.kps;
  const int mb1 = (mb0 + pr.kps) < pr.MB ? (mb0 + pr.kps) : pr.MB;
  const int64_t P = pr.P, Q = pr.Q;
  if (p0 >= P || q0 >= Q) return;  // 32-wide edge of a 64-wide tile; no barriers in this kernel
  float4_t acc[2][2];
  tl_zero(acc);
  constexpr int KB = 4;
  struct Grp {
    uint4_t a[KB][2], b[KB][2];
  };
  auto load = [&](Grp& g, int mbs) {
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      const int64_t mb = (mbs + u) < mb1 ? (mbs + u) : (mb1 - 1);
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        g.a[u][f] = *reinterpret_cast<const uint4_t*>(pr.G + ((mb * P + p0 + f * 16 + lr) * 32 + lk));
        g.b[u][f] = *reinterpret_cast<const uint4_t*>(pr.X + ((mb * Q + q0 + f * 16 + lr) * 32 + lk));
      }
    }
  };
  auto compute = [&](const Grp& g, int mbs) {
#pragma unroll
    for (int u = 0; u < KB; ++u) {
      if (mbs + u >= mb1) break;  // uniform
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn) acc[fm][fn] = mfma16(g.a[u][fm], g.b[u][fn], acc[fm][fn]);
    }
  };
  if (mb0 < mb1) {
    Grp A, B;
    load(A, mb0);
    for (int mbs = mb0; mbs < mb1; mbs += 2 * KB) {
      load(B, mbs + KB);
      compute(A, mbs);
      if (mbs + KB >= mb1) break;
      load(A, mbs + 2 * KB);
      compute(B, mbs + KB);
    }
  }
  float* out = pr.part + static_cast<int64_t>(s) * P * Q;
#pragma unroll
  for (int fm = 0; fm < 2; ++fm)
#pragma unroll
    for (int fn = 0; fn < 2; ++fn)
#pragma unroll
      for (int j = 0; j < 4; ++j)
        out[(p0 + fm * 16 + (lane >> 4) * 4 + j) * Q + q0 + fn * 16 + lr] = acc[fm][fn][j];
}

__global__ __launch_bounds__(256, 2) void tr_dw_all_kernel(TrDwLaunch a) {
  __shared__ __attribute__((aligned(16))) RouteLds gs;
  __shared__ uint4_t lut[256];
  const int b = blockIdx.x;
  if (a.nroute > 0 && b < a.rwg[a.nroute]) {  // routed blocks: the fragment-spread table first
    tr_spread_lut_init(lut);
    __syncthreads();
  }
  if (a.nroute > 0 && b < a.rwg[1]) {
    if (a.route_impl == 1) tr_dw_route_reg_body(a.route[0], b, lut, a.prof);
    else tr_dw_route_body(a.route[0], b, gs, lut, a.prof);
  } else if (a.nroute > 1 && b < a.rwg[2]) {
    if (a.route_impl == 1) tr_dw_route_reg_body(a.route[1], b - a.rwg[1], lut, nullptr);
    else tr_dw_route_body(a.route[1], b - a.rwg[1], gs, lut, nullptr);
  } else {
    const int r = a.rwg[a.nroute];
    tr_dw_plain_body(a.plain, b - r, static_cast<int>(gridDim.x) - r);
  }
}

// ----------------------------------------------------------------------------
// tr_opt: split-K reduce and/or the optimizer over the flat fp32 parameters, the bf16
// weight shadows, loss hand-off and the RNG counter advance (hipGraph-replay safe)
// ----------------------------------------------------------------------------
// GATHER: the launch also carries the next step's layer-0 gather tiles (pipelined step);
// a separate instantiation so the plain optimizer keeps its small register footprint
// one 8 x 32 (or 256-element) tile of the optimizer launch: split-K reduce and / or the
// update, the bf16 shadows of weight tiles; block 0 also reduces the head statistics
template <int MODE>
__device__ __forceinline__ void tr_opt_tile(const TrOptArgs& a, int b, float (*tile_s)[33]) {
  const int tid = threadIdx.x;
  if (b == 0 && tid < 64 && MODE != 3 && a.nhead > 0) {
    // head statistics: reduce (modes 0/2) the per-block partials; hand the loss over (1/2);
    // nhead == 0: a segment-subset reduce launch that leaves them to another launch
    if (MODE != 1) {
      float v[4] = {0.f, 0.f, 0.f, 0.f};
      for (int k = tid; k < a.nhead; k += 64)
#pragma unroll
        for (int c = 0; c < 4; ++c) v[c] += a.head_part[k * 4 + c];
#pragma unroll
      for (int c = 0; c < 4; ++c) v[c] = wave_sum(v[c]);
      if (tid == 0) {
        a.loss_acc[0] = v[0];
        if (a.stat_f) {
          a.stat_f[0] += v[1];
        } else if (a.counts) {
          a.counts[0] += static_cast<uint32_t>(v[1]);
          a.counts[1] += static_cast<uint32_t>(v[2]);
          a.counts[2] += static_cast<uint32_t>(v[3]);
        }
        if (MODE == 2) a.loss_out[0] = v[0];
      }
    } else if (tid == 0) {
      a.loss_out[0] = a.loss_acc[0];
    }
  }
  TrSeg sg = a.seg[0];
#pragma unroll
  for (int k = 1; k < kTrMaxSegs; ++k)
    if (k < a.nseg && b >= a.seg[k].blk0) sg = a.seg[k];
  const int local = b - sg.blk0;
  int64_t i;
  int r = 0, c = 0;
  bool valid = true;
  // vector segment with slab groups (tr_seg_prepare): thread = (group, element); uniform per block
  const int grp = sg.cols == 0 && sg.sgrp > 1 ? sg.sgrp : 1;
  const int per = 256 / grp, sub = tid / per;
  if (sg.cols > 0) {  // 8 x 32 tile of a weight matrix
    const int tiles_c = sg.cols >> 5;
    const int tr = local / tiles_c, tc = local - tr * tiles_c;
    r = tr * 8 + (tid >> 5);
    c = tc * 32 + (tid & 31);
    i = sg.off + static_cast<int64_t>(r) * sg.cols + c;
  } else {
    i = sg.off + static_cast<int64_t>(local) * per + (tid - sub * per);
    valid = i < sg.off + sg.n;
    if (!valid) i = sg.off;  // clamped: no early return before the tile barrier
    valid = valid && sub == 0;  // groups 1.. only help with the slab sum
  }
  float p = a.p[i];
  // optimizer slots loaded up front: independent of the split-K sum, so their latency
  // overlaps the partial-slab loads instead of adding a round trip after them
  float m = 0.f, v = 0.f;
  if (MODE == 1 || MODE == 2) {
    m = a.m[i];
    v = a.v[i];
  }
  if (MODE != 3) {
    float g;
    if (MODE != 1) {
      // split-K slabs: 16 loads in flight, indices clamped (no branch around a load; 32 in
      // flight measured slower: 9.38 vs 8.75 us, profiles/r3_headline/)
      const float* src = sg.part + (i - sg.off);
      g = 0.f;
      // slabs sub, sub + grp, ... (grp == 1: all of them, in order)
      for (int s0 = sub; s0 < sg.S; s0 += 16 * grp) {
        float v[16];
#pragma unroll
        for (int u = 0; u < 16; ++u) {
          const int sl = s0 + u * grp;
          v[u] = src[static_cast<int64_t>(sl < sg.S ? sl : sg.S - 1) * sg.n];
        }
#pragma unroll
        for (int u = 0; u < 16; ++u) g += (s0 + u * grp < sg.S) ? v[u] : 0.f;
      }
      if (grp > 1) {  // the groups' sums, in group order (deterministic)
        float* red = &tile_s[0][0];
        red[tid] = g;
        __syncthreads();
        const int e = tid - sub * per;
        g = red[e];
        for (int q = 1; q < grp; ++q) g += red[q * per + e];
      }
      if (MODE == 0) {
        if (valid) {
          if (a.g16) a.g16[i] = f2bf(g);
          else a.g[i] = g;
        }
        return;
      }
    } else {
      g = a.g16 ? bf2f(a.g16[i]) : a.g[i];
    }
    const float t = static_cast<float>(a.step[0]);
    const float gi = g * a.grad_scale + a.wd * p;
    if (a.kind == 0) {
      const float bc1 = 1.f - __powf(a.b1, t), bc2 = 1.f - __powf(a.b2, t);
      m = a.b1 * m + (1.f - a.b1) * gi;
      v = a.b2 * v + (1.f - a.b2) * gi * gi;
      p -= a.lr * (m / bc1) / (sqrtf(v / bc2) + a.eps);
    } else if (a.kind == 1) {
      v += gi * gi;
      p -= a.lr * gi / (sqrtf(v) + a.eps);
    } else if (a.kind == 2) {
      p -= a.lr * gi;
    } else {
      m = a.b1 * m + gi;
      p -= a.lr * m;
    }
    if (valid) {
      a.p[i] = p;
      a.m[i] = m;
      a.v[i] = v;
    }
  }
  // bf16 shadows of a weight tile: rows as 16-B fm chunks (threads 0-31), columns of the
  // transpose (threads 32-63)
  if (sg.cols > 0 && sg.sh) {
    tile_s[tid >> 5][tid & 31] = p;
    __syncthreads();
    const int r0 = r - (tid >> 5), c0 = c - (tid & 31);
    if (tid < 32) {
      const int row = tid >> 2, kc = (tid & 3) * 8;
      float t8[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) t8[k] = tile_s[row][kc + k];
      *reinterpret_cast<uint4_t*>(sg.sh + fm_off(r0 + row, c0 + kc, sg.cols)) = pack_bf16x8(t8);
    } else if (tid < 64 && sg.shT) {
      const int col = tid - 32;
      float t8[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) t8[k] = tile_s[k][col];
      *reinterpret_cast<uint4_t*>(sg.shT + fm_off(c0 + col, r0, sg.rows)) = pack_bf16x8(t8);
    }
  }
}

template <int MODE, typename FT, int GATHER>
__global__ __launch_bounds__(256, GATHER ? 4 : 1) void tr_opt_kernel(TrOptArgs a) {
  __shared__ float tile_s[8][33];
  __shared__ int32_t node_s[kTrSampleRows];
  extern __shared__ __attribute__((aligned(16))) bf16_t glds[];  // gather tiles only
  int b = blockIdx.x;
  // GATHER launches: opt_tpb parameter tiles per block, so the parameter blocks take few of
  // the slots the gather tiles need
  const int tpb = GATHER && a.opt_tpb > 1 ? a.opt_tpb : 1;
  const int nopt = (a.nblk + tpb - 1) / tpb;
  if constexpr (GATHER) {
    // the next step's layer-0 gather (pipelined step): first in the grid unless
    // gather_first == 0
    if (a.gather_first) {
      if (b < a.ngather) {
        tr_gather32_tile<FT>(a.gat, b, glds);
        return;
      }
      b -= a.ngather;
    } else if (b >= nopt + a.nsample) {
      tr_gather32_tile<FT>(a.gat, b - nopt - a.nsample, glds);
      return;
    }
  }
  if (b >= nopt) {  // the next step's sampler (modes 1/2)
    tr_sample_block<256>(a.smp, b - nopt, node_s);
    return;
  }
  for (int r = 0; r < tpb; ++r) {
    const int bt = b * tpb + r;
    if (bt >= a.nblk) break;  // uniform across the block
    tr_opt_tile<MODE>(a, bt, tile_s);
    if (tpb > 1) __syncthreads();  // tile_s is reused by the next tile
  }
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

size_t eh_tr_fwd_lds(int D, int H, int bm, int FL, int mode) {
  const int K2 = 2 * D;
  const bool alias_out = H <= kTrBN && kTrBN <= K2;
  size_t b = static_cast<size_t>(bm) * (K2 + 8) * sizeof(bf16_t);
  if (mode != 1 && !alias_out) b += static_cast<size_t>(bm) * (kTrBN + 8) * sizeof(bf16_t);
  if (mode != 2) b += static_cast<size_t>(bm) * (1 + FL) * sizeof(int32_t);
  return b;
}

size_t eh_tr_fwd2_lds(int D, int FL) {
  const size_t a = static_cast<size_t>(kF2Rows) * 2 * D, o = static_cast<size_t>(kTrBN) * kF2Ldt;
  return (F2_ALIAS ? (a > o ? a : o) : a + o) * sizeof(bf16_t) + static_cast<size_t>(kF2Rows) * (1 + FL) * sizeof(int32_t);
}

// the 64-row / 8-wave layer-0 kernel applies (EULER_AMD_FWD2=0 disables it)
static bool fwd2_fits(const TrFwdArgs& a) {
  static const bool off = [] {
    const char* e = std::getenv("EULER_AMD_FWD2");
    return e && e[0] == '0';
  }();
  if (off || !a.a_kt) return false;
  if (a.D % 64 != 0 || a.M % kF2Rows != 0 || a.logPg < 2 || (1 << a.logPg) > kF2Rows) return false;
  if (F2_ALIAS && a.H > kTrBN) return false;  // the aliased A tile must outlive every column chunk
  return eh_tr_fwd2_lds(a.D, a.FL) <= 80 * 1024;  // two blocks per CU
}

hipError_t eh_tr_sample(const TrSampleArgs* a, hipStream_t s) {
  if (a->M <= 0) return hipSuccess;
  if (!a->g.indptr || !a->g.nbr || !a->g.cumw || !a->g.prob || !a->g.alias || !a->tr.rng || !a->roots ||
      !a->nodes || !a->leaf || a->FL < 1 || a->lv < 0 || a->lv > 2)
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(tr_sample_kernel, dim3(static_cast<uint32_t>(ceil_div(a->M, kTrSampleRows))), dim3(256), 0, s,
                     *a);
  return hipGetLastError();
}

hipError_t eh_tr_fwd(const TrFwdArgs* a, int mode, int feat_fp32, int bm, hipStream_t s) {
  if (a->M <= 0) return hipSuccess;
  // every pointer the chosen mode dereferences must be set
  if (!a->x || !a->a_next) return hipErrorInvalidValue;
  if (mode != 2 && (!a->nodes || !a->leaf || !a->rng || a->FL < 1 || !a->roots_in || !a->roots_cur || a->B < 1))
    return hipErrorInvalidValue;
  if (mode != 1 && !a->W) return hipErrorInvalidValue;
  if (a->D % 16 != 0 || a->D <= 0 || a->M % bm != 0) return hipErrorInvalidValue;
  if (mode != 1 && (a->H % 64 != 0 || a->H <= 0 || (bm >> a->logPg) < 1 || (bm & ((1 << a->logPg) - 1)) != 0 ||
                    a->Fg >= (1 << a->logPg)))
    return hipErrorInvalidValue;
  if (mode == 2 && feat_fp32) return hipErrorInvalidValue;
  if (a->ncomb < 0 || (a->ncomb > 0 && (mode == 2 || !a->comb.wout || !a->comb.bfc || !a->comb.Wc ||
                                        !a->comb.WcT || !a->comb.bc || !a->comb.wout_sh || !a->comb.wfcT_sh ||
                                        a->comb.C % 16 != 0 || a->comb.H % 16 != 0 || a->comb.E % 32 != 0)))
    return hipErrorInvalidValue;
  if (mode == 3) {  // GEMM-only (pipelined step): the A rows come from the gather blocks
    if (!fwd2_fits(*a) || !a->a_rows) return hipErrorInvalidValue;
    const size_t l2 = eh_tr_fwd2_lds(a->D, a->FL);
    EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(tr_fwd2_kernel<bf16_t, 1>),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(l2)));
    hipLaunchKernelGGL((tr_fwd2_kernel<bf16_t, 1>), dim3(static_cast<uint32_t>(a->M / kF2Rows)), dim3(kF2Threads), l2,
                       s, *a);
    return hipGetLastError();
  }
  if (mode == 0 && fwd2_fits(*a)) {
    const size_t l2 = eh_tr_fwd2_lds(a->D, a->FL);
    const dim3 g2(static_cast<uint32_t>(a->M / kF2Rows));
#define TR_FWD2(FT)                                                                                          \
  do {                                                                                                       \
    EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(tr_fwd2_kernel<FT, 0>),               \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(l2)));   \
    hipLaunchKernelGGL((tr_fwd2_kernel<FT, 0>), g2, dim3(kF2Threads), l2, s, *a);                            \
    return hipGetLastError();                                                                                \
  } while (0)
    if (feat_fp32) TR_FWD2(float);
    TR_FWD2(bf16_t);
#undef TR_FWD2
  }
  const size_t lds = eh_tr_fwd_lds(a->D, a->H, bm, a->FL, mode);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const dim3 grid(static_cast<uint32_t>(a->M / bm));
#define TR_FWD(FT, BMV, MODEV)                                                                               \
  do {                                                                                                       \
    EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(tr_fwd_kernel<FT, BMV, MODEV>),         \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds))); \
    hipLaunchKernelGGL((tr_fwd_kernel<FT, BMV, MODEV>), grid, dim3(256), lds, s, *a);                       \
    return hipGetLastError();                                                                                \
  } while (0)
#define TR_FWD_BM(FT, MODEV)                 \
  do {                                       \
    if (bm == 32) TR_FWD(FT, 32, MODEV);     \
    if (bm == 64) TR_FWD(FT, 64, MODEV);     \
    if (bm == 128) TR_FWD(FT, 128, MODEV);   \
  } while (0)
  if (mode == 0) {
    if (feat_fp32) TR_FWD_BM(float, 0);
    else TR_FWD_BM(bf16_t, 0);
  } else if (mode == 1) {
    if (feat_fp32) TR_FWD_BM(float, 1);
    else TR_FWD_BM(bf16_t, 1);
  } else if (mode == 2) {
    TR_FWD_BM(bf16_t, 2);
  }
#undef TR_FWD_BM
#undef TR_FWD
  return hipErrorInvalidValue;
}

size_t eh_tr_head_lds(int Hin2, int H, int E, int C, int label_mode) {
  (void)E;
  size_t el = static_cast<size_t>(HB) * ((Hin2 + 16) + 2 * (H + 16) + (C + 16));
  if (label_mode == 2) el += static_cast<size_t>(HB) * C;
  return el * sizeof(bf16_t);
}

hipError_t eh_tr_head(const TrHeadArgs* a, int64_t B, hipStream_t s) {
  if (!a->A || !a->W || !a->Wfc || !a->WfcT || !a->Wout || !a->WoutT || !a->Wc || !a->WcT || !a->bc || !a->bfc ||
      !a->roots || !a->labels ||
      !a->A_kt || !a->h_kt || !a->emb_kt || !a->dlog_kt || !a->demb_kt || !a->g_kt || !a->dbfc_part || !a->head_part ||
      (a->dA && !a->WT))
    return hipErrorInvalidValue;
  if (B % 32 != 0 || a->H % 16 != 0 || a->E % 32 != 0 || a->C % 32 != 0 || a->Hin2 % 32 != 0 ||
      a->C_real > a->C || a->C_real <= 0)
    return hipErrorInvalidValue;
  const size_t lds = eh_tr_head_lds(a->Hin2, a->H, a->E, a->C, a->label_mode);
  if (lds > 160 * 1024 - 64) return hipErrorInvalidValue;
  EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(tr_head_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  if (a->nsample > 0) {
    const TrSampleArgs& m = a->smp;
    if (!m.g.indptr || !m.g.nbr || !m.g.cumw || !m.g.prob || !m.g.alias || !m.tr.rng || !m.roots || !m.nodes ||
        !m.leaf || m.FL < 1 || m.lv < 0 || m.lv > 2 || a->nsample != ceil_div(m.M, kTrHeadSampleRows) ||
        m.roots == a->roots)
      return hipErrorInvalidValue;
  }
  hipLaunchKernelGGL(tr_head_kernel, dim3(static_cast<uint32_t>(B / HB + a->nsample)), dim3(HNW * 64), lds, s, *a);
  return hipGetLastError();
}

hipError_t eh_tr_bwd(const TrBwdArgs* a, hipStream_t s) {
  if (!a->dA || !a->mask || !a->WT || !a->dA_out) return hipErrorInvalidValue;
  if (a->M % 32 != 0 || a->Hk % 32 != 0 || a->K2out % 64 != 0 || a->logPg < 4) return hipErrorInvalidValue;
  const size_t lds = static_cast<size_t>(32) * (a->Hk + 8) * sizeof(bf16_t);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(tr_bwd_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  hipLaunchKernelGGL(tr_bwd_kernel, dim3(static_cast<uint32_t>(a->M / 32)), dim3(256), lds, s, *a);
  return hipGetLastError();
}

size_t eh_tr_pair_head_lds(int K, int H0x2, int H1, int E) {
  const size_t rows = 16 * static_cast<size_t>(2 + K);
  const size_t abytes = rows * (H0x2 + 16) * 2, ebytes = rows * E * 4, gbytes = rows * (H1 + 16) * 2;
  const size_t region = std::max(std::max(abytes, ebytes), gbytes);
  return region + rows * (H1 + 16) * 2 + rows * (E + 16) * 2 + 2 * 16 * static_cast<size_t>(E) * 4;
}

hipError_t eh_tr_pair_head(const TrPairHeadArgs* a, hipStream_t s) {
  if (a->B <= 0 || a->B % 16 != 0 || a->K < 1 || a->K > 15 || a->H0x2 % 32 != 0 || a->H1 % 32 != 0 ||
      a->E % 32 != 0 || a->E > 1024)
    return hipErrorInvalidValue;
  const TrPairTower* tw[2] = {&a->s, &a->c};
  for (const TrPairTower* t : tw)
    if (!t->A1 || !t->W1 || !t->W1T || !t->Wfc || !t->WfcT || !t->bfc || !t->A1_kt || !t->h_kt || !t->de_kt ||
        !t->g_kt || !t->dA1 || !t->dbfc_part)
      return hipErrorInvalidValue;
  if (!a->head_part) return hipErrorInvalidValue;
  const size_t lds = eh_tr_pair_head_lds(a->K, a->H0x2, a->H1, a->E);
  if (lds > 160 * 1024 - 256) return hipErrorInvalidValue;
  EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(tr_pair_head_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  hipLaunchKernelGGL(tr_pair_head_kernel, dim3(static_cast<uint32_t>(a->B / 16)), dim3(HNW * 64), lds, s, *a);
  return hipGetLastError();
}

hipError_t eh_tr_dw(TrDwLaunch* L, hipStream_t s) {
  TrDwProbs* pr = &L->plain;
  if (pr->n < 0 || pr->n > kTrMaxProbs || L->nroute < 0 || L->nroute > 2) return hipErrorInvalidValue;
  L->rwg[0] = 0;
  for (int r = 0; r < L->nroute; ++r) {
    TrDwProb* p = &L->route[r];
    if (!p->route || !p->dA || !p->mask || !p->X || !p->part) return hipErrorInvalidValue;
    if (p->P % kRP != 0 || p->Q % 32 != 0 || p->MB < 1 || p->kps < 1 || p->logPg < 3) return hipErrorInvalidValue;
    // the XCD-aware block mapping needs S % 8 == 0 (splits past MB write zero slabs)
    if (p->S % 8 != 0 || static_cast<int64_t>(p->S) * p->kps < p->MB) return hipErrorInvalidValue;
    p->tiles_q = static_cast<int>(ceil_div(p->Q, kRQ));
    p->ntiles = (p->P / kRP) * p->tiles_q;
    p->wg0 = 0;
    L->rwg[r + 1] = L->rwg[r] + p->ntiles * p->S;
  }
  int wg = 0;
  for (int i = 0; i < pr->n; ++i) {
    TrDwProb& p = pr->p[i];
    if (p.P % 32 != 0 || p.Q % 32 != 0 || p.MB < 1 || p.kps < 1) return hipErrorInvalidValue;
    if (p.route || !p.G || !p.X || !p.part) return hipErrorInvalidValue;
    if (static_cast<int64_t>(p.S) * p.kps < p.MB) return hipErrorInvalidValue;
    p.tiles_q = (p.Q + 63) / 64;
    p.ntiles = ((p.P + 63) / 64) * p.tiles_q;
    p.wg0 = wg;
    wg += p.ntiles * p.S;
  }
  const int total = L->rwg[L->nroute] + wg;
  if (total == 0) return hipSuccess;
  hipLaunchKernelGGL(tr_dw_all_kernel, dim3(static_cast<uint32_t>(total)), dim3(256), 0, s, *L);
  return hipGetLastError();
}

size_t eh_tr_gather32_lds(int D, int FL) {
  return static_cast<size_t>(kG32Rows) * 2 * D * sizeof(bf16_t) + static_cast<size_t>(kG32Rows) * (1 + FL) * sizeof(int32_t);
}

hipError_t eh_tr_opt(const TrOptArgs* ain, int mode, hipStream_t s) {
  TrOptArgs A = *ain;
  const TrOptArgs* a = &A;
  if (!(mode == 1 || mode == 2)) A.nsample = 0;  // the sampler runs in modes 1/2 only
  if (mode == 3) A.ngather = 0;
  if (a->nseg < 1 || a->nseg > kTrMaxSegs || a->nblk < 1) return hipErrorInvalidValue;
  if (!a->p || !a->g || !a->m || !a->v || !a->step || !a->loss_acc || !a->loss_out || !a->head_part ||
      a->nhead < 0 || (a->nhead == 0 && mode != 0 && mode != 3))
    return hipErrorInvalidValue;
  int blk = 0;
  for (int i = 0; i < a->nseg; ++i) {
    const TrSeg& g = a->seg[i];
    if (!g.part || g.S < 1 || g.blk0 != blk) return hipErrorInvalidValue;
    if (g.cols > 0) {
      if (g.rows % 8 != 0 || g.cols % 32 != 0 || static_cast<int64_t>(g.rows) * g.cols != g.n)
        return hipErrorInvalidValue;
    } else {
      if (g.sh || g.shT || g.sgrp != tr_seg_groups(g)) return hipErrorInvalidValue;  // tr_seg_prepare
    }
    blk += tr_seg_blocks(g);
  }
  if (blk != a->nblk) return hipErrorInvalidValue;
  int extra = 0;
  if (a->nsample > 0) {
    const TrSampleArgs& m = a->smp;
    if (!m.g.indptr || !m.g.nbr || !m.g.cumw || !m.g.prob || !m.g.alias || !m.tr.rng || !m.roots || !m.nodes ||
        !m.leaf || m.FL < 1 || m.lv < 0 || m.lv > 2 || a->nsample != ceil_div(m.M, kTrSampleRows))
      return hipErrorInvalidValue;
    extra = a->nsample;
  }
  size_t lds = 0;
  if (a->ngather > 0) {
    // every gather tile reads ids and features and writes both A copies of its 32 rows;
    // sibling groups must fit a tile (P <= 32) and rows be whole 16-byte chunks
    const TrFwdArgs& g = a->gat;
    if (!g.x || !g.nodes || !g.leaf || !g.a_kt || !g.a_rows || g.FL < 1 || g.D % 8 != 0 || g.D <= 0 ||
        g.M % kG32Rows != 0 || a->ngather != g.M / kG32Rows || g.logPg < 2 || (1 << g.logPg) > kG32Rows ||
        g.Fg >= (1 << g.logPg))
      return hipErrorInvalidValue;
    lds = eh_tr_gather32_lds(g.D, g.FL);
    if (lds > 64 * 1024) return hipErrorInvalidValue;
    extra += a->ngather;
  }
  const int tpb = a->ngather > 0 && a->opt_tpb > 1 ? a->opt_tpb : 1;
  const int nopt = (a->nblk + tpb - 1) / tpb;
  const dim3 grid(static_cast<uint32_t>(nopt + extra));
#define TR_OPT(MODEV, FT, G) hipLaunchKernelGGL((tr_opt_kernel<MODEV, FT, G>), grid, dim3(256), lds, s, A)
  if (a->ngather > 0 && a->gat_fp32) {
    if (mode == 0) TR_OPT(0, float, 1);
    else if (mode == 1) TR_OPT(1, float, 1);
    else if (mode == 2) TR_OPT(2, float, 1);
    else return hipErrorInvalidValue;
  } else if (a->ngather > 0) {
    if (mode == 0) TR_OPT(0, bf16_t, 1);
    else if (mode == 1) TR_OPT(1, bf16_t, 1);
    else if (mode == 2) TR_OPT(2, bf16_t, 1);
    else return hipErrorInvalidValue;
  } else {
    if (mode == 0) TR_OPT(0, bf16_t, 0);
    else if (mode == 1) TR_OPT(1, bf16_t, 0);
    else if (mode == 2) TR_OPT(2, bf16_t, 0);
    else if (mode == 3) TR_OPT(3, bf16_t, 0);
    else return hipErrorInvalidValue;
  }
#undef TR_OPT
  return hipGetLastError();
}

}  // extern "C"
