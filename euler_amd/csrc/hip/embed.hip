// Embedding-training kernels:
//
//   sgns_fwd / sgns_bwd  (K11) skip-gram / unsupervised sigmoid-CE over
//       logits[b, k] = <emb[b], ctx[b, k]>, label 1 for the P positives, 0 for the K negatives
//       (reference mp_utils/base.py:80-91, solution/logits.py:30-34: a batched matmul, two
//       sigmoid-CE ops, a concat and a mean; and the same again in the backward)
//   kg_fwd / kg_bwd      (K10) TransE (L1 / L2) and DistMult scores that gather the entity /
//       relation rows straight from the tables, L2-normalise them in registers and, in the
//       backward, push the row gradients through the normalisation and atomically into the
//       fp32 table gradients (reference examples/TransX/transX.py:72-145,
//       distmult.py:74-77: 4 embedding lookups, 4 normalisations, tile copies per negative).
//
// Both map one row b to a group of lanes (4 fp32 / 8 bf16 columns per lane) like gat.hip,
// so a wave covers several short rows and the row reductions are group shuffles.
#include "hip/common.h"
#include "hip/launchers.h"

#include <hipcub/hipcub.hpp>

namespace euler_hip {

template <typename T>
struct EV;
template <>
struct EV<bf16_t> {
  static constexpr int N = 8;
  __device__ __forceinline__ static void load(const bf16_t* p, float* f) {
    const uint4_t u = *reinterpret_cast<const uint4_t*>(p);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      f[2 * i] = __uint_as_float(u[i] << 16);
      f[2 * i + 1] = __uint_as_float(u[i] & 0xffff0000u);
    }
  }
  __device__ __forceinline__ static void store(bf16_t* p, const float* f) {
    *reinterpret_cast<uint4_t*>(p) = pack_bf16x8(f);
  }
};
template <>
struct EV<float> {
  static constexpr int N = 4;
  __device__ __forceinline__ static void load(const float* p, float* f) {
    const float4_t u = *reinterpret_cast<const float4_t*>(p);
    f[0] = u[0];
    f[1] = u[1];
    f[2] = u[2];
    f[3] = u[3];
  }
  __device__ __forceinline__ static void store(float* p, const float* f) {
    *reinterpret_cast<float4_t*>(p) = float4_t{f[0], f[1], f[2], f[3]};
  }
};

// sum over aligned groups of g lanes; all lanes of a group follow the same path
__device__ __forceinline__ float emb_group_sum(float v, int g) {
  for (int o = g >> 1; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

struct RowLane {
  int64_t row;
  int sub;
  bool ok;
};
__device__ __forceinline__ RowLane row_lane(int lp, int64_t rows) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  RowLane r;
  r.row = wave * (64 / lp) + lane / lp;
  r.sub = lane & (lp - 1);
  r.ok = r.row < rows;
  return r;
}

// numerically stable sigmoid cross-entropy with logits
__device__ __forceinline__ float sigmoid_ce(float x, float y) {
  return fmaxf(x, 0.f) - x * y + __logf(1.f + __expf(-fabsf(x)));
}
__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + __expf(-x)); }

// ----------------------------------------------------------------------------- K11
// emb [B, D], pos [B, P, D], neg [B, K, D]; a row is D/V chunks, one per lane of its group
template <typename T>
__global__ __launch_bounds__(256) void sgns_fwd_kernel(const T* __restrict__ emb, const T* __restrict__ pos,
                                                       const T* __restrict__ neg, int64_t B, int P, int K, int D,
                                                       int lp, float* __restrict__ logits,
                                                       float* __restrict__ loss_rows) {
  constexpr int V = EV<T>::N;
  const RowLane L = row_lane(lp, B);
  const bool ok = L.ok && L.sub * V < D;
  float e[V], c[V];
#pragma unroll
  for (int v = 0; v < V; ++v) e[v] = 0.f;
  if (ok) EV<T>::load(emb + L.row * D + L.sub * V, e);
  float loss = 0.f;
  const int KK = P + K;
  for (int k = 0; k < KK; ++k) {
    const bool is_pos = k < P;
    float part = 0.f;
    if (ok) {
      const T* src = is_pos ? pos + (L.row * P + k) * D : neg + (L.row * K + (k - P)) * D;
      EV<T>::load(src + L.sub * V, c);
#pragma unroll
      for (int v = 0; v < V; ++v) part += e[v] * c[v];
    }
    const float x = emb_group_sum(part, lp);
    loss += sigmoid_ce(x, is_pos ? 1.f : 0.f);
    if (L.ok && L.sub == 0) logits[L.row * KK + k] = x;
  }
  if (L.ok && L.sub == 0) loss_rows[L.row] = loss;
}

// g_bk = (sigmoid(x) - y) * gscale ; demb = sum_k g ctx ; dctx = g emb
template <typename T>
__global__ __launch_bounds__(256) void sgns_bwd_kernel(const T* __restrict__ emb, const T* __restrict__ pos,
                                                       const T* __restrict__ neg, int64_t B, int P, int K, int D,
                                                       int lp, const float* __restrict__ logits, float gscale,
                                                       T* __restrict__ demb, T* __restrict__ dpos,
                                                       T* __restrict__ dneg) {
  constexpr int V = EV<T>::N;
  const RowLane L = row_lane(lp, B);
  if (!L.ok || L.sub * V >= D) return;  // no cross-lane exchange in the backward
  float e[V], c[V], de[V], dc[V];
  EV<T>::load(emb + L.row * D + L.sub * V, e);
#pragma unroll
  for (int v = 0; v < V; ++v) de[v] = 0.f;
  const int KK = P + K;
  for (int k = 0; k < KK; ++k) {
    const bool is_pos = k < P;
    const int64_t off = is_pos ? (L.row * P + k) * D : (L.row * K + (k - P)) * D;
    const float g = (sigmoidf(logits[L.row * KK + k]) - (is_pos ? 1.f : 0.f)) * gscale;
    EV<T>::load((is_pos ? pos : neg) + off + L.sub * V, c);
#pragma unroll
    for (int v = 0; v < V; ++v) {
      de[v] += g * c[v];
      dc[v] = g * e[v];
    }
    EV<T>::store((is_pos ? dpos : dneg) + off + L.sub * V, dc);
  }
  EV<T>::store(demb + L.row * D + L.sub * V, de);
}

// ----------------------------------------------------------------------------- K11b
// Index-driven skip-gram step with no per-pair gradient rows (DeepWalk / LINE tables).
// A step has P pairs, each with one positive and K negatives.  Rows are addressed through
// two levels: inv (per occurrence, into the de-duplicated ids) and map (unique id -> table
// row; null = identity).  Context occurrences are ordered [P positives | P*K negatives].
//
//   sgns_fwd_idx : logits straight from the tables, writes coef[p, s] = (sigmoid(x) - y) * gscale
//   sgns_update  : per UNIQUE row u, its gradient is rebuilt from the occurrence list of u
//                  (CSR over inv: occ_fill) instead of being scattered from per-pair rows:
//                    side 0 (target):  g_u = sum_{p in occ(u)} sum_s coef[p, s] * C[ctx(p, s)]
//                    side 1 (context): g_u = sum_{(p,s) in occ(u)} coef[p, s] * E[tgt(p)]
//                  then either written out (sharded tables: sent to the owners) or applied in
//                  place with row-sparse Adam / Adagrad / SGD (one rank owns every row).
// Compared with sgns_bwd + index_add_rows + sparse_optim this drops the per-pair gradient
// rows (P*(1+K)*D*4 bytes written and read back), the zero fill of the accumulator, every
// float atomic, and the accumulator round trip.

// table row of occurrence i, or -1 when the row is outside [0, n) (the load is skipped)
// (map holds n_map entries; inv values outside it are dropped as well)
__device__ __forceinline__ int64_t occ_row(const int64_t* __restrict__ map, int64_t n_map,
                                           const int64_t* __restrict__ inv, int64_t i, int64_t n) {
  const int64_t u = inv[i];
  if (map && (u < 0 || u >= n_map)) return -1;
  const int64_t r = map ? map[u] : u;
  return r >= 0 && r < n ? r : -1;
}
__device__ __forceinline__ void load_row4(const float* __restrict__ base, int64_t r, int D, int d, float* x) {
  if (r >= 0) {
    EV<float>::load(base + r * D + d, x);
  } else {
    x[0] = x[1] = x[2] = x[3] = 0.f;
  }
}
typedef uint32_t tl2u __attribute__((ext_vector_type(2)));  // 4 bf16 = one 8-byte load

// fp32 or bf16 rows (bf: the exchanged rows of a sharded table stay in the bf16 wire dtype)
__device__ __forceinline__ void load_row4v(const void* __restrict__ base, int bf, int64_t r, int D, int d, float* x) {
  if (!bf) {
    load_row4(static_cast<const float*>(base), r, D, d, x);
    return;
  }
  if (r >= 0) {
    const tl2u v = *reinterpret_cast<const tl2u*>(static_cast<const bf16_t*>(base) + r * D + d);
    x[0] = bf2f(static_cast<bf16_t>(v[0] & 0xffffu));
    x[1] = bf2f(static_cast<bf16_t>(v[0] >> 16));
    x[2] = bf2f(static_cast<bf16_t>(v[1] & 0xffffu));
    x[3] = bf2f(static_cast<bf16_t>(v[1] >> 16));
  } else {
    x[0] = x[1] = x[2] = x[3] = 0.f;
  }
}

// context occurrence index of slot s (0 = positive) of pair p
__device__ __forceinline__ int64_t ctx_occ(int64_t p, int s, int64_t P, int K) {
  return s == 0 ? p : P + p * K + (s - 1);
}

__global__ __launch_bounds__(256) void sgns_fwd_idx_kernel(const void* __restrict__ T, const int64_t* __restrict__ tmap,
                                                           int64_t nTm, const int64_t* __restrict__ tinv, int64_t nT,
                                                           const void* __restrict__ C, int bf,
                                                           const int64_t* __restrict__ cmap, int64_t nCm,
                                                           const int64_t* __restrict__ cinv, int64_t nC, int64_t P,
                                                           int K, int D,
                                                           int lp, float gscale, float* __restrict__ coef,
                                                           float* __restrict__ loss_rows) {
  const RowLane L = row_lane(lp, P);
  const bool ok = L.ok && L.sub * 4 < D;
  const int d = L.sub * 4;
  float e[4] = {0.f, 0.f, 0.f, 0.f};
  if (ok) load_row4v(T, bf, occ_row(tmap, nTm, tinv, L.row, nT), D, d, e);
  float loss = 0.f;
  // SG context rows per round: their index chains and row loads are all in flight together
  constexpr int SG = 4;
  for (int s0 = 0; s0 <= K; s0 += SG) {
    int64_t r[SG];
    float c[SG][4];
#pragma unroll
    for (int j = 0; j < SG; ++j)
      r[j] = ok && s0 + j <= K ? occ_row(cmap, nCm, cinv, ctx_occ(L.row, s0 + j, P, K), nC) : -1;
#pragma unroll
    for (int j = 0; j < SG; ++j) load_row4v(C, bf, r[j], D, d, c[j]);
#pragma unroll
    for (int j = 0; j < SG; ++j) {
      const int s = s0 + j;
      if (s > K) break;  // uniform across the group
      float part = 0.f;
#pragma unroll
      for (int v = 0; v < 4; ++v) part += e[v] * c[j][v];
      const float x = emb_group_sum(part, lp);
      const float y = s == 0 ? 1.f : 0.f;
      loss += sigmoid_ce(x, y);
      if (L.ok && L.sub == 0) coef[L.row * (K + 1) + s] = (sigmoidf(x) - y) * gscale;
    }
  }
  if (L.ok && L.sub == 0) loss_rows[L.row] = loss;
}

// occurrence lists: list[ptr[inv[o]] + k] = o (order inside a list follows the atomics)
__global__ __launch_bounds__(256) void occ_fill_kernel(const int64_t* __restrict__ inv, int64_t n,
                                                       const int64_t* __restrict__ ptr, int* __restrict__ cursor,
                                                       int* __restrict__ list) {
  const int64_t o = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (o >= n) return;
  const int64_t u = inv[o];
  list[ptr[u] + atomicAdd(cursor + u, 1)] = static_cast<int>(o);
}

// occurrence counts: cnt[inv[o]] += 1 (int32, exact); the first thread also zeroes ptr[0]
__global__ __launch_bounds__(256) void occ_count_kernel(const int64_t* __restrict__ inv, int64_t n,
                                                        int* __restrict__ cnt, int64_t* __restrict__ ptr) {
  const int64_t o = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (o == 0) ptr[0] = 0;
  if (o >= n) return;
  atomicAdd(cnt + inv[o], 1);
}

// deterministic occurrence CSR (keys < 0 skipped): counts + scan for ptr, and a stable
// radix sort of (key, occurrence id) over the key's bits only for perm, so every segment's
// occurrences are in ascending id order and a segment sum over perm adds in that order
__global__ __launch_bounds__(256) void det_count_kernel(const int64_t* __restrict__ keys, int64_t n, int64_t S,
                                                        int* __restrict__ cnt, int64_t* __restrict__ ptr) {
  const int64_t o = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (o == 0) ptr[0] = 0;
  // runs of equal keys inside a wave (target-major edge lists, hub rows) add once per run:
  // the run's first lane adds its length, so a hot key costs one atomic per wave, not 64
  const int lane = threadIdx.x & 63;
  const int64_t k = o < n ? keys[o] : -1;
  const int64_t prev = __shfl_up(k, 1, 64);
  const bool head = lane == 0 || prev != k;
  const unsigned long long heads = __ballot(head);
  if (head && k >= 0 && k < S) {
    const unsigned long long rest = lane == 63 ? 0ull : (heads >> (lane + 1));
    const int len = rest ? __ffsll(static_cast<long long>(rest)) : 64 - lane;
    atomicAdd(cnt + k, len);
  }
}

// the radix sort's inputs: 32-bit keys (a skipped key sorts last, as S) and occurrence ids
__global__ __launch_bounds__(256) void det_prep_kernel(const int64_t* __restrict__ keys, int64_t n, int64_t S,
                                                       int* __restrict__ k32, int* __restrict__ iota) {
  const int64_t o = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (o >= n) return;
  const int64_t k = keys[o];
  k32[o] = (k >= 0 && k < S) ? static_cast<int>(k) : static_cast<int>(S);
  iota[o] = static_cast<int>(o);
}

// out[s] = sum of src[perm[e]] over e in [ptr[s], ptr[s + 1]), in a fixed order: one block
// per segment, row e on row-slot (e - ptr[s]) % RB (RB = 256 / (D / 4) slots side by side,
// U rows of each slot in flight), each slot summing its rows in order, then the slot
// partials added in slot order through LDS.  A hot row's occurrences spread over the whole
// block instead of one wave's serial chain.  fp32, D / 4 a power of two <= 64.
__global__ __launch_bounds__(256) void det_segsum_kernel(const float* __restrict__ src, int D,
                                                         const int64_t* __restrict__ ptr,
                                                         const int* __restrict__ perm, int64_t S,
                                                         float* __restrict__ out) {
  __shared__ __attribute__((aligned(16))) float red[256 * 4];
  const int LP = D >> 2, RB = 256 / LP;
  const int tid = threadIdx.x, slot = tid / LP, d0 = (tid - slot * LP) * 4;
  constexpr int U = 4;
  for (int64_t s = blockIdx.x; s < S; s += gridDim.x) {  // uniform per block
    const int64_t a = ptr[s], b = ptr[s + 1];
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    for (int64_t e0 = a + slot; e0 < b; e0 += static_cast<int64_t>(RB) * U) {
      int64_t row[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e = e0 + static_cast<int64_t>(u) * RB;
        row[u] = e < b ? static_cast<int64_t>(perm[e]) : -1;
      }
      float v[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (row[u] >= 0) {
          EV<float>::load(src + row[u] * D + d0, v[u]);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i) v[u][i] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] += v[u][i];
    }
    if (b - a <= 1) {  // one row (or none): no combine needed, slot 0 holds it
      if (slot == 0) EV<float>::store(out + s * D + d0, acc);
      continue;
    }
#pragma unroll
    for (int i = 0; i < 4; ++i) red[slot * D + d0 + i] = acc[i];
    __syncthreads();
    if (tid < LP) {
      float t[4] = {0.f, 0.f, 0.f, 0.f};
      for (int r = 0; r < RB; ++r)
#pragma unroll
        for (int i = 0; i < 4; ++i) t[i] += red[r * D + tid * 4 + i];
      EV<float>::store(out + s * D + tid * 4, t);
    }
    __syncthreads();
  }
}

struct SgnsUpd {
  const int64_t* ptr;   // [n_u + 1]
  const int* list;      // occurrence ids
  const float* coef;    // [P, K + 1]
  const void* src;      // rows the gradient is built from (fp32, or bf16 when src_bf16)
  const int64_t* smap;  // unique id -> src row (null = identity)
  const int64_t* sinv;  // occurrence -> unique id of the OTHER table (side 0: context occ, side 1: target occ)
  void* gout;           // [n_u, D] (fp32, or bf16 when gout_bf16) or null (apply the optimizer instead)
  float* table;
  float* m;
  float* v;
  const int64_t* rows;  // unique id -> row of `table` (null = identity)
  const int64_t* step;
  int64_t n_u, P, n_rows, n_src, n_smap;
  int K, D, lp, split, lsh, side, kind;  // lsh = log2(lp * split)
  float lr, b1, b2, eps;
  int src_bf16, gout_bf16;
};

// One row group of lpe = lp * split lanes per unique id (lpe <= 256): `split` sub-groups of
// lp lanes walk the occurrence list with stride split; partial gradients are summed with xor
// shuffles at multiples of lp inside a wave and, for row groups wider than a wave, through
// LDS in wave order.  Lanes outside the table width or the id range stay live (no work) up to
// that exchange, so the barrier sees every wave.  split > 1 only when the ids alone cannot
// fill the chip (eh_sgns_update): small graphs with long occurrence lists shorten their chains.
// kWide (lpe > 64) is its own instantiation: the wave-sized one keeps early exits and no LDS.
template <bool kWide>
__global__ __launch_bounds__(256) void sgns_update_kernel(SgnsUpd a) {
  const int lpe = a.lp * a.split;
  const int64_t gt = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int64_t row = gt >> a.lsh;
  const int lsub = static_cast<int>(gt) & (lpe - 1);
  const int sub = lsub & (a.lp - 1), part = lsub / a.lp;
  const int d = sub * 4;
  // the table row, its slots and the occurrence range are loaded first, so their latency
  // overlaps the dependent index chain of the gradient below
  const bool apply = a.gout == nullptr;
  bool live = row < a.n_u && d < a.D;
  if constexpr (!kWide) {
    if (!live) return;  // partners share the row and the column slice
  }
  int64_t r = -1;
  float4_t p{}, mi{}, vi{};
  if (live && apply) {
    r = a.rows ? a.rows[row] : row;
    live = r >= 0 && r < a.n_rows;  // uniform over the row group
    if constexpr (!kWide) {
      if (!live) return;
    }
  }
  if (live && apply && part == 0) {
    const int64_t off = r * a.D + d;
    p = *reinterpret_cast<const float4_t*>(a.table + off);
    if (a.kind != 2) vi = *reinterpret_cast<const float4_t*>(a.v + off);
    if (a.kind == 0) mi = *reinterpret_cast<const float4_t*>(a.m + off);
  }
  float g[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t beg = live ? a.ptr[row] : 0, end = live ? a.ptr[row + 1] : 0;
  const int KK = a.K + 1;
  constexpr int SG = 4;
  for (int64_t i = beg + part; i < end; i += a.split) {
    const int64_t o = a.list[i];
    if (a.side == 0) {
      // target occurrence o is pair o: all of its context rows, SG at a time
      for (int s0 = 0; s0 < KK; s0 += SG) {
        int64_t rr[SG];
        float c[SG][4];
#pragma unroll
        for (int j = 0; j < SG; ++j)
          rr[j] = s0 + j < KK ? occ_row(a.smap, a.n_smap, a.sinv, ctx_occ(o, s0 + j, a.P, a.K), a.n_src) : -1;
#pragma unroll
        for (int j = 0; j < SG; ++j) load_row4v(a.src, a.src_bf16, rr[j], a.D, d, c[j]);
#pragma unroll
        for (int j = 0; j < SG; ++j) {
          const float w = s0 + j < KK ? a.coef[o * KK + s0 + j] : 0.f;
#pragma unroll
          for (int k = 0; k < 4; ++k) g[k] += w * c[j][k];
        }
      }
    } else {
      // context occurrence o -> (pair, slot)
      int64_t pp;
      int s;
      if (o < a.P) {
        pp = o;
        s = 0;
      } else {
        const int64_t q = o - a.P;
        pp = q / a.K;
        s = 1 + static_cast<int>(q - pp * a.K);
      }
      float e[4];
      const float w = a.coef[pp * KK + s];
      load_row4v(a.src, a.src_bf16, occ_row(a.smap, a.n_smap, a.sinv, pp, a.n_src), a.D, d, e);
#pragma unroll
      for (int k = 0; k < 4; ++k) g[k] += w * e[k];
    }
  }
  for (int o = a.lp; o < lpe && o < 64; o <<= 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) g[k] += __shfl_xor(g[k], o, 64);
  }
  if constexpr (kWide) {
    // lpe is a multiple of 64: the row's waves are consecutive in the block
    __shared__ float4_t red[4][64];
    const int w = threadIdx.x >> 6, lane = threadIdx.x & 63;
    if (lane < a.lp) red[w][lane] = float4_t{g[0], g[1], g[2], g[3]};
    __syncthreads();
    if (part != 0) return;
    const int nw = lpe >> 6;
    float4_t t = red[w][sub];
    for (int j = 1; j < nw; ++j) t += red[w + j][sub];
#pragma unroll
    for (int k = 0; k < 4; ++k) g[k] = t[k];
  }
  if (part != 0 || !live) return;
  if (!apply) {
    // rows without occurrences on this side are left untouched: two launches (target and
    // context side) can fill one buffer whose rows each belong to exactly one side
    if (end > beg) {
      if (a.gout_bf16) {
        tl2u v;
        v[0] = pack_bf16x2(g[0], g[1]);
        v[1] = pack_bf16x2(g[2], g[3]);
        *reinterpret_cast<tl2u*>(static_cast<bf16_t*>(a.gout) + row * a.D + d) = v;
      } else {
        EV<float>::store(static_cast<float*>(a.gout) + row * a.D + d, g);
      }
    }
    return;
  }
  const int64_t off = r * a.D + d;
  if (a.kind == 0) {
    const float st = static_cast<float>(a.step[0]);
    const float bc1 = 1.f - __powf(a.b1, st), bc2 = 1.f - __powf(a.b2, st);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mi[k] = a.b1 * mi[k] + (1.f - a.b1) * g[k];
      vi[k] = a.b2 * vi[k] + (1.f - a.b2) * g[k] * g[k];
      p[k] -= a.lr * (mi[k] / bc1) / (sqrtf(vi[k] / bc2) + a.eps);
    }
    *reinterpret_cast<float4_t*>(a.m + off) = mi;
    *reinterpret_cast<float4_t*>(a.v + off) = vi;
  } else if (a.kind == 1) {
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      vi[k] += g[k] * g[k];
      p[k] -= a.lr * g[k] / (sqrtf(vi[k]) + a.eps);
    }
    *reinterpret_cast<float4_t*>(a.v + off) = vi;
  } else {
#pragma unroll
    for (int k = 0; k < 4; ++k) p[k] -= a.lr * g[k];
  }
  *reinterpret_cast<float4_t*>(a.table + off) = p;
}

__global__ void sgns_step_inc_kernel(int64_t* step) { step[0] += 1; }

// ----------------------------------------------------------------------------- K10
// score kinds: 0 TransE-L1, 1 TransE-L2, 2 DistMult.  corrupt: 0 front (neg replaces src),
// 1 tail (neg replaces dst), 2 both (front scores then tail scores).  Tables fp32 [*, D].
struct KgArgs {
  const float* ent;
  const float* rel;
  const int64_t* src;
  const int64_t* dst;
  const int64_t* ridx;
  const int64_t* neg;
  int64_t B;
  int K, D, kind, corrupt, normalize, lp;
};

__device__ __forceinline__ void kg_load_norm(const float* tab, int64_t row, int sub, int D, int lp, bool normalize,
                                             float* x, float& nrm) {
  float part = 0.f;
#pragma unroll
  for (int v = 0; v < 4; ++v) x[v] = 0.f;
  if (sub * 4 < D && row >= 0) {
    EV<float>::load(tab + row * D + sub * 4, x);
#pragma unroll
    for (int v = 0; v < 4; ++v) part += x[v] * x[v];
  }
  nrm = 1.f;
  if (normalize) {
    nrm = fmaxf(sqrtf(emb_group_sum(part, lp)), 1e-12f);
#pragma unroll
    for (int v = 0; v < 4; ++v) x[v] /= nrm;
  }
}

// this lane's part of a score; the caller reduces over the group
__device__ __forceinline__ float kg_part(int kind, const float* h, const float* r, const float* t) {
  float p = 0.f;
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    if (kind == 2) {
      p += h[v] * r[v] * t[v];
    } else {
      const float d = h[v] + r[v] - t[v];
      p += kind == 0 ? fabsf(d) : d * d;
    }
  }
  return p;
}

__device__ __forceinline__ float kg_finish(int kind, float s) {
  return kind == 0 ? -s : (kind == 1 ? -sqrtf(s) : s);
}

__global__ __launch_bounds__(256) void kg_fwd_kernel(KgArgs a, float* __restrict__ pos_score,
                                                     float* __restrict__ neg_score) {
  const RowLane L = row_lane(a.lp, a.B);
  if (!L.ok) return;  // whole lane groups exit together
  float h[4], r[4], t[4], n[4], nh, nr, nt, nn;
  kg_load_norm(a.ent, a.src[L.row], L.sub, a.D, a.lp, a.normalize, h, nh);
  kg_load_norm(a.rel, a.ridx[L.row], L.sub, a.D, a.lp, a.normalize, r, nr);
  kg_load_norm(a.ent, a.dst[L.row], L.sub, a.D, a.lp, a.normalize, t, nt);
  const float ps = kg_finish(a.kind, emb_group_sum(kg_part(a.kind, h, r, t), a.lp));
  if (L.sub == 0) pos_score[L.row] = ps;
  const int nneg = a.corrupt == 2 ? 2 * a.K : a.K;
  for (int k = 0; k < a.K; ++k) {
    kg_load_norm(a.ent, a.neg[L.row * a.K + k], L.sub, a.D, a.lp, a.normalize, n, nn);
    if (a.corrupt != 1) {  // front
      const float s = kg_finish(a.kind, emb_group_sum(kg_part(a.kind, n, r, t), a.lp));
      if (L.sub == 0) neg_score[L.row * nneg + k] = s;
    }
    if (a.corrupt != 0) {  // tail
      const float s = kg_finish(a.kind, emb_group_sum(kg_part(a.kind, h, r, n), a.lp));
      if (L.sub == 0) neg_score[L.row * nneg + (a.corrupt == 2 ? a.K : 0) + k] = s;
    }
  }
}

// d score / d (h, r, t) of one score with upstream g, accumulated into dh, dr, dt
__device__ __forceinline__ void kg_grad(int kind, int lp, float g, const float* h, const float* r, const float* t,
                                        float* dh, float* dr, float* dt) {
  float coef = 1.f;
  if (kind == 1) {
    float p = 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v) {
      const float d = h[v] + r[v] - t[v];
      p += d * d;
    }
    const float nrm = sqrtf(emb_group_sum(p, lp));
    // 0 below 1e-12 (a triple already satisfied exactly): 1 / nrm of a denormal norm is
    // inf and 0 * inf = NaN on the components with d = 0
    coef = nrm > 1e-12f ? 1.f / nrm : 0.f;
  }
#pragma unroll
  for (int v = 0; v < 4; ++v) {
    if (kind == 2) {
      dh[v] += g * r[v] * t[v];
      dr[v] += g * h[v] * t[v];
      dt[v] += g * h[v] * r[v];
    } else {
      const float d = h[v] + r[v] - t[v];
      // score = -|d|_1  or  -|d|_2
      const float gd = -g * (kind == 0 ? (d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f)) : d * coef);
      dh[v] += gd;
      dr[v] += gd;
      dt[v] -= gd;
    }
  }
}

// push the gradient w.r.t. a normalised row through x / |x| and add it to the table grad
// (occ: store it as occurrence row ``row`` instead — summed per table row afterwards by a
// segment reduction, no atomics on hot rows)
__device__ __forceinline__ void kg_scatter(float* __restrict__ dtab, int64_t row, int sub, int D, int lp,
                                           bool normalize, const float* xhat, float nrm, float* dx, bool occ = false) {
  if (normalize) {
    float p = 0.f;
#pragma unroll
    for (int v = 0; v < 4; ++v) p += xhat[v] * dx[v];
    const float dot = emb_group_sum(p, lp);
#pragma unroll
    for (int v = 0; v < 4; ++v) dx[v] = (dx[v] - xhat[v] * dot) / nrm;
  }
  if (sub * 4 < D && row >= 0) {
    if (occ) {
      EV<float>::store(dtab + row * D + sub * 4, dx);
      return;
    }
#pragma unroll
    for (int v = 0; v < 4; ++v) atomicAdd(dtab + row * D + sub * 4 + v, dx[v]);
  }
}

__global__ __launch_bounds__(256) void kg_bwd_kernel(KgArgs a, const float* __restrict__ gpos,
                                                     const float* __restrict__ gneg, float* __restrict__ dent,
                                                     float* __restrict__ drel, int occ) {
  const RowLane L = row_lane(a.lp, a.B);
  if (!L.ok) return;
  float h[4], r[4], t[4], n[4], nh, nr, nt, nn;
  float dh[4] = {0.f, 0.f, 0.f, 0.f}, dr[4] = {0.f, 0.f, 0.f, 0.f}, dt[4] = {0.f, 0.f, 0.f, 0.f};
  const int64_t hs = a.src[L.row], rs = a.ridx[L.row], ts = a.dst[L.row];
  kg_load_norm(a.ent, hs, L.sub, a.D, a.lp, a.normalize, h, nh);
  kg_load_norm(a.rel, rs, L.sub, a.D, a.lp, a.normalize, r, nr);
  kg_load_norm(a.ent, ts, L.sub, a.D, a.lp, a.normalize, t, nt);
  kg_grad(a.kind, a.lp, gpos[L.row], h, r, t, dh, dr, dt);
  const int nneg = a.corrupt == 2 ? 2 * a.K : a.K;
  for (int k = 0; k < a.K; ++k) {
    const int64_t ns = a.neg[L.row * a.K + k];
    kg_load_norm(a.ent, ns, L.sub, a.D, a.lp, a.normalize, n, nn);
    float dn[4] = {0.f, 0.f, 0.f, 0.f};
    if (a.corrupt != 1) kg_grad(a.kind, a.lp, gneg[L.row * nneg + k], n, r, t, dn, dr, dt);
    if (a.corrupt != 0)
      kg_grad(a.kind, a.lp, gneg[L.row * nneg + (a.corrupt == 2 ? a.K : 0) + k], h, r, n, dh, dr, dn);
    // occurrence rows of triple i: [h, t, neg_0 .. neg_{K-1}] (entities), i (relation)
    kg_scatter(dent, occ ? L.row * (2 + a.K) + 2 + k : ns, L.sub, a.D, a.lp, a.normalize, n, nn, dn, occ);
  }
  kg_scatter(dent, occ ? L.row * (2 + a.K) : hs, L.sub, a.D, a.lp, a.normalize, h, nh, dh, occ);
  kg_scatter(drel, occ ? L.row : rs, L.sub, a.D, a.lp, a.normalize, r, nr, dr, occ);
  kg_scatter(dent, occ ? L.row * (2 + a.K) + 1 : ts, L.sub, a.D, a.lp, a.normalize, t, nt, dt, occ);
}

// ----------------------------------------------------------------------------- K10b
// One TransE margin step on an encoder's output without torch glue (the R-GCN + TransE
// training step of BASELINE config 5, models/rgcn_kg_step.py).
//   fwd: each lane group draws its triple (uniform over `pool`) and K corruptions
//        (uniform entities) with Philox(seed, step, row), scores the triple and its 2K
//        front / tail corruptions, and keeps
//          loss_i = relu(margin + mean_k neg_ik - pos_i),   c_i = [loss_i > 0] / B,
//        plus one partial loss sum per block (no atomics: the bwd kernel's block 0 adds the
//        partials in a fixed order);
//   bwd: d loss / d pos_i = -c_i, d loss / d neg_ik = c_i / 2K, pushed through the scores
//        into the encoder-output and relation-table gradients (kg_grad / kg_scatter).
struct KgStepArgs {
  KgArgs k;  // ent = the encoder output h; src / dst / ridx / neg = the o_* buffers below
  int64_t *o_src, *o_dst, *o_ridx, *o_neg;
  const int64_t* pool;  // candidate triple rows
  const int64_t* t_src;  // training triples
  const int64_t* t_dst;
  const int64_t* t_rel;
  int64_t P, num_ent;
  const int64_t* step;  // Philox counter: the optimizer's step count (advanced by its launch)
  uint64_t seed;
  float margin;
  float* coef;  // [B]
  float* part;  // [blocks of the fwd launch]
  float* loss;  // [1]
  int nparts;
  float* drel_rep;     // [rep][R][D] relation-gradient replicas (rep == 0: add into drel directly)
  int64_t rep_stride;  // R * D
  int rep;
  int64_t* key_e;  // deterministic mode: entity of every occurrence row (-1: no gradient)
  int64_t* key_r;  // relation of every triple's relation row (-1: no gradient)
};

// drel += sum of the replicas (fixed order)
__global__ __launch_bounds__(256) void kg_rep_reduce_kernel(const float* __restrict__ rep, int nrep, int64_t n,
                                                            float* __restrict__ drel) {
  grid_stride(n, [&](int64_t i) {
    float v = 0.f;
    for (int r = 0; r < nrep; ++r) v += rep[static_cast<int64_t>(r) * n + i];
    drel[i] += v;
  });
}

__device__ __forceinline__ uint32_t kg_word(uint64_t seed, uint64_t ctr, int64_t row, int w) {
  const uint4_t r = Philox::gen(seed, ctr, static_cast<uint64_t>(row) * 64u + static_cast<uint64_t>(w >> 2));
  return r[w & 3];
}

__global__ __launch_bounds__(256) void kg_step_fwd_kernel(KgStepArgs s) {
  __shared__ float red[4];
  const KgArgs& a = s.k;
  const RowLane L = row_lane(a.lp, a.B);
  float li = 0.f;
  if (L.ok) {
    const uint64_t ctr = static_cast<uint64_t>(s.step[0]);
    const int64_t pi = static_cast<int64_t>((static_cast<uint64_t>(kg_word(s.seed, ctr, L.row, 0)) *
                                             static_cast<uint64_t>(s.P)) >> 32);
    const int64_t tri = s.pool[pi];
    const int64_t hs = s.t_src[tri], rs = s.t_rel[tri], ts = s.t_dst[tri];
    if (L.sub == 0) {
      s.o_src[L.row] = hs;
      s.o_ridx[L.row] = rs;
      s.o_dst[L.row] = ts;
    }
    float h[4], r[4], t[4], n[4], nh, nr, nt, nn;
    kg_load_norm(a.ent, hs, L.sub, a.D, a.lp, a.normalize, h, nh);
    kg_load_norm(a.rel, rs, L.sub, a.D, a.lp, a.normalize, r, nr);
    kg_load_norm(a.ent, ts, L.sub, a.D, a.lp, a.normalize, t, nt);
    const float ps = kg_finish(a.kind, emb_group_sum(kg_part(a.kind, h, r, t), a.lp));
    float nsum = 0.f;
    for (int k = 0; k < a.K; ++k) {
      const int64_t ns = static_cast<int64_t>((static_cast<uint64_t>(kg_word(s.seed, ctr, L.row, 1 + k)) *
                                               static_cast<uint64_t>(s.num_ent)) >> 32);
      if (L.sub == 0) s.o_neg[L.row * a.K + k] = ns;
      kg_load_norm(a.ent, ns, L.sub, a.D, a.lp, a.normalize, n, nn);
      nsum += kg_finish(a.kind, emb_group_sum(kg_part(a.kind, n, r, t), a.lp));   // front
      nsum += kg_finish(a.kind, emb_group_sum(kg_part(a.kind, h, r, n), a.lp));   // tail
    }
    li = fmaxf(s.margin + nsum / static_cast<float>(2 * a.K) - ps, 0.f);
    if (L.sub == 0) s.coef[L.row] = li > 0.f ? 1.f / static_cast<float>(a.B) : 0.f;
    if (L.sub != 0) li = 0.f;
  }
  for (int o = 32; o >= 1; o >>= 1) li += __shfl_xor(li, o, 64);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = li;
  __syncthreads();
  if (threadIdx.x == 0) s.part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
}

__global__ __launch_bounds__(256) void kg_step_bwd_kernel(KgStepArgs s, float* __restrict__ dent,
                                                          float* __restrict__ drel, int occ) {
  const KgArgs& a = s.k;
  if (blockIdx.x == 0) {  // the step's loss: partial sums in a fixed order
    __shared__ float red[256];
    float v = 0.f;
    for (int i = threadIdx.x; i < s.nparts; i += 256) v += s.part[i];
    red[threadIdx.x] = v;
    __syncthreads();
    for (int w = 128; w >= 1; w >>= 1) {
      if (static_cast<int>(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
      __syncthreads();
    }
    if (threadIdx.x == 0) s.loss[0] = red[0] / static_cast<float>(a.B);
  }
  const RowLane L = row_lane(a.lp, a.B);
  if (!L.ok) return;
  const float c = s.coef[L.row];
  const int64_t hs = a.src[L.row], rs = a.ridx[L.row], ts = a.dst[L.row];
  if (occ && L.sub == 0) {
    // deterministic mode: the row keys of this triple's occurrences; a triple whose margin
    // holds has no gradient, its rows are skipped (key -1) instead of written as zeros
    int64_t* ke = s.key_e + L.row * (2 + a.K);
    const bool live = c != 0.f;
    ke[0] = live ? hs : -1;
    ke[1] = live ? ts : -1;
    for (int k = 0; k < a.K; ++k) ke[2 + k] = live ? a.neg[L.row * a.K + k] : -1;
    s.key_r[L.row] = live ? rs : -1;
  }
  if (c == 0.f) return;  // whole lane group: the margin holds, no gradient
  const float gp = -c, gn = c / static_cast<float>(2 * a.K);
  float h[4], r[4], t[4], n[4], nh, nr, nt, nn;
  float dh[4] = {0.f, 0.f, 0.f, 0.f}, dr[4] = {0.f, 0.f, 0.f, 0.f}, dt[4] = {0.f, 0.f, 0.f, 0.f};
  kg_load_norm(a.ent, hs, L.sub, a.D, a.lp, a.normalize, h, nh);
  kg_load_norm(a.rel, rs, L.sub, a.D, a.lp, a.normalize, r, nr);
  kg_load_norm(a.ent, ts, L.sub, a.D, a.lp, a.normalize, t, nt);
  kg_grad(a.kind, a.lp, gp, h, r, t, dh, dr, dt);
  for (int k = 0; k < a.K; ++k) {
    const int64_t ns = a.neg[L.row * a.K + k];
    kg_load_norm(a.ent, ns, L.sub, a.D, a.lp, a.normalize, n, nn);
    float dn[4] = {0.f, 0.f, 0.f, 0.f};
    kg_grad(a.kind, a.lp, gn, n, r, t, dn, dr, dt);
    kg_grad(a.kind, a.lp, gn, h, r, n, dh, dr, dn);
    // deterministic mode: occurrence rows [h, t, neg_0 .. neg_{K-1}] per triple (summed per
    // entity later in a fixed order), else fp32 atomics into the table gradient
    kg_scatter(dent, occ ? L.row * (2 + a.K) + 2 + k : ns, L.sub, a.D, a.lp, a.normalize, n, nn, dn, occ);
  }
  kg_scatter(dent, occ ? L.row * (2 + a.K) : hs, L.sub, a.D, a.lp, a.normalize, h, nh, dh, occ);
  // relation rows: the power-law relation table makes a few of them hot; with replicas each
  // block adds into its own copy (blockIdx % rep), summed by kg_rep_reduce_kernel
  if (occ)
    kg_scatter(drel, L.row, L.sub, a.D, a.lp, a.normalize, r, nr, dr, true);
  else
    kg_scatter(s.rep ? s.drel_rep + static_cast<int64_t>(blockIdx.x % s.rep) * s.rep_stride : drel, rs, L.sub, a.D,
               a.lp, a.normalize, r, nr, dr);
  kg_scatter(dent, occ ? L.row * (2 + a.K) + 1 : ts, L.sub, a.D, a.lp, a.normalize, t, nt, dt, occ);
}

// self-loop dropout of the R-GCN step: keep_i = [u01(Philox(seed, step, salt * 2^40 + i))
// >= p] (the autograd model's torch.rand(n, 1) >= p, drawn on the device), x0 = x * keep
__global__ __launch_bounds__(256) void drop_rows_kernel(const float* __restrict__ x, int64_t n, int d4, float p,
                                                        uint64_t seed, const int64_t* __restrict__ step, uint64_t salt,
                                                        float* __restrict__ x0, float* __restrict__ keep) {
  const uint64_t ctr = static_cast<uint64_t>(step[0]);
  grid_stride(n * d4, [&](int64_t t) {
    const int64_t i = t / d4;
    const int64_t d = t - i * d4;
    const uint4_t r = Philox::gen(seed, ctr, (salt << 40) | static_cast<uint64_t>(i));
    const float k = u01(r[0]) >= p ? 1.f : 0.f;
    const float4_t v = reinterpret_cast<const float4_t*>(x)[t];
    reinterpret_cast<float4_t*>(x0)[t] = v * k;
    if (d == 0) keep[i] = k;
  });
}

// x = 0 with vector stores on the compute queue (n16: 16-byte items; tail bytes by the
// first thread of the grid)
__global__ __launch_bounds__(256) void zero_kernel(uint4_t* __restrict__ x, int64_t n16, unsigned char* tail,
                                                   int ntail) {
  grid_stride(n16, [&](int64_t i) { x[i] = uint4_t{0u, 0u, 0u, 0u}; });
  if (blockIdx.x == 0 && threadIdx.x < static_cast<unsigned>(ntail)) tail[threadIdx.x] = 0;
}

// unaligned buffers: one byte per item
__global__ __launch_bounds__(256) void zero_bytes_kernel(unsigned char* __restrict__ x, int64_t n) {
  grid_stride(n, [&](int64_t i) { x[i] = 0; });
}

// multi-label sigmoid cross-entropy of logits x [B, C] against label rows labels[rows[b]]
// (the full-flow trainer's loss, F.binary_cross_entropy_with_logits mean) and the F1
// counts of the thresholded predictions: per-block partial loss sums (a second one-block
// launch adds them in order) and tp / fp / fn added into counts
__global__ __launch_bounds__(256) void bce_f1_fwd_kernel(const float* __restrict__ x, const float* __restrict__ labels,
                                                         const int64_t* __restrict__ rows, int64_t B, int C,
                                                         float* __restrict__ part,
                                                         unsigned long long* __restrict__ counts) {
  __shared__ float red[4];
  __shared__ unsigned int cred[4][3];
  float l = 0.f;
  unsigned int tp = 0, fp = 0, fn = 0;
  grid_stride(B * C, [&](int64_t i) {
    const int64_t b = i / C;
    const int c = static_cast<int>(i - b * C);
    const float xv = x[i], y = labels[rows[b] * C + c];
    l += fmaxf(xv, 0.f) - xv * y + log1pf(__expf(-fabsf(xv)));
    const bool pred = xv >= 0.f, pos = y > 0.5f;
    tp += pred && pos;
    fp += pred && !pos;
    fn += !pred && pos;
  });
  for (int o = 32; o >= 1; o >>= 1) {
    l += __shfl_xor(l, o, 64);
    tp += __shfl_xor(tp, o, 64);
    fp += __shfl_xor(fp, o, 64);
    fn += __shfl_xor(fn, o, 64);
  }
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[w] = l;
    cred[w][0] = tp;
    cred[w][1] = fp;
    cred[w][2] = fn;
  }
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = (red[0] + red[1]) + (red[2] + red[3]);
  if (threadIdx.x < 3) {
    const unsigned int v = cred[0][threadIdx.x] + cred[1][threadIdx.x] + cred[2][threadIdx.x] + cred[3][threadIdx.x];
    if (v) atomicAdd(counts + threadIdx.x, static_cast<unsigned long long>(v));
  }
}

__global__ __launch_bounds__(256) void bce_sum_kernel(const float* __restrict__ part, int nparts, float inv_n,
                                                      float* __restrict__ loss) {
  __shared__ float red[256];
  float v = 0.f;
  for (int i = threadIdx.x; i < nparts; i += 256) v += part[i];
  red[threadIdx.x] = v;
  __syncthreads();
  for (int w = 128; w >= 1; w >>= 1) {
    if (static_cast<int>(threadIdx.x) < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) loss[0] = red[0] * inv_n;
}

// d loss / d x = (sigmoid(x) - y) * g / (B C), g = the upstream gradient (device scalar)
__global__ __launch_bounds__(256) void bce_bwd_kernel(const float* __restrict__ x, const float* __restrict__ labels,
                                                      const int64_t* __restrict__ rows, int64_t B, int C,
                                                      const float* __restrict__ g, float inv_n,
                                                      float* __restrict__ dx) {
  const float s = g[0] * inv_n;
  grid_stride(B * C, [&](int64_t i) {
    const int64_t b = i / C;
    const int c = static_cast<int>(i - b * C);
    const float xv = x[i], y = labels[rows[b] * C + c];
    dx[i] = (1.f / (1.f + __expf(-xv)) - y) * s;
  });
}

// fp32 -> bf16, 4 elements per item (n4 = n / 4)
__global__ __launch_bounds__(256) void cast_bf16_kernel(const float* __restrict__ x, int64_t n4,
                                                        bf16_t* __restrict__ out) {
  grid_stride(n4, [&](int64_t i) {
    const float4_t v = reinterpret_cast<const float4_t*>(x)[i];
    tl2u w;
    w[0] = pack_bf16x2(v[0], v[1]);
    w[1] = pack_bf16x2(v[2], v[3]);
    reinterpret_cast<tl2u*>(out)[i] = w;
  });
}

inline int row_lanes(int chunks) {
  int lp = 1;
  while (lp < chunks && lp < 64) lp <<= 1;
  return lp;
}
inline dim3 row_grid(int64_t rows, int lp) {
  const int64_t rpw = 64 / lp;
  const int64_t waves = (rows + rpw - 1) / rpw;
  return dim3(static_cast<uint32_t>((waves + 3) / 4));
}

__global__ __launch_bounds__(256) void gather_f32_bf16_kernel(const float* __restrict__ x, int64_t n_rows, int D,
                                                              const int64_t* __restrict__ idx, int64_t n,
                                                              bf16_t* __restrict__ out) {
  const int D4 = D >> 2;
  grid_stride(n * D4, [&](int64_t t) {
    const int64_t e = t / D4;
    const int d = static_cast<int>(t - e * D4) * 4;
    const int64_t r = idx[e];
    float4_t v = {0.f, 0.f, 0.f, 0.f};
    if (r >= 0 && r < n_rows) v = *reinterpret_cast<const float4_t*>(x + r * D + d);
    tl2u w;
    w[0] = pack_bf16x2(v[0], v[1]);
    w[1] = pack_bf16x2(v[2], v[3]);
    *reinterpret_cast<tl2u*>(out + e * D + d) = w;
  });
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

hipError_t eh_sgns_fwd(const void* emb, const void* pos, const void* neg, int is_bf16, int64_t B, int P, int K, int D,
                       float* logits, float* loss_rows, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const int V = is_bf16 ? 8 : 4;
  if (D % V != 0 || D / V > 64) return hipErrorInvalidValue;
  const int lp = row_lanes(D / V);
  if (is_bf16)
    hipLaunchKernelGGL(sgns_fwd_kernel<bf16_t>, row_grid(B, lp), dim3(256), 0, s, static_cast<const bf16_t*>(emb),
                       static_cast<const bf16_t*>(pos), static_cast<const bf16_t*>(neg), B, P, K, D, lp, logits,
                       loss_rows);
  else
    hipLaunchKernelGGL(sgns_fwd_kernel<float>, row_grid(B, lp), dim3(256), 0, s, static_cast<const float*>(emb),
                       static_cast<const float*>(pos), static_cast<const float*>(neg), B, P, K, D, lp, logits,
                       loss_rows);
  return hipGetLastError();
}

hipError_t eh_sgns_bwd(const void* emb, const void* pos, const void* neg, int is_bf16, int64_t B, int P, int K, int D,
                       const float* logits, float gscale, void* demb, void* dpos, void* dneg, hipStream_t s) {
  if (B == 0) return hipSuccess;
  const int V = is_bf16 ? 8 : 4;
  if (D % V != 0 || D / V > 64) return hipErrorInvalidValue;
  const int lp = row_lanes(D / V);
  if (is_bf16)
    hipLaunchKernelGGL(sgns_bwd_kernel<bf16_t>, row_grid(B, lp), dim3(256), 0, s, static_cast<const bf16_t*>(emb),
                       static_cast<const bf16_t*>(pos), static_cast<const bf16_t*>(neg), B, P, K, D, lp, logits,
                       gscale, static_cast<bf16_t*>(demb), static_cast<bf16_t*>(dpos), static_cast<bf16_t*>(dneg));
  else
    hipLaunchKernelGGL(sgns_bwd_kernel<float>, row_grid(B, lp), dim3(256), 0, s, static_cast<const float*>(emb),
                       static_cast<const float*>(pos), static_cast<const float*>(neg), B, P, K, D, lp, logits, gscale,
                       static_cast<float*>(demb), static_cast<float*>(dpos), static_cast<float*>(dneg));
  return hipGetLastError();
}

static KgArgs kg_args(const float* ent, const float* rel, const int64_t* src, const int64_t* dst, const int64_t* ridx,
                      const int64_t* neg, int64_t B, int K, int D, int kind, int corrupt, int normalize) {
  KgArgs a;
  a.ent = ent;
  a.rel = rel;
  a.src = src;
  a.dst = dst;
  a.ridx = ridx;
  a.neg = neg;
  a.B = B;
  a.K = K;
  a.D = D;
  a.kind = kind;
  a.corrupt = corrupt;
  a.normalize = normalize;
  a.lp = row_lanes((D + 3) / 4);
  return a;
}

hipError_t eh_kg_fwd(const float* ent, const float* rel, const int64_t* src, const int64_t* dst, const int64_t* ridx,
                     const int64_t* neg, int64_t B, int K, int D, int kind, int corrupt, int normalize,
                     float* pos_score, float* neg_score, hipStream_t s) {
  if (B == 0) return hipSuccess;
  if (D % 4 != 0 || D > 256 || kind < 0 || kind > 2 || corrupt < 0 || corrupt > 2) return hipErrorInvalidValue;
  const KgArgs a = kg_args(ent, rel, src, dst, ridx, neg, B, K, D, kind, corrupt, normalize);
  hipLaunchKernelGGL(kg_fwd_kernel, row_grid(B, a.lp), dim3(256), 0, s, a, pos_score, neg_score);
  return hipGetLastError();
}

hipError_t eh_kg_bwd(const float* ent, const float* rel, const int64_t* src, const int64_t* dst, const int64_t* ridx,
                     const int64_t* neg, int64_t B, int K, int D, int kind, int corrupt, int normalize,
                     const float* gpos, const float* gneg, float* dent, float* drel, int occ, hipStream_t s) {
  if (B == 0) return hipSuccess;
  if (D % 4 != 0 || D > 256 || kind < 0 || kind > 2 || corrupt < 0 || corrupt > 2) return hipErrorInvalidValue;
  const KgArgs a = kg_args(ent, rel, src, dst, ridx, neg, B, K, D, kind, corrupt, normalize);
  hipLaunchKernelGGL(kg_bwd_kernel, row_grid(B, a.lp), dim3(256), 0, s, a, gpos, gneg, dent, drel, occ);
  return hipGetLastError();
}

hipError_t eh_sgns_fwd_idx(const void* T, const int64_t* tmap, int64_t nTm, const int64_t* tinv, int64_t nT,
                           const void* C, const int64_t* cmap, int64_t nCm, const int64_t* cinv, int64_t nC,
                           int64_t P, int K, int D,
                           float gscale, float* coef, float* loss_rows, int rows_bf16, hipStream_t s) {
  if (P == 0) return hipSuccess;
  if (D % 4 != 0 || D / 4 > 64 || K < 0) return hipErrorInvalidValue;
  const int lp = row_lanes(D / 4);
  hipLaunchKernelGGL(sgns_fwd_idx_kernel, row_grid(P, lp), dim3(256), 0, s, T, tmap, nTm, tinv, nT, C, rows_bf16, cmap,
                     nCm, cinv, nC,
                     P, K,
                     D, lp, gscale, coef, loss_rows);
  return hipGetLastError();
}

// ptr[1 + u] = inclusive prefix sum of the occurrence counts (counts of one launch < 2^31).
// `temp` null: *temp_bytes receives the scan's scratch size and nothing runs.
hipError_t eh_occ_count_scan(const int64_t* inv, int64_t n, int64_t n_u, int* cnt, int64_t* ptr, void* temp,
                             size_t* temp_bytes, hipStream_t s) {
  if (n_u <= 0) return hipErrorInvalidValue;
  if (!temp) return hipcub::DeviceScan::InclusiveSum(nullptr, *temp_bytes, cnt, ptr + 1, static_cast<int>(n_u), s);
  hipLaunchKernelGGL(occ_count_kernel, dim3(static_cast<uint32_t>(ceil_div(n > 0 ? n : 1, 256))), dim3(256), 0, s,
                     inv, n, cnt, ptr);
  const hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  return hipcub::DeviceScan::InclusiveSum(temp, *temp_bytes, cnt, ptr + 1, static_cast<int>(n_u), s);
}

// ptr [S + 1] and perm [n] int32 (the first ptr[S] entries used) of the keys >= 0.
// work: 4 n int32 (32-bit keys, ids, sorted keys) + S int32 counts, zeroed by the caller
// where noted; temp: hipcub scratch for the larger of the scan and the sort (null: size
// query into *temp_bytes)
hipError_t eh_det_occ(const int64_t* keys, int64_t n, int64_t S, int* cnt, int64_t* ptr, int* work, int* perm,
                      void* temp, size_t* temp_bytes, hipStream_t s) {
  if (S <= 0 || S >= (int64_t{1} << 30) || n >= (int64_t{1} << 31)) return hipErrorInvalidValue;
  int bits = 1;
  while ((int64_t{1} << bits) <= S) ++bits;  // keys 0 .. S (S = skipped)
  if (!temp) {
    size_t a = 0, b = 0;
    EULER_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(nullptr, a, cnt, ptr + 1, static_cast<int>(S), s));
    EULER_HIP_CHECK(hipcub::DeviceRadixSort::SortPairs(nullptr, b, work, work, work, perm, static_cast<int>(n), 0,
                                                       bits, s));
    *temp_bytes = a > b ? a : b;
    return hipSuccess;
  }
  const dim3 g(static_cast<uint32_t>(ceil_div(n > 0 ? n : 1, 256)));
  hipLaunchKernelGGL(det_count_kernel, g, dim3(256), 0, s, keys, n, S, cnt, ptr);
  EULER_HIP_CHECK(hipGetLastError());
  EULER_HIP_CHECK(hipcub::DeviceScan::InclusiveSum(temp, *temp_bytes, cnt, ptr + 1, static_cast<int>(S), s));
  if (n == 0) return hipSuccess;
  int* k32 = work;
  int* iota = work + n;
  int* ksorted = work + 2 * n;
  hipLaunchKernelGGL(det_prep_kernel, g, dim3(256), 0, s, keys, n, S, k32, iota);
  EULER_HIP_CHECK(hipGetLastError());
  return hipcub::DeviceRadixSort::SortPairs(temp, *temp_bytes, k32, ksorted, iota, perm, static_cast<int>(n), 0, bits,
                                            s);
}

hipError_t eh_det_segsum(const float* src, int D, const int64_t* ptr, const int* perm, int64_t S, float* out,
                         hipStream_t s) {
  if (S <= 0) return hipSuccess;
  const int LP = D / 4;
  if (D % 4 != 0 || LP > 64 || LP < 1 || (LP & (LP - 1)) != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(det_segsum_kernel, dim3(static_cast<uint32_t>(S < 16384 ? S : 16384)), dim3(256), 0, s, src, D,
                     ptr, perm, S, out);
  return hipGetLastError();
}

hipError_t eh_occ_fill(const int64_t* inv, int64_t n, const int64_t* ptr, int* cursor, int* list, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(occ_fill_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, inv, n, ptr,
                     cursor, list);
  return hipGetLastError();
}

hipError_t eh_sgns_update(int side, int64_t n_u, const int64_t* ptr, const int* list, const float* coef, int64_t P,
                          int K, int D, const void* src, int src_bf16, int64_t n_src, const int64_t* smap,
                          int64_t n_smap, const int64_t* sinv, void* gout, int gout_bf16, float* table, float* m,
                          float* v, const int64_t* rows, int64_t n_rows, int64_t* step, int inc_step, float lr,
                          float b1, float b2, float eps, int kind, hipStream_t s) {
  if (D % 4 != 0 || D / 4 > 64 || (side != 0 && side != 1) || (side == 1 && K < 0) || kind < 0 || kind > 2)
    return hipErrorInvalidValue;
  if (!gout && inc_step) hipLaunchKernelGGL(sgns_step_inc_kernel, dim3(1), dim3(1), 0, s, step);
  if (n_u == 0) return hipGetLastError();
  SgnsUpd a;
  a.ptr = ptr;
  a.list = list;
  a.coef = coef;
  a.src = src;
  a.smap = smap;
  a.sinv = sinv;
  a.gout = gout;
  a.table = table;
  a.m = m;
  a.v = v;
  a.rows = rows;
  a.step = step;
  a.n_u = n_u;
  a.P = P;
  a.n_rows = n_rows;
  a.n_src = n_src;
  a.n_smap = n_smap;
  a.K = K;
  a.D = D;
  a.lp = row_lanes(D / 4);
  // widen the row groups (up to a block) while the widened groups still fit the chip's
  // resident lanes (256 CUs x 2048)
  constexpr int64_t kFillLanes = int64_t{1} << 19;
  a.split = 1;
  while (a.lp * a.split < 256 && n_u * a.lp * a.split * 2 <= kFillLanes) a.split <<= 1;
  a.lsh = 0;
  while ((1 << a.lsh) < a.lp * a.split) ++a.lsh;
  a.side = side;
  a.kind = kind;
  a.lr = lr;
  a.b1 = b1;
  a.b2 = b2;
  a.eps = eps;
  a.src_bf16 = src_bf16;
  a.gout_bf16 = gout_bf16;
  const int64_t lanes = n_u * a.lp * a.split;
  const dim3 grid(static_cast<uint32_t>((lanes + 255) / 256));
  if (a.lp * a.split > 64)
    hipLaunchKernelGGL(sgns_update_kernel<true>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(sgns_update_kernel<false>, grid, dim3(256), 0, s, a);
  return hipGetLastError();
}

// rows idx of an fp32 table as bf16 (idx < 0: a zero row): the sharded-table exchange
// packs its send buffer in the wire dtype in the gather itself
hipError_t eh_gather_f32_bf16(const float* x, int64_t n_rows, int D, const int64_t* idx, int64_t n, void* out,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (D % 4 != 0) return hipErrorInvalidValue;
  const int64_t tot = n * (D / 4);
  hipLaunchKernelGGL(gather_f32_bf16_kernel, grid_for(tot), dim3(256), 0, s, x,
                     n_rows, D, idx, n, static_cast<bf16_t*>(out));
  return hipGetLastError();
}


// the fused TransE margin step (KgStepArgs): returns the fwd launch's block count through
// nparts_out so the caller can size `part`; part == null: only report it
hipError_t eh_kg_step(const float* ent, const float* rel, const int64_t* pool, int64_t P, const int64_t* t_src,
                      const int64_t* t_dst, const int64_t* t_rel, int64_t num_ent, const int64_t* step, uint64_t seed,
                      int64_t B, int K, int D, int kind, int normalize, float margin, int64_t* o_src, int64_t* o_dst,
                      int64_t* o_ridx, int64_t* o_neg, float* coef, float* part, float* loss, float* dent,
                      float* drel, int* nparts_out, float* drel_rep, int rep, int64_t num_rel, hipStream_t s,
                      float* occ_e, float* occ_r, int64_t* key_e, int64_t* key_r) {
  if (B <= 0 || K <= 0 || K > 255 || P <= 0 || num_ent <= 0 || rep < 0) return hipErrorInvalidValue;
  if (D % 4 != 0 || D > 256 || kind < 0 || kind > 2) return hipErrorInvalidValue;
  KgStepArgs a;
  a.k = kg_args(ent, rel, o_src, o_dst, o_ridx, o_neg, B, K, D, kind, 2, normalize);
  const dim3 grid = row_grid(B, a.k.lp);
  if (nparts_out) *nparts_out = static_cast<int>(grid.x);
  if (!part) return hipSuccess;
  a.o_src = o_src;
  a.o_dst = o_dst;
  a.o_ridx = o_ridx;
  a.o_neg = o_neg;
  a.pool = pool;
  a.t_src = t_src;
  a.t_dst = t_dst;
  a.t_rel = t_rel;
  a.P = P;
  a.num_ent = num_ent;
  a.step = step;
  a.seed = seed;
  a.margin = margin;
  a.coef = coef;
  a.part = part;
  a.loss = loss;
  a.nparts = static_cast<int>(grid.x);
  const bool occ = occ_e != nullptr;
  if (occ && (!occ_r || !key_e || !key_r)) return hipErrorInvalidValue;
  a.key_e = key_e;
  a.key_r = key_r;
  a.rep = drel_rep && !occ ? rep : 0;
  a.drel_rep = drel_rep;
  a.rep_stride = num_rel * D;
  if (a.rep) EULER_HIP_CHECK(eh_zero(drel_rep, a.rep * a.rep_stride * 4, s));
  hipLaunchKernelGGL(kg_step_fwd_kernel, grid, dim3(256), 0, s, a);
  hipLaunchKernelGGL(kg_step_bwd_kernel, grid, dim3(256), 0, s, a, occ ? occ_e : dent, occ ? occ_r : drel,
                     occ ? 1 : 0);
  if (a.rep)
    hipLaunchKernelGGL(kg_rep_reduce_kernel, grid_for(a.rep_stride), dim3(256), 0, s, drel_rep, a.rep, a.rep_stride,
                       drel);
  return hipGetLastError();
}

hipError_t eh_drop_rows(const float* x, int64_t n, int d, float p, uint64_t seed, const int64_t* step, uint64_t salt,
                        float* x0, float* keep, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (d % 4 != 0 || salt >= (1ull << 24)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(drop_rows_kernel, grid_for(n * (d / 4)), dim3(256), 0, s, x, n, d / 4, p, seed, step, salt, x0,
                     keep);
  return hipGetLastError();
}

hipError_t eh_zero(void* x, int64_t bytes, hipStream_t s) {
  if (bytes <= 0) return hipSuccess;
  if (reinterpret_cast<uintptr_t>(x) % 16 != 0) {
    hipLaunchKernelGGL(zero_bytes_kernel, grid_for(bytes), dim3(256), 0, s, static_cast<unsigned char*>(x), bytes);
    return hipGetLastError();
  }
  const int64_t n16 = bytes / 16;
  const int ntail = static_cast<int>(bytes - n16 * 16);
  hipLaunchKernelGGL(zero_kernel, grid_for(n16 > 0 ? n16 : 1), dim3(256), 0, s, static_cast<uint4_t*>(x), n16,
                     static_cast<unsigned char*>(x) + n16 * 16, ntail);
  return hipGetLastError();
}

int eh_bce_parts(int64_t n) {
  const int64_t b = ceil_div(n, 256);
  return static_cast<int>(b < 1024 ? (b > 0 ? b : 1) : 1024);
}

hipError_t eh_bce_f1_fwd(const float* x, const float* labels, const int64_t* rows, int64_t B, int C, float* part,
                         float* loss, int64_t* counts, hipStream_t s) {
  if (B <= 0 || C <= 0) return hipErrorInvalidValue;
  const int np = eh_bce_parts(B * C);
  hipLaunchKernelGGL(bce_f1_fwd_kernel, dim3(np), dim3(256), 0, s, x, labels, rows, B, C, part,
                     reinterpret_cast<unsigned long long*>(counts));
  hipLaunchKernelGGL(bce_sum_kernel, dim3(1), dim3(256), 0, s, part, np, 1.f / static_cast<float>(B * C), loss);
  return hipGetLastError();
}

hipError_t eh_bce_bwd(const float* x, const float* labels, const int64_t* rows, int64_t B, int C, const float* g,
                      float* dx, hipStream_t s) {
  if (B <= 0 || C <= 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(bce_bwd_kernel, grid_for(B * C), dim3(256), 0, s, x, labels, rows, B, C, g,
                     1.f / static_cast<float>(B * C), dx);
  return hipGetLastError();
}

hipError_t eh_cast_bf16(const float* x, int64_t n, void* out, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n % 4 != 0) return hipErrorInvalidValue;
  hipLaunchKernelGGL(cast_bf16_kernel, grid_for(n / 4), dim3(256), 0, s, x, n / 4, static_cast<bf16_t*>(out));
  return hipGetLastError();
}
}  // extern "C"
