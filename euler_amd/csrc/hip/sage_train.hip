// One fused GraphSAGE training step on gfx950 (the bench.py flagship; SURVEY §2.7
// K1/K2/K3/K11/K12, §7.3).
//
// Model (reference examples/graphsage/graphsage.py:56-67 + mp_utils/base.py:24-47):
//   h0   = relu([x[level1] | mean_k x[nb2]] @ W0^T)          level-1 rows  [M1, H]
//   h1   = relu([h0[self] | mean_k h0[nb1]] @ W1^T)          roots         [B,  H]
//   emb  = h1 @ Wfc^T + bfc ;  logits = emb @ Wout^T          [B, C]
//   loss = mean(sigmoid_ce(logits, onehot(label)))
//
// Instead of autograd over ~60 small library launches, a step is ten kernels:
//   roots -> hop1 -> hop2 (sampling) -> fwd L0 -> fwd L1 -> head (fc, out, loss and the
//   whole head backward down to dA1 = g1 @ W1) -> route (dA1 -> relu mask -> g0) ->
//   grouped split-K dW for all four weights -> split-K reduce -> Adam (+ bf16 weight
//   shadows for the next step's MFMAs).
//
// Operands of every weight-gradient GEMM are emitted by their producer kernels in the
// "kt" (k-tiled) layout X_kt[M/32][N][32]: the reduction index m is contiguous, so
// both MFMA fragments of dW = G^T X are single 16-byte loads
// (lane l: 8 consecutive m at column l&15), no LDS transpose in the dW kernel.
#include "hip/common.h"
#include "hip/launchers.h"

namespace euler_hip {

typedef __bf16 st_bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t st_uint2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float4_t st_mfma(uint4_t a, uint4_t b, float4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(st_bf16x8, a), __builtin_bit_cast(st_bf16x8, b),
                                                 c, 0, 0, 0);
}

// offset of element (m, n) of an [M][N] matrix stored k-tiled ([M/32][N][32])
__device__ __forceinline__ int64_t kt_off(int64_t m, int64_t n, int64_t N) {
  return ((m >> 5) * N + n) * 32 + (m & 31);
}

// "fm" (fragment-major) layout of the bf16 weight shadows W[N][K] used as MFMA B operands:
// Wf[N/16][K/32][64 lanes][8].  The B fragment of (16-column slab, 32-deep k-step) is one
// contiguous 1 KB (lane l: W[n0 + (l&15)][k0 + 8*(l>>4) .. +8]), so each wave load is
// fully coalesced instead of 16 rows x 64 B (which the texture path serves at a quarter
// of the rate and made the head kernel load-issue bound).
__device__ __forceinline__ int64_t fm_off(int64_t n, int64_t k, int64_t K) {
  return (((n >> 4) * (K >> 5) + (k >> 5)) * 64 + ((k & 31) >> 3) * 16 + (n & 15)) * 8 + (k & 7);
}
// the B fragment of slab n0 (multiple of 16), k-step k0 (multiple of 32) for this lane
__device__ __forceinline__ uint4_t fm_frag(const bf16_t* __restrict__ Wf, int n0, int k0, int K, int lane) {
  return *reinterpret_cast<const uint4_t*>(
      Wf + ((static_cast<int64_t>(n0 >> 4) * (K >> 5) + (k0 >> 5)) * 64 + lane) * 8);
}

__device__ __forceinline__ bool bf_pos(bf16_t v) { return (v & 0x8000u) == 0 && (v & 0x7fffu) != 0; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ----------------------------------------------------------------------------
// 1. roots: alias-sample B rows, write them to roots and the tail of level1, gather
//    their labels, and bump the Adam step (read later in this step by the optimizer).
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void st_roots_kernel(const float* __restrict__ prob,
                                                       const int32_t* __restrict__ alias, int64_t pop, int B,
                                                       const int64_t* __restrict__ rng, uint64_t stream_id,
                                                       const int16_t* __restrict__ labels,
                                                       int32_t* __restrict__ roots, int32_t* __restrict__ level1_tail,
                                                       int32_t* __restrict__ label_idx, int64_t* __restrict__ step) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i == 0) step[0] += 1;
  if (i >= B) return;
  const uint4_t r = Philox::gen(static_cast<uint64_t>(rng[0]), (static_cast<uint64_t>(rng[1]) << 8) ^ stream_id,
                                static_cast<uint64_t>(i));
  const uint64_t x = (static_cast<uint64_t>(r[0]) << 32) | r[1];
  int64_t k = static_cast<int64_t>(__umul64hi(x, static_cast<uint64_t>(pop)));
  if (k >= pop) k = pop - 1;
  const int32_t pick = (u01(r[2]) < prob[k]) ? static_cast<int32_t>(k) : alias[k];
  roots[i] = pick;
  level1_tail[i] = pick;
  label_idx[i] = labels[pick];
}

// ----------------------------------------------------------------------------
// 2. fused gather + mean + MFMA linear + ReLU for fixed-fanout tiles, BM rows / block.
//    Emits out (row-major bf16, LDS-staged 16-byte stores) and the A tile in kt layout.
// ----------------------------------------------------------------------------
template <int BM, int BN>
__global__ __launch_bounds__(256, BM <= 32 ? 4 : 2) void st_sage_fwd_kernel(
    const bf16_t* __restrict__ x, int D, const int32_t* __restrict__ self_idx, const int32_t* __restrict__ nbr_idx,
    int F, int include_self, float inv_cnt, const bf16_t* __restrict__ W, int H, int64_t M,
    bf16_t* __restrict__ out, bf16_t* __restrict__ a_kt, uint32_t* __restrict__ relu_mask) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int K2 = 2 * D;
  const int ldsw = K2 + 8;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t row0 = static_cast<int64_t>(tile) * BM;
  const int cpr = D >> 3;
  // phase 1: gather. item = (row r, 8-column chunk c); all fanout loads of a chunk in flight
  for (int it = threadIdx.x; it < BM * cpr; it += 256) {
    const int r = it / cpr;
    const int c = it - r * cpr;
    const int64_t grow = row0 + r;
    uint4_t sv = {0u, 0u, 0u, 0u};
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    if (grow < M) {
      const int64_t s = self_idx[grow];
      if (s >= 0) sv = *reinterpret_cast<const uint4_t*>(x + s * D + c * 8);
      if (include_self) acc_bf16x8(acc, sv);
      // nbr_idx == nullptr: tree layout, the neighbours of row m are rows m*F .. m*F+F-1
      // (no index loads, the addresses are known up front)
      const bool contig = nbr_idx == nullptr;
      const int32_t* nb = contig ? nullptr : nbr_idx + grow * F;
      constexpr int G = 12;  // neighbour rows in flight per item (fits 4 waves/SIMD)
      for (int k = 0; k < F; k += G) {
        int32_t j[G];
        uint4_t v[G];
#pragma unroll
        for (int u = 0; u < G; ++u)
          j[u] = (k + u < F) ? (contig ? static_cast<int32_t>(grow * F + k + u) : nb[k + u]) : -1;
#pragma unroll
        for (int u = 0; u < G; ++u)
          v[u] = j[u] >= 0 ? *reinterpret_cast<const uint4_t*>(x + static_cast<int64_t>(j[u]) * D + c * 8)
                           : uint4_t{0u, 0u, 0u, 0u};
#pragma unroll
        for (int u = 0; u < G; ++u) acc_bf16x8(acc, v[u]);
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] *= inv_cnt;
    *reinterpret_cast<uint4_t*>(lds + r * ldsw + c * 8) = sv;
    *reinterpret_cast<uint4_t*>(lds + r * ldsw + D + c * 8) = pack_bf16x8(acc);
  }
  __syncthreads();
  // A tile -> kt layout: item = (column n, 8-row chunk q); 4 lanes cover one 32-row column segment
  if (a_kt) {
    constexpr int CH = BM / 8;
    for (int it = threadIdx.x; it < K2 * CH; it += 256) {
      const int q = it % CH;
      const int n = it / CH;
      const int64_t g = row0 + q * 8;
      if (g >= M) continue;
      float v[8];
#pragma unroll
      for (int i = 0; i < 8; ++i) v[i] = bf2f(lds[(q * 8 + i) * ldsw + n]);
      *reinterpret_cast<uint4_t*>(a_kt + kt_off(g, n, K2)) = pack_bf16x8(v);
    }
  }
  // phase 2: MFMA GEMM out of LDS; each wave owns a 64-column slab of a BN chunk
  constexpr int WN = BN / 64;
  constexpr int WM = 4 / WN;
  constexpr int RW = BM / WM;
  constexpr int FM = RW / 16;
  constexpr int FN = 4;
  static_assert(RW % 16 == 0, "rows per wave must be a multiple of 16");
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  // [BM][BN + 8] output staging tile: aliases the (then dead) A tile when one column chunk
  // covers H, which halves the LDS footprint and doubles the resident blocks per CU
  const bool alias_out = H <= BN && BN <= K2;
  bf16_t* otile = alias_out ? lds : lds + BM * ldsw;
  const int ldo = BN + 8;
  for (int cchunk = 0; cchunk < H; cchunk += BN) {
    const int cb = cchunk + wn * 64;
    float4_t acc[FM][FN];
#pragma unroll
    for (int m = 0; m < FM; ++m)
#pragma unroll
      for (int n = 0; n < FN; ++n) acc[m][n] = float4_t{0.f, 0.f, 0.f, 0.f};
    if (cb < H) {
      uint4_t bcur[FN];
#pragma unroll
      for (int n = 0; n < FN; ++n) bcur[n] = fm_frag(W, cb + n * 16, 0, K2, lane);
      for (int k0 = 0; k0 < K2; k0 += 32) {
        uint4_t bnext[FN];
        const bool more = k0 + 32 < K2;
#pragma unroll
        for (int n = 0; n < FN; ++n)
          bnext[n] = more ? fm_frag(W, cb + n * 16, k0 + 32, K2, lane) : uint4_t{0u, 0u, 0u, 0u};
        uint4_t a[FM];
#pragma unroll
        for (int m = 0; m < FM; ++m)
          a[m] = *reinterpret_cast<const uint4_t*>(lds + (wm * RW + m * 16 + lr) * ldsw + k0 + lk);
#pragma unroll
        for (int m = 0; m < FM; ++m)
#pragma unroll
          for (int n = 0; n < FN; ++n) acc[m][n] = st_mfma(a[m], bcur[n], acc[m][n]);
#pragma unroll
        for (int n = 0; n < FN; ++n) bcur[n] = bnext[n];
      }
    }
    if (alias_out) __syncthreads();  // every wave is done reading the A tile
    if (cb < H) {
      // ReLU + bf16 into the staging tile (C map: col = lane&15, row = (lane>>4)*4 + j)
#pragma unroll
      for (int m = 0; m < FM; ++m)
#pragma unroll
        for (int n = 0; n < FN; ++n)
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = wm * RW + m * 16 + (lane >> 4) * 4 + j;
            otile[row * ldo + wn * 64 + n * 16 + lr] = f2bf(fmaxf(acc[m][n][j], 0.f));
          }
    }
    __syncthreads();
    // coalesced 16-byte stores of the chunk
    const int ncols = (H - cchunk) < BN ? (H - cchunk) : BN;
    const int cpc = ncols >> 3;
    for (int it = threadIdx.x; it < BM * cpc; it += 256) {
      const int r = it / cpc, c = it - r * cpc;
      const int64_t grow = row0 + r;
      if (grow < M)
        *reinterpret_cast<uint4_t*>(out + grow * H + cchunk + c * 8) =
            *reinterpret_cast<const uint4_t*>(otile + r * ldo + c * 8);
    }
    // ReLU mask bits for the backward: word (k-block, column) has bit i set iff row
    // 32*kb + i is positive (0.85 MB instead of re-reading the 13.6 MB activation)
    if (relu_mask) {
      constexpr int KBB = BM / 32;
      for (int it = threadIdx.x; it < KBB * ncols; it += 256) {
        const int kbl = it / ncols, n = it - kbl * ncols;
        const int64_t g = row0 + kbl * 32;
        if (g >= M) continue;
        uint32_t bits = 0;
#pragma unroll
        for (int i = 0; i < 32; ++i) bits |= (bf_pos(otile[(kbl * 32 + i) * ldo + n]) ? 1u : 0u) << i;
        relu_mask[(g >> 5) * H + cchunk + n] = bits;
      }
    }
    __syncthreads();
  }
}

// ----------------------------------------------------------------------------
// 3. head: fc + out_fc + sigmoid-CE + backward down to dA1 = g1 @ W1, 32 rows / block.
// ----------------------------------------------------------------------------
// acc[FM][FN] += A_lds[row0 + m*16 + r][k] * Bg[col0 + n*16 + r][k]  (Bg row-major [N][K])
constexpr int ST_KC = 8;  // k-steps (x32) per B chunk of the head GEMMs

// issue the first B chunk of a head GEMM (slab col0 of fm weight Bf[N][K]) ahead of time
__device__ __forceinline__ void st_prefetch(const bf16_t* __restrict__ Bf, int col0, int N, int K, int lane,
                                            uint4_t (&b)[ST_KC]) {
  // branch-free (clamped addresses; out-of-range fragments are loaded but never used) so
  // all ST_KC loads stay in flight together
  const int c = col0 < N ? col0 : 0;
#pragma unroll
  for (int s = 0; s < ST_KC; ++s) b[s] = fm_frag(Bf, c, s * 32 < K ? s * 32 : 0, K, lane);
}

template <int FM>
__device__ __forceinline__ void st_mfma_chunk(const bf16_t* A, int lda, int kc, int K, const uint4_t (&b)[ST_KC],
                                              float4_t (&acc)[FM][1], int lane) {
  const int lr = lane & 15, lk = (lane >> 4) * 8;
#pragma unroll
  for (int s = 0; s < ST_KC; ++s) {
    if (kc + s * 32 < K) {  // uniform guard, no early exit: keeps the chunk's loads batched
      uint4_t a[FM];
#pragma unroll
      for (int m = 0; m < FM; ++m)
        a[m] = *reinterpret_cast<const uint4_t*>(A + (m * 16 + lr) * lda + kc + s * 32 + lk);
#pragma unroll
      for (int m = 0; m < FM; ++m) acc[m][0] = st_mfma(a[m], b[s], acc[m][0]);
    }
  }
}

template <int FM>
__device__ __forceinline__ void st_gemm_lds_glb(const bf16_t* A, int lda, const bf16_t* __restrict__ Bf, int col0,
                                                int K, float4_t (&acc)[FM][1], int lane, const uint4_t (&pre)[ST_KC]) {
  // B = fm-layout weight shadow [N][K]; its first 256-deep chunk was issued by
  // st_prefetch before the preceding barrier (weights do not depend on the previous
  // phase), later chunks issue all their loads before the first MFMA.  The head runs one
  // block per CU, so it is latency-bound: this leaves ~one exposed L2 latency per phase.
  st_mfma_chunk<FM>(A, lda, 0, K, pre, acc, lane);
  for (int kc = 32 * ST_KC; kc < K; kc += 32 * ST_KC) {
    uint4_t b[ST_KC];
#pragma unroll
    for (int s = 0; s < ST_KC; ++s) b[s] = fm_frag(Bf, col0, kc + s * 32 < K ? kc + s * 32 : 0, K, lane);
    st_mfma_chunk<FM>(A, lda, kc, K, b, acc, lane);
  }
}

template <int FM, int FN>
__device__ __forceinline__ void st_zero(float4_t (&acc)[FM][FN]) {
#pragma unroll
  for (int m = 0; m < FM; ++m)
#pragma unroll
    for (int n = 0; n < FN; ++n) acc[m][n] = float4_t{0.f, 0.f, 0.f, 0.f};
}

// store 4 consecutive rows (j = 0..3) of one column to a kt matrix: one 8-byte store
__device__ __forceinline__ void st_kt4(bf16_t* kt, int64_t row, int col, int N, float a, float b, float c,
                                       float d) {
  st_uint2 v;
  v[0] = pack_bf16x2(a, b);
  v[1] = pack_bf16x2(c, d);
  *reinterpret_cast<st_uint2*>(kt + kt_off(row, col, N)) = v;
}

constexpr int HB = kStHeadRows;  // head rows per block: the head is a chain of six dependent GEMM
                         // phases, so twice the blocks (16 rows each, 64 at batch 1024) halve
                         // each phase's per-block work; measured 0.1221 -> 0.1174 ms/step vs 32
                         // rows although every block streams all head weights from L2
constexpr int HFM = HB / 16;
constexpr int HNW = 16;  // head waves per block (1024 threads): short per-wave instruction chains

// inner hop of the tree layout, without the GEMM: A1[t] = [h0[nb_rows + t] | mean_k h0[t*F1 + k]]
// (row-major bf16 [B][2H]).  Thread = (root t, 8-column chunk): all of a root's
// neighbour rows are one contiguous block of h0, so every load address is known up front.
__global__ __launch_bounds__(256) void st_tree_mean_kernel(const bf16_t* __restrict__ h0, int H, int64_t B,
                                                           int F1, int include_self, float inv_cnt,
                                                           bf16_t* __restrict__ A1) {
  const int64_t it = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const int cpr = (2 * H) >> 3;
  if (it >= B * cpr) return;
  const int64_t t = it / cpr;
  const int c = static_cast<int>(it - t * cpr);
  const int64_t nb_rows = B * F1;
  uint4_t out;
  if (c * 8 < H) {
    out = *reinterpret_cast<const uint4_t*>(h0 + (nb_rows + t) * H + c * 8);
  } else {
    const int cc = c * 8 - H;
    float acc[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] = 0.f;
    if (include_self) acc_bf16x8(acc, *reinterpret_cast<const uint4_t*>(h0 + (nb_rows + t) * H + cc));
    constexpr int G = 16;
    for (int k = 0; k < F1; k += G) {
      uint4_t v[G];
#pragma unroll
      for (int u = 0; u < G; ++u)
        v[u] = (k + u < F1) ? *reinterpret_cast<const uint4_t*>(h0 + (t * F1 + k + u) * H + cc)
                            : uint4_t{0u, 0u, 0u, 0u};
#pragma unroll
      for (int u = 0; u < G; ++u) acc_bf16x8(acc, v[u]);
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] *= inv_cnt;
    out = pack_bf16x8(acc);
  }
  *reinterpret_cast<uint4_t*>(A1 + t * 2 * H + c * 8) = out;
}

// LDS tile rows -> kt layout (16 rows = two 8-row chunks per column)
__device__ __forceinline__ void st_lds_to_kt(const bf16_t* tile, int ld, int N, int64_t r0, bf16_t* kt) {
  for (int it = threadIdx.x; it < N * (HB / 8); it += HNW * 64) {
    const int q = it % (HB / 8), n = it / (HB / 8);
    float v[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) v[i] = bf2f(tile[(q * 8 + i) * ld + n]);
    *reinterpret_cast<uint4_t*>(kt + kt_off(r0 + q * 8, n, N)) = pack_bf16x8(v);
  }
}

// head: h1 = relu(A1 W1^T) ; emb = h1 Wfc^T + bfc ; logits = emb Wout^T ; sigmoid-CE ;
// backward through out_fc, fc and the L1 ReLU down to dA1 = g1 W1.  HB rows per block,
// 16 waves; wave w owns 16-column slabs w, w + 16, ... of every product.
__global__ __launch_bounds__(HNW * 64) void st_head_kernel(
    const bf16_t* __restrict__ A1g, int H, int C, const bf16_t* __restrict__ W1b, const bf16_t* __restrict__ Wfc,
    const bf16_t* __restrict__ WfcT, const float* __restrict__ bfc, const bf16_t* __restrict__ Wout,
    const bf16_t* __restrict__ WoutT, const bf16_t* __restrict__ W1T, const int32_t* __restrict__ label_idx,
    float inv_scale, bf16_t* __restrict__ A1_kt, bf16_t* __restrict__ h1_kt, bf16_t* __restrict__ emb_kt,
    bf16_t* __restrict__ dlog_kt, bf16_t* __restrict__ demb_kt, bf16_t* __restrict__ g1_kt, float* __restrict__ dA1,
    float* __restrict__ dbfc, float* __restrict__ loss_acc, long long* __restrict__ prof) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  // optional phase timestamps (100 MHz wall clock) of every block: prof[block][8]
#define ST_STAMP(k) \
  if (prof && threadIdx.x == 0) prof[blockIdx.x * 8 + (k)] = static_cast<long long>(wall_clock64())
  ST_STAMP(0);
  const int H2 = 2 * H;
  const int lda = H2 + 8, ldh = H + 8, ldc = C + 8;
  bf16_t* Aa = lds;              // [HB][2H+8] A1 tile
  bf16_t* Ah = Aa + HB * lda;    // [HB][H+8]  h1
  bf16_t* Eb = Ah + HB * ldh;    // [HB][H+8]  emb, later g1
  bf16_t* Db = Eb + HB * ldh;    // [HB][H+8]  demb
  bf16_t* Dl = Db + HB * ldh;    // [HB][C+8]  dlogits
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * HB;
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lr = lane & 15, lg = lane >> 4;
  constexpr int NT = HNW * 64;

  // the block's labels, staged in LDS up front (used in S3's epilogue)
  __shared__ int lab_s[HB];
  if (threadIdx.x < HB) lab_s[threadIdx.x] = label_idx[r0 + threadIdx.x];

  // S0: A1 tile -> LDS (+ A1_kt); h1 = relu(A1 @ W1^T) -> Ah
  uint4_t pre[ST_KC];
  st_prefetch(W1b, wave * 16, H, H2, lane, pre);
  const int cpa = H2 >> 3;
  for (int it = threadIdx.x; it < HB * cpa; it += NT) {
    const int r = it / cpa, c = it - r * cpa;
    *reinterpret_cast<uint4_t*>(Aa + r * lda + c * 8) = *reinterpret_cast<const uint4_t*>(A1g + (r0 + r) * H2 + c * 8);
  }
  __syncthreads();
  ST_STAMP(1);
  st_lds_to_kt(Aa, lda, H2, r0, A1_kt);
  for (int cc = wave * 16; cc < H; cc += HNW * 16) {
    float4_t acc[HFM][1];
    st_zero(acc);
    st_gemm_lds_glb<HFM>(Aa, lda, W1b, cc, H2, acc, lane, pre);
    if (cc + HNW * 16 < H) st_prefetch(W1b, cc + HNW * 16, H, H2, lane, pre);
#pragma unroll
    for (int m = 0; m < HFM; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) Ah[(m * 16 + lg * 4 + j) * ldh + cc + lr] = f2bf(fmaxf(acc[m][0][j], 0.f));
  }
  st_prefetch(Wfc, wave * 16, H, H, lane, pre);  // next phase's first chunk, ahead of the barrier
  __syncthreads();
  ST_STAMP(2);
  st_lds_to_kt(Ah, ldh, H, r0, h1_kt);

  // S2: emb = h1 @ Wfc^T + bfc
  for (int cc = wave * 16; cc < H; cc += HNW * 16) {
    float4_t acc[HFM][1];
    st_zero(acc);
    st_gemm_lds_glb<HFM>(Ah, ldh, Wfc, cc, H, acc, lane, pre);
    if (cc + HNW * 16 < H) st_prefetch(Wfc, cc + HNW * 16, H, H, lane, pre);
    const int col = cc + lr;
    const float b = bfc[col];
#pragma unroll
    for (int m = 0; m < HFM; ++m) {
      float e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        e[j] = bf2f(f2bf(acc[m][0][j] + b));
        Eb[(m * 16 + lg * 4 + j) * ldh + col] = f2bf(e[j]);
      }
      st_kt4(emb_kt, r0 + m * 16 + lg * 4, col, H, e[0], e[1], e[2], e[3]);
    }
  }
  st_prefetch(Wout, wave * 16, C, H, lane, pre);  // next phase's first chunk, ahead of the barrier
  __syncthreads();
  ST_STAMP(3);

  // S3: logits = emb @ Wout^T ; dlogits, loss
  float lsum = 0.f;
  for (int cc = wave * 16; cc < C; cc += HNW * 16) {
    float4_t acc[HFM][1];
    st_zero(acc);
    st_gemm_lds_glb<HFM>(Eb, ldh, Wout, cc, H, acc, lane, pre);
    if (cc + HNW * 16 < C) st_prefetch(Wout, cc + HNW * 16, C, H, lane, pre);
    const int col = cc + lr;
#pragma unroll
    for (int m = 0; m < HFM; ++m) {
      float d[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + lg * 4 + j;
        const float xv = acc[m][0][j];
        const float y = (lab_s[row] == col) ? 1.f : 0.f;
        const float p = 1.f / (1.f + __expf(-xv));
        lsum += fmaxf(xv, 0.f) - xv * y + log1pf(__expf(-fabsf(xv)));
        d[j] = bf2f(f2bf((p - y) * inv_scale));
        Dl[row * ldc + col] = f2bf(d[j]);
      }
      st_kt4(dlog_kt, r0 + m * 16 + lg * 4, col, C, d[0], d[1], d[2], d[3]);
    }
  }
  if (wave * 16 < C) {
    lsum = wave_sum(lsum);
    if (lane == 0) atomicAdd(loss_acc, lsum * inv_scale);
  }
  st_prefetch(WoutT, wave * 16, H, C, lane, pre);  // next phase's first chunk, ahead of the barrier
  __syncthreads();
  ST_STAMP(4);

  // S4: demb = dlogits @ Wout (B operand from WoutT [H][C]); dbfc = column sums
  for (int cc = wave * 16; cc < H; cc += HNW * 16) {
    float4_t acc[HFM][1];
    st_zero(acc);
    st_gemm_lds_glb<HFM>(Dl, ldc, WoutT, cc, C, acc, lane, pre);
    if (cc + HNW * 16 < H) st_prefetch(WoutT, cc + HNW * 16, H, C, lane, pre);
    const int col = cc + lr;
    float cs = 0.f;
#pragma unroll
    for (int m = 0; m < HFM; ++m) {
      float e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        cs += acc[m][0][j];
        e[j] = bf2f(f2bf(acc[m][0][j]));
        Db[(m * 16 + lg * 4 + j) * ldh + col] = f2bf(e[j]);
      }
      st_kt4(demb_kt, r0 + m * 16 + lg * 4, col, H, e[0], e[1], e[2], e[3]);
    }
    cs += __shfl_xor(cs, 16, 64);
    cs += __shfl_xor(cs, 32, 64);
    if (lg == 0) atomicAdd(dbfc + col, cs);
  }
  st_prefetch(WfcT, wave * 16, H, H, lane, pre);  // next phase's first chunk, ahead of the barrier
  __syncthreads();
  ST_STAMP(5);

  // S5: dh1 = demb @ Wfc (B operand from WfcT); g1 = dh1 * (h1 > 0) -> Eb, g1_kt
  for (int cc = wave * 16; cc < H; cc += HNW * 16) {
    float4_t acc[HFM][1];
    st_zero(acc);
    st_gemm_lds_glb<HFM>(Db, ldh, WfcT, cc, H, acc, lane, pre);
    if (cc + HNW * 16 < H) st_prefetch(WfcT, cc + HNW * 16, H, H, lane, pre);
    const int col = cc + lr;
#pragma unroll
    for (int m = 0; m < HFM; ++m) {
      float e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = m * 16 + lg * 4 + j;
        e[j] = bf2f(f2bf(bf_pos(Ah[row * ldh + col]) ? acc[m][0][j] : 0.f));
        Eb[row * ldh + col] = f2bf(e[j]);
      }
      st_kt4(g1_kt, r0 + m * 16 + lg * 4, col, H, e[0], e[1], e[2], e[3]);
    }
  }
  st_prefetch(W1T, wave * 16, H2, H, lane, pre);  // next phase's first chunk, ahead of the barrier
  __syncthreads();
  ST_STAMP(6);

  // S6: dA1 = g1 @ W1 (B operand from W1T [2H][H]) -> fp32 row-major [B][2H]
  for (int cc = wave * 16; cc < H2; cc += HNW * 16) {
    float4_t acc[HFM][1];
    st_zero(acc);
    st_gemm_lds_glb<HFM>(Eb, ldh, W1T, cc, H, acc, lane, pre);
    if (cc + HNW * 16 < H2) st_prefetch(W1T, cc + HNW * 16, H2, H, lane, pre);
#pragma unroll
    for (int m = 0; m < HFM; ++m)
#pragma unroll
      for (int j = 0; j < 4; ++j) dA1[(r0 + m * 16 + lg * 4 + j) * H2 + cc + lr] = acc[m][0][j];
  }
  ST_STAMP(7);
#undef ST_STAMP
}

// ----------------------------------------------------------------------------
// 4. route dA1 back to the level-1 rows through the tree layout, apply the L0 ReLU
//    mask and emit g0 in kt layout.
//    rows [0, B*F1): neighbour slot k of target r / F1 ; rows [B*F1, M1): self of r - B*F1
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void st_route_kernel(const float* __restrict__ dA1, int H, int nb_rows,
                                                       uint32_t magic, int shift, int include_self, float inv_cnt,
                                                       const uint32_t* __restrict__ mask, bf16_t* __restrict__ g0_kt) {
  // one block = one 32-row k-block; item = (column n, 8-row chunk q): 4 lanes cover a
  // column's 32 rows, so a wave stores 16 columns x 64 B = 1 KB contiguous of the kt
  // output.  The L0 ReLU mask comes from the forward's bit mask ([M/32][H], bit = row&31),
  // so h0 is never re-read; row -> target is a 32-bit magic division.  A thread's U items
  // issue all their loads before any use (one exposed latency per thread, not 2U).
  constexpr int U = 4;
  const int kb = blockIdx.x;
  const uint32_t H2 = 2u * static_cast<uint32_t>(H);  // dA1 holds < 2^31 elements: 32-bit offsets
  const float inv_self = include_self ? inv_cnt : 0.f;
  const int items = H * 4;
  for (int base = 0; base < items; base += 256 * U) {
    uint32_t bits[U];
    float v[U][8];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      // branch-free: every load is unconditional (clamped item, selected address), so the
      // compiler issues all 2*8*U of them before the first wait
      const int it = min(base + u * 256 + static_cast<int>(threadIdx.x), items - 1);
      const uint32_t q = it & 3, n = it >> 2;
      bits[u] = (mask[static_cast<int64_t>(kb) * H + n] >> (q * 8)) & 0xffu;
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const uint32_t r = static_cast<uint32_t>(kb) * 32u + q * 8u + static_cast<uint32_t>(i);
        const bool nb = static_cast<int>(r) < nb_rows;
        const uint32_t tn = shift < 0 ? r : (__umulhi(r, magic) >> shift);
        const uint32_t ts = nb ? 0u : r - static_cast<uint32_t>(nb_rows);
        const float x1 = dA1[nb ? tn * H2 + H + n : ts * H2 + n];
        const float x2 = dA1[ts * H2 + H + n];
        // arithmetic blend (not a select) so neither load can be sunk into a branch
        const float w1 = nb ? inv_cnt : 1.f, w2 = nb ? 0.f : inv_self;
        v[u][i] = x1 * w1 + x2 * w2;
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int it = base + u * 256 + threadIdx.x;
      if (it >= items) continue;
      const int q = it & 3, n = it >> 2;
#pragma unroll
      for (int i = 0; i < 8; ++i) v[u][i] = ((bits[u] >> i) & 1u) ? v[u][i] : 0.f;
      *reinterpret_cast<uint4_t*>(g0_kt + (static_cast<int64_t>(kb) * H + n) * 32 + q * 8) = pack_bf16x8(v[u]);
    }
  }
}

// ----------------------------------------------------------------------------
// 5. grouped split-K weight gradients: part[s][p][q] = sum_{m in split s} G[m][p] X[m][q]
//    for up to 4 problems in one launch; 64x64 tiles, 4 waves of 32x32.
// ----------------------------------------------------------------------------
struct StDwProb {
  const bf16_t* G;
  const bf16_t* X;
  float* part;
  int P, Q, MB, kps, S, tiles_q, ntiles, wg0;
  // route mode (outer SAGE layer): G = g0 is never materialised; its fragments are built
  // from dA1 [B][2P] (fp32), the tree layout and the forward's ReLU mask bits
  const uint32_t* mask;
  const float* dA1;
  int route, nb_rows, include_self;
  uint32_t magic;  // t = mulhi(m, magic) >> shift  ==  m / F1  for m < 2^31
  int shift;
  float inv_cnt;
};

// G^T fragment of the outer layer: rows mb*32 + lk .. +7 at column p
__device__ __forceinline__ uint4_t st_route_frag(const StDwProb& pr, int mb, int p, int lk) {
  const uint32_t bits = (pr.mask[static_cast<int64_t>(mb) * pr.P + p] >> lk) & 0xffu;
  const int64_t H2 = 2 * static_cast<int64_t>(pr.P);
  float v[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) {
    float val = 0.f;
    if ((bits >> i) & 1u) {
      const uint32_t m = static_cast<uint32_t>(mb) * 32u + static_cast<uint32_t>(lk + i);
      if (static_cast<int>(m) < pr.nb_rows) {
        const uint32_t t = __umulhi(m, pr.magic) >> pr.shift;
        val = pr.dA1[t * H2 + pr.P + p] * pr.inv_cnt;
      } else {
        const int64_t t = static_cast<int64_t>(m) - pr.nb_rows;
        val = pr.dA1[t * H2 + p];
        if (pr.include_self) val += pr.dA1[t * H2 + pr.P + p] * pr.inv_cnt;
      }
    }
    v[i] = val;
  }
  return pack_bf16x8(v);
}
struct StDwProbs {
  StDwProb p[4];
  int n;
};

__global__ __launch_bounds__(256) void st_dw_kernel(StDwProbs probs) {
  const int id = xcd_remap(blockIdx.x, gridDim.x);
  // select the problem with constant indices only (no dynamic indexing of kernel args)
  StDwProb pr = probs.p[0];
  if (probs.n > 1 && id >= probs.p[1].wg0) pr = probs.p[1];
  if (probs.n > 2 && id >= probs.p[2].wg0) pr = probs.p[2];
  if (probs.n > 3 && id >= probs.p[3].wg0) pr = probs.p[3];
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
  if (p0 >= P || q0 >= Q) return;  // 32-wide edge of a 64-wide tile (P or Q % 64 == 32); no barriers here
  float4_t acc[2][2];
  st_zero(acc);
  if (pr.route) {
    constexpr int KR = 4;
    for (int mbc = mb0; mbc < mb1; mbc += KR) {
      uint4_t a[KR][2], b[KR][2];
#pragma unroll
      for (int u = 0; u < KR; ++u)
#pragma unroll
        for (int f = 0; f < 2; ++f) {
          const int mb = mbc + u;
          const bool ok = mb < mb1;
          b[u][f] = ok ? *reinterpret_cast<const uint4_t*>(pr.X + ((mb * Q + q0 + f * 16 + lr) * 32 + lk))
                       : uint4_t{0u, 0u, 0u, 0u};
          a[u][f] = ok ? st_route_frag(pr, mb, p0 + f * 16 + lr, lk) : uint4_t{0u, 0u, 0u, 0u};
        }
#pragma unroll
      for (int u = 0; u < KR; ++u)
#pragma unroll
        for (int fm = 0; fm < 2; ++fm)
#pragma unroll
          for (int fn = 0; fn < 2; ++fn) acc[fm][fn] = st_mfma(a[u][fm], b[u][fn], acc[fm][fn]);
    }
  }
  // 8 k-blocks of fragments in flight per wave (the grid is ~2 waves per SIMD, so the
  // loop is latency-bound unless many loads are outstanding)
  constexpr int KB = 8;
  for (int mbc = pr.route ? mb1 : mb0; mbc < mb1; mbc += KB) {
    uint4_t a[KB][2], b[KB][2];
#pragma unroll
    for (int u = 0; u < KB; ++u)
#pragma unroll
      for (int f = 0; f < 2; ++f) {
        const int64_t mb = mbc + u;
        const bool ok = mb < mb1;
        a[u][f] = ok ? *reinterpret_cast<const uint4_t*>(pr.G + ((mb * P + p0 + f * 16 + lr) * 32 + lk))
                     : uint4_t{0u, 0u, 0u, 0u};
        b[u][f] = ok ? *reinterpret_cast<const uint4_t*>(pr.X + ((mb * Q + q0 + f * 16 + lr) * 32 + lk))
                     : uint4_t{0u, 0u, 0u, 0u};
      }
#pragma unroll
    for (int u = 0; u < KB; ++u)
#pragma unroll
      for (int fm = 0; fm < 2; ++fm)
#pragma unroll
        for (int fn = 0; fn < 2; ++fn) acc[fm][fn] = st_mfma(a[u][fm], b[u][fn], acc[fm][fn]);
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

// ----------------------------------------------------------------------------
// 6. split-K reduce into the flat gradient (overwrites)
// ----------------------------------------------------------------------------
struct StRed {
  const float* part[4];
  float* out[4];
  int64_t n4[4];  // float4 count per problem
  int S[4];
  int n;
};

__global__ __launch_bounds__(256) void st_reduce_kernel(StRed rd) {
  int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
#pragma unroll
  for (int p = 0; p < 4; ++p) {
    if (p < rd.n && i < rd.n4[p]) {
      const float4_t* src = reinterpret_cast<const float4_t*>(rd.part[p]) + i;
      const int64_t stride = rd.n4[p];
      const int S = rd.S[p];
      float4_t acc = float4_t{0.f, 0.f, 0.f, 0.f};
      // 8 independent partial loads in flight per iteration
      for (int s0 = 0; s0 < S; s0 += 8) {
        float4_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = (s0 + u < S) ? src[(s0 + u) * stride] : float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int u = 0; u < 8; ++u) acc += v[u];
      }
      reinterpret_cast<float4_t*>(rd.out[p])[i] = acc;
      return;
    }
    i -= rd.n4[p];
  }
}

// ----------------------------------------------------------------------------
// 7. Adam over the flat parameters + bf16 (and transposed bf16) weight shadows for the
//    next step's MFMAs, zeroing of atomically accumulated grads, loss hand-off and the
//    RNG counter advance (hipGraph-replay safe: all state lives on the device).
// ----------------------------------------------------------------------------
struct StShadow {
  int64_t off[6];
  int64_t n[6];
  int cols[6];
  bf16_t* sh[6];
  bf16_t* shT[6];
  int count;
};

// element i of the flat buffer -> its bf16 shadow (and transposed shadow) if it is a weight
__device__ __forceinline__ void st_write_shadow(const StShadow& sh, int64_t i, float val) {
#pragma unroll
  for (int s = 0; s < 6; ++s) {
    if (s >= sh.count) break;
    const int64_t l = i - sh.off[s];
    if (l >= 0 && l < sh.n[s]) {
      // both shadows in fm layout: W [rows][cols] and W^T [cols][rows]
      const bf16_t b = f2bf(val);
      const int64_t rows = sh.n[s] / sh.cols[s];
      const int64_t r = l / sh.cols[s], c = l - r * sh.cols[s];
      sh.sh[s][fm_off(r, c, sh.cols[s])] = b;
      if (sh.shT[s]) sh.shT[s][fm_off(c, r, rows)] = b;
    }
  }
}

__global__ __launch_bounds__(256) void st_adam_kernel(float* __restrict__ p, float* __restrict__ g,
                                                      float* __restrict__ m, float* __restrict__ v, int64_t n,
                                                      const int64_t* __restrict__ step, float lr, float b1, float b2,
                                                      float eps, float wd, float grad_scale, StShadow sh,
                                                      int64_t zero_off, int64_t zero_n, float* __restrict__ loss_acc,
                                                      float* __restrict__ loss_out, int64_t* __restrict__ rng) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i == 0) {
    loss_out[0] = loss_acc[0];
    loss_acc[0] = 0.f;
    rng[1] += 1;
  }
  if (i >= n) return;
  const float gi = g[i] * grad_scale + wd * p[i];
  const float t = static_cast<float>(step[0]);
  const float mi = b1 * m[i] + (1.f - b1) * gi;
  const float vi = b2 * v[i] + (1.f - b2) * gi * gi;
  m[i] = mi;
  v[i] = vi;
  const float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
  const float pi = p[i] - lr * (mi / bc1) / (sqrtf(vi / bc2) + eps);
  p[i] = pi;
  if (i >= zero_off && i < zero_off + zero_n) g[i] = 0.f;
  st_write_shadow(sh, i, pi);
}

// initial shadows (before the first step) without an update
__global__ __launch_bounds__(256) void st_shadow_kernel(const float* __restrict__ p, int64_t n, StShadow sh) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  st_write_shadow(sh, i, p[i]);
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

hipError_t eh_st_roots(const float* prob, const int32_t* alias, int64_t pop, int B, const int64_t* rng,
                       uint64_t stream_id, const int16_t* labels, int32_t* roots, int32_t* level1_tail,
                       int32_t* label_idx, int64_t* step, hipStream_t s) {
  hipLaunchKernelGGL(st_roots_kernel, dim3(static_cast<uint32_t>(ceil_div(B, 256))), dim3(256), 0, s, prob, alias,
                     pop, B, rng, stream_id, labels, roots, level1_tail, label_idx, step);
  return hipGetLastError();
}

hipError_t eh_st_sage_fwd(const void* x, int D, const int32_t* self_idx, const int32_t* nbr_idx, int F,
                          int include_self, float inv_cnt, const void* W, int H, int64_t M, void* out, void* a_kt,
                          uint32_t* relu_mask, int bm, hipStream_t s) {
  if (M == 0) return hipSuccess;
  if (D % 16 != 0 || D > 512 || H % 64 != 0 || M % 32 != 0) return hipErrorInvalidValue;
  if (relu_mask && bm % 32 != 0) return hipErrorInvalidValue;
  const int BN = 256;
  const bool alias_out = H <= BN && BN <= 2 * D;  // must match the kernel's choice
  const size_t lds = (static_cast<size_t>(bm) * (2 * D + 8) + (alias_out ? 0 : static_cast<size_t>(bm) * (BN + 8))) *
                     sizeof(bf16_t);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const dim3 grid(static_cast<uint32_t>(ceil_div(M, bm)));
#define ST_LAUNCH(BMV)                                                                                         \
  do {                                                                                                         \
    EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(st_sage_fwd_kernel<BMV, 256>),            \
                                        hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));                \
    hipLaunchKernelGGL((st_sage_fwd_kernel<BMV, 256>), grid, dim3(256), lds, s, static_cast<const bf16_t*>(x), D, \
                       self_idx, nbr_idx, F, include_self, inv_cnt, static_cast<const bf16_t*>(W), H, M,        \
                       static_cast<bf16_t*>(out), static_cast<bf16_t*>(a_kt), relu_mask);                      \
  } while (0)
  if (bm == 16) ST_LAUNCH(16);
  else if (bm == 32) ST_LAUNCH(32);
  else if (bm == 64) ST_LAUNCH(64);
  else return hipErrorInvalidValue;
#undef ST_LAUNCH
  return hipGetLastError();
}

hipError_t eh_st_tree_mean(const void* h0, int H, int64_t B, int F1, int include_self, float inv_cnt, void* A1,
                           hipStream_t s) {
  if (H % 8 != 0) return hipErrorInvalidValue;
  const int64_t items = B * (2 * H / 8);
  hipLaunchKernelGGL(st_tree_mean_kernel, dim3(static_cast<uint32_t>(ceil_div(items, 256))), dim3(256), 0, s,
                     static_cast<const bf16_t*>(h0), H, B, F1, include_self, inv_cnt, static_cast<bf16_t*>(A1));
  return hipGetLastError();
}

hipError_t eh_st_head(const void* A1, int B, int H, int C, const void* W1b, const void* Wfc, const void* WfcT,
                      const float* bfc, const void* Wout, const void* WoutT, const void* W1T, const int32_t* label_idx,
                      float inv_scale, void* A1_kt, void* h1_kt, void* emb_kt, void* dlog_kt, void* demb_kt,
                      void* g1_kt, float* dA1, float* dbfc, float* loss_acc, long long* prof, hipStream_t s) {
  if (B % HB != 0 || H % 64 != 0 || C % 32 != 0 || C > 256) return hipErrorInvalidValue;
  const size_t lds = (static_cast<size_t>(HB) * (2 * H + 8) + 3 * static_cast<size_t>(HB) * (H + 8) +
                      static_cast<size_t>(HB) * (C + 8)) * sizeof(bf16_t);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(st_head_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  hipLaunchKernelGGL(st_head_kernel, dim3(B / HB), dim3(HNW * 64), lds, s, static_cast<const bf16_t*>(A1), H, C,
                     static_cast<const bf16_t*>(W1b), static_cast<const bf16_t*>(Wfc),
                     static_cast<const bf16_t*>(WfcT), bfc, static_cast<const bf16_t*>(Wout),
                     static_cast<const bf16_t*>(WoutT), static_cast<const bf16_t*>(W1T), label_idx, inv_scale,
                     static_cast<bf16_t*>(A1_kt), static_cast<bf16_t*>(h1_kt), static_cast<bf16_t*>(emb_kt),
                     static_cast<bf16_t*>(dlog_kt), static_cast<bf16_t*>(demb_kt), static_cast<bf16_t*>(g1_kt), dA1,
                     dbfc, loss_acc, prof);
  return hipGetLastError();
}

// round-up magic division, exact for 31-bit numerators and F1 >= 2: l = ceil(log2 F1),
// magic = ceil(2^(31+l) / F1), m / F1 == mulhi(m, magic) >> (l - 1)
static void st_magic(int F1, uint32_t* magic, int* shift) {
  int l = 0;
  while ((int64_t(1) << l) < F1) ++l;
  const uint64_t num = uint64_t(1) << (31 + l);
  *magic = static_cast<uint32_t>((num + static_cast<uint64_t>(F1) - 1) / static_cast<uint64_t>(F1));
  *shift = l - 1;
}

hipError_t eh_st_route(const float* dA1, int H, int64_t nb_rows, int F1, int include_self, float inv_cnt,
                       const uint32_t* mask, int64_t M1, void* g0_kt, hipStream_t s) {
  if (M1 % 32 != 0 || H % 8 != 0 || F1 < 1 || M1 >= (int64_t(1) << 31)) return hipErrorInvalidValue;
  uint32_t magic = 0;
  int shift = -1;  // F1 == 1: identity
  if (F1 >= 2) st_magic(F1, &magic, &shift);
  hipLaunchKernelGGL(st_route_kernel, dim3(static_cast<uint32_t>(M1 / 32)), dim3(256), 0, s, dA1, H,
                     static_cast<int>(nb_rows), magic, shift, include_self, inv_cnt, mask,
                     static_cast<bf16_t*>(g0_kt));
  return hipGetLastError();
}

// probs: n problems of (G_kt, X_kt, part, P, Q, M, kps)
hipError_t eh_st_dw(int n, const void* const* G, const void* const* X, float* const* part, const int* P,
                    const int* Q, const int64_t* M, const int* kps, const uint32_t* route_mask,
                    const float* route_dA1, int64_t nb_rows, int F1, int include_self, float inv_cnt, hipStream_t s) {
  if (n < 1 || n > 4) return hipErrorInvalidValue;
  StDwProbs pr{};
  pr.n = n;
  int wg = 0;
  for (int i = 0; i < n; ++i) {
    if (P[i] % 32 != 0 || Q[i] % 32 != 0 || M[i] % 32 != 0 || kps[i] < 1) return hipErrorInvalidValue;
    StDwProb& p = pr.p[i];
    if (i == 0 && route_mask) {
      if (F1 < 2 || M[0] >= (int64_t(1) << 31)) return hipErrorInvalidValue;
      p.route = 1;
      p.mask = route_mask;
      p.dA1 = route_dA1;
      p.nb_rows = static_cast<int>(nb_rows);
      p.include_self = include_self;
      p.inv_cnt = inv_cnt;
      // round-up magic division, exact for 31-bit numerators: l = ceil(log2 F1),
      // magic = ceil(2^(31+l) / F1), m / F1 == mulhi(m, magic) >> (l - 1)
      st_magic(F1, &p.magic, &p.shift);
    }
    p.G = static_cast<const bf16_t*>(G[i]);
    p.X = static_cast<const bf16_t*>(X[i]);
    p.part = part[i];
    p.P = P[i];
    p.Q = Q[i];
    p.MB = static_cast<int>(M[i] / 32);
    p.kps = kps[i];
    p.S = static_cast<int>(ceil_div(p.MB, kps[i]));
    p.tiles_q = (Q[i] + 63) / 64;
    p.ntiles = ((P[i] + 63) / 64) * p.tiles_q;
    p.wg0 = wg;
    wg += p.ntiles * p.S;
  }
  hipLaunchKernelGGL(st_dw_kernel, dim3(wg), dim3(256), 0, s, pr);
  return hipGetLastError();
}

hipError_t eh_st_reduce(int n, const float* const* part, float* const* out, const int64_t* numel, const int* S,
                        hipStream_t s) {
  if (n < 1 || n > 4) return hipErrorInvalidValue;
  StRed rd{};
  rd.n = n;
  int64_t tot = 0;
  for (int i = 0; i < n; ++i) {
    if (numel[i] % 4 != 0) return hipErrorInvalidValue;
    rd.part[i] = part[i];
    rd.out[i] = out[i];
    rd.n4[i] = numel[i] / 4;
    rd.S[i] = S[i];
    tot += rd.n4[i];
  }
  hipLaunchKernelGGL(st_reduce_kernel, dim3(static_cast<uint32_t>(ceil_div(tot, 256))), dim3(256), 0, s, rd);
  return hipGetLastError();
}

static hipError_t st_fill_shadow(StShadow& sh, int count, const int64_t* off, const int64_t* n, const int* cols,
                                 void* const* shadow, void* const* shadowT) {
  if (count > 6) return hipErrorInvalidValue;
  sh.count = count;
  for (int i = 0; i < count; ++i) {
    // fm layout needs rows % 16 == 0 and cols % 32 == 0 (and the transpose the converse)
    if (cols[i] <= 0 || n[i] % cols[i] != 0) return hipErrorInvalidValue;
    const int64_t rows = n[i] / cols[i];
    if (rows % 16 != 0 || cols[i] % 32 != 0) return hipErrorInvalidValue;
    if (shadowT[i] && (rows % 32 != 0 || cols[i] % 16 != 0)) return hipErrorInvalidValue;
    sh.off[i] = off[i];
    sh.n[i] = n[i];
    sh.cols[i] = cols[i];
    sh.sh[i] = static_cast<bf16_t*>(shadow[i]);
    sh.shT[i] = static_cast<bf16_t*>(shadowT[i]);
  }
  return hipSuccess;
}

hipError_t eh_st_adam(float* p, float* g, float* m, float* v, int64_t n, const int64_t* step, float lr, float b1,
                      float b2, float eps, float wd, float grad_scale, int sh_count, const int64_t* sh_off,
                      const int64_t* sh_n, const int* sh_cols, void* const* sh_ptr, void* const* shT_ptr,
                      int64_t zero_off, int64_t zero_n, float* loss_acc, float* loss_out, int64_t* rng,
                      hipStream_t s) {
  StShadow sh{};
  EULER_HIP_CHECK(st_fill_shadow(sh, sh_count, sh_off, sh_n, sh_cols, sh_ptr, shT_ptr));
  hipLaunchKernelGGL(st_adam_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, p, g, m, v, n,
                     step, lr, b1, b2, eps, wd, grad_scale, sh, zero_off, zero_n, loss_acc, loss_out, rng);
  return hipGetLastError();
}

hipError_t eh_st_shadow(const float* p, int64_t n, int sh_count, const int64_t* sh_off, const int64_t* sh_n,
                        const int* sh_cols, void* const* sh_ptr, void* const* shT_ptr, hipStream_t s) {
  StShadow sh{};
  EULER_HIP_CHECK(st_fill_shadow(sh, sh_count, sh_off, sh_n, sh_cols, sh_ptr, shT_ptr));
  hipLaunchKernelGGL(st_shadow_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, p, n, sh);
  return hipGetLastError();
}

}  // extern "C"
