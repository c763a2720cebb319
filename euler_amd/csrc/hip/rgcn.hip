// K6: relation-typed transform for R-GCN as a grouped MFMA GEMM.
//
// Reference (tf_euler/python/convolution/relation_conv.py:63-70): every edge gathers its
// own [dim, fea_dim] relation matrix and does a batched [E, dim, fea] x [E, fea, 1] matmul,
// i.e. it materialises E x dim x fea floats.  Here the edges are sorted by relation once
// per block and cut into tiles of <= 64 edges of ONE relation; a workgroup gathers its
// tile's source rows into LDS (the gather is fused into the GEMM prologue) and multiplies
// by that relation's weight with bf16 MFMA (16x16x32, fp32 accumulate).  The epilogue
// either stores the messages (bf16) or scales them and atomically adds them into the
// destination rows (mean aggregation fused: no [E, dim] buffer at all).
//
//   rel_gemm    : Y[o_idx[e]] (+)= scale[e] * A[a_idx[e]] @ B[rel]^T
//                 forward  (A = x,    B = W  [R][N][K], o = dst)
//                 backward (A = dout, B = W^T [R][K][N], o = src)  -> dx
//   rel_gemm_dw : dW[rel] += sum_e (scale[e] * G[g_idx[e]])^T X[x_idx[e]]  (per-chunk
//                 outer-product GEMM, fragments by transposing LDS reads; a relation's
//                 only chunk stores its slab, longer relations add with fp32 atomics)
#include <algorithm>
#include <cstdlib>

#include "hip/common.h"
#include "hip/launchers.h"
#include "hip/tile.h"

namespace euler_hip {

typedef __bf16 rg_bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float4_t rg_mfma(uint4_t a, uint4_t b, float4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(rg_bf16x8, a), __builtin_bit_cast(rg_bf16x8, b),
                                                 c, 0, 0, 0);
}

constexpr int RG_BM = 64;  // edges per tile

#ifndef RG_TM
#define RG_TM 128  // max edges per message-GEMM tile (tm): one W_rel read serves up to tm edges;
                   // gnn_ops picks tm = 64 (sweep: profiles/r2_final/sweeps/rel_gemm_tile.txt)
#endif
constexpr int RG_TMF = RG_TM / 16;

__global__ __launch_bounds__(256) void rel_gemm_kernel(const bf16_t* __restrict__ A, int K,
                                                       const int32_t* __restrict__ a_idx,
                                                       const int32_t* __restrict__ trel,
                                                       const int32_t* __restrict__ tstart,
                                                       const int32_t* __restrict__ tlen, const bf16_t* __restrict__ B,
                                                       int N, const float* __restrict__ scale,
                                                       const int32_t* __restrict__ o_idx, int mode, int tm, void* Y) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  __shared__ int32_t orow_s[RG_TM];
  __shared__ float osc_s[RG_TM];
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int r = trel[t], e0 = tstart[t], ne = min(tlen[t], tm);  // tm bounds the LDS rows
  const int ldk = K + 8;
  const int cpr = K >> 3;
  // epilogue bookkeeping per tile row: output row and scale
  for (int row = threadIdx.x; row < RG_TM; row += 256) {
    orow_s[row] = row < ne ? o_idx[e0 + row] : -1;
    osc_s[row] = (row < ne && scale) ? scale[e0 + row] : 1.f;
  }
  // prologue: gather the tile's A rows (zero rows past the tile / for padding ids)
  for (int it = threadIdx.x; it < tm * cpr; it += 256) {
    const int row = it / cpr, c = it - row * cpr;
    uint4_t v = {0u, 0u, 0u, 0u};
    if (row < ne) {
      const int64_t src = a_idx[e0 + row];
      if (src >= 0) v = *reinterpret_cast<const uint4_t*>(A + src * K + c * 8);
    }
    *reinterpret_cast<uint4_t*>(lds + row * ldk + c * 8) = v;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  const bf16_t* __restrict__ Br = B + static_cast<int64_t>(r) * N * K;
  const int ldn = N + 8;
  bf16_t* otile = lds + tm * ldk;  // mode 0 output tile [tm][N + 8]
  // fragments past the tile's last edge multiply zero rows: skip them (uniform per block)
  const int mf = (ne + 15) >> 4;
  for (int n0 = wave * 16; n0 < N; n0 += 64) {
    float4_t acc[RG_TMF];
#pragma unroll
    for (int m = 0; m < RG_TMF; ++m) acc[m] = float4_t{0.f, 0.f, 0.f, 0.f};
    uint4_t b = *reinterpret_cast<const uint4_t*>(Br + static_cast<int64_t>(n0 + lr) * K + lk);
    for (int k0 = 0; k0 < K; k0 += 32) {
      const bool more = k0 + 32 < K;
      const uint4_t bn = more ? *reinterpret_cast<const uint4_t*>(Br + static_cast<int64_t>(n0 + lr) * K + k0 + 32 + lk)
                              : uint4_t{0u, 0u, 0u, 0u};
#pragma unroll
      for (int m = 0; m < RG_TMF; ++m) {
        if (m < mf) {
          const uint4_t a = *reinterpret_cast<const uint4_t*>(lds + (m * 16 + lr) * ldk + k0 + lk);
          acc[m] = rg_mfma(a, b, acc[m]);
        }
      }
      b = bn;
    }
    const int col = n0 + lr;
    if (mode == 0) {
      // stage the bf16 tile in LDS; rows leave as 16-byte stores below
#pragma unroll
      for (int m = 0; m < RG_TMF; ++m)
        if (m < mf)  // rows < tm: inside the tile's LDS rows
#pragma unroll
          for (int j = 0; j < 4; ++j) {
            const int row = m * 16 + (lane >> 4) * 4 + j;
            otile[row * ldn + col] = f2bf(acc[m][j] * osc_s[row]);
          }
    } else {
#pragma unroll
      for (int m = 0; m < RG_TMF; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = m * 16 + (lane >> 4) * 4 + j;
          const int64_t o = orow_s[row];
          if (o >= 0) atomicAdd(static_cast<float*>(Y) + o * N + col, acc[m][j] * osc_s[row]);
        }
    }
  }
  if (mode == 0) {
    __syncthreads();
    const int cpn = N >> 3;
    for (int it = threadIdx.x; it < ne * cpn; it += 256) {
      const int row = it / cpn, c = it - row * cpn;
      const int64_t o = orow_s[row];
      if (o >= 0)
        *reinterpret_cast<uint4_t*>(static_cast<bf16_t*>(Y) + o * N + c * 8) =
            *reinterpret_cast<const uint4_t*>(otile + row * ldn + c * 8);
    }
  }
}

// dW for one (chunk of <= RG_CH edges of ONE relation, T x T slab of dW[rel]) per workgroup:
// the chunk's 64-edge sub-tiles are staged in LDS and accumulated in registers, so each dW
// element receives one write per chunk instead of one atomic per 64-edge tile.
constexpr int RG_CH = 512;  // edges per dW chunk (256: same time, more atomics; 1024: long serial chunks)

// MFMA fragments of dW = Gs^T X straight from edge-major LDS images with the gfx950
// transposing read ds_read_b64_tr_b16: a 16-lane group reads a 4-edge x 16-column block and
// lane i receives column i (4 edges).  Two reads give the 8 reduction elements of a lane:
// group g takes edges e0 + 4g .. +3 and e0 + 16 + 4g .. +3 (A and B use the same edge map,
// which is all the MFMA needs).  Images are [64 edges][T + 16] bf16: with a row stride of
// 40 (T = 64) or 72 (T = 128) dwords the 8 rows a 32-lane half reads land on 8 disjoint
// 8-bank sets (conflict-free), and the 16-byte row-segment stores of 8 consecutive lanes
// cover the 32 banks once.
// one workgroup = one (chunk of <= RG_CH edges of one relation) x (T x T slab of dW[rel]);
// T = 128 covers a 128 x 128 weight in one slab, so every edge row is read once.  Wave w
// owns rows w*T/4 .. of the slab (T/64 MFMA row tiles) x all T columns (T/16 tiles).
// A chunk that is its relation's only one (csolo) stores its slab (accum: adds it to the
// slab's current contents, no other workgroup touches that slab); otherwise fp32 atomics.
template <int T>
__global__ __launch_bounds__(256) void rel_gemm_dw_kernel(const bf16_t* __restrict__ G, int N,
                                                          const int32_t* __restrict__ g_idx,
                                                          const bf16_t* __restrict__ X, int K,
                                                          const int32_t* __restrict__ x_idx,
                                                          const float* __restrict__ scale,
                                                          const int32_t* __restrict__ crel,
                                                          const int32_t* __restrict__ cstart,
                                                          const int32_t* __restrict__ clen,
                                                          const int32_t* __restrict__ csolo, float* __restrict__ dW,
                                                          int accum, const int32_t* __restrict__ cslot,
                                                          float* __restrict__ part) {
  constexpr int LD = T + 16;
  constexpr int FM = T / 64, FN = T / 16;
  constexpr int CPR = T / 8;               // 16-byte chunks per row segment
  constexpr int IT = RG_BM * CPR / 256;    // items per thread and operand
  __shared__ __attribute__((aligned(16))) bf16_t gS[RG_BM * LD];
  __shared__ __attribute__((aligned(16))) bf16_t xS[RG_BM * LD];
  const int SN = N / T, SK = K / T;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = b / (SN * SK), s = b - chunk * (SN * SK);
  const int sn = s / SK, sk = s - sn * SK;
  const int r = crel[chunk], c0 = cstart[chunk], clen_ = clen[chunk];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  float4_t acc[FM][FN];
#pragma unroll
  for (int m = 0; m < FM; ++m)
#pragma unroll
    for (int f = 0; f < FN; ++f) acc[m][f] = float4_t{0.f, 0.f, 0.f, 0.f};
  // item = (edge e = it / CPR, 16-byte column chunk c = it % CPR): consecutive lanes move
  // one row segment (coalesced loads, conflict-free LDS stores).  The next sub-tile's rows
  // are loaded into registers while the current one's MFMAs run.
  uint4_t gv[IT], xv[IT];
  float gs[IT];
  auto prefetch = [&](int sub) {
    const int ne = min(RG_BM, clen_ - sub);
#pragma unroll
    for (int h = 0; h < IT; ++h) {
      const int it = threadIdx.x + h * 256;
      const int e = it / CPR, c = it % CPR;
      gv[h] = uint4_t{0u, 0u, 0u, 0u};
      xv[h] = uint4_t{0u, 0u, 0u, 0u};
      gs[h] = 0.f;
      if (e < ne) {
        const int64_t gi = g_idx[c0 + sub + e];
        const int64_t xi = x_idx[c0 + sub + e];
        if (gi >= 0) {
          gv[h] = *reinterpret_cast<const uint4_t*>(G + gi * N + sn * T + c * 8);
          gs[h] = scale ? scale[c0 + sub + e] : 1.f;
        }
        if (xi >= 0) xv[h] = *reinterpret_cast<const uint4_t*>(X + xi * K + sk * T + c * 8);
      }
    }
  };
  prefetch(0);
  for (int sub = 0; sub < clen_; sub += RG_BM) {
#pragma unroll
    for (int h = 0; h < IT; ++h) {
      const int it = threadIdx.x + h * 256;
      const int e = it / CPR, c = it % CPR;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      acc_bf16x8(v, gv[h], gs[h]);
      *reinterpret_cast<uint4_t*>(gS + e * LD + c * 8) = pack_bf16x8(v);
      *reinterpret_cast<uint4_t*>(xS + e * LD + c * 8) = xv[h];
    }
    __syncthreads();
    if (sub + RG_BM < clen_) prefetch(sub + RG_BM);
#pragma unroll
    for (int k0 = 0; k0 < RG_BM; k0 += 32) {
      uint4_t a[FM];
#pragma unroll
      for (int m = 0; m < FM; ++m) a[m] = tl_tr_frag<LD>(gS, k0, wave * (T / 4) + m * 16, lane);
#pragma unroll
      for (int f = 0; f < FN; ++f) {
        const uint4_t bb = tl_tr_frag<LD>(xS, k0, f * 16, lane);
#pragma unroll
        for (int m = 0; m < FM; ++m) acc[m][f] = rg_mfma(a[m], bb, acc[m][f]);
      }
    }
    __syncthreads();
  }
  float* __restrict__ dWr = dW + static_cast<int64_t>(r) * N * K;
  const bool solo = csolo && csolo[chunk];
  // deterministic mode (cslot): a chunk of a multi-chunk relation stores its slab into its
  // own partial slot; rel_dw_reduce_kernel adds the slots of each relation in chunk order
  if (cslot && !solo) dWr = part + static_cast<int64_t>(cslot[chunk]) * N * K;
#pragma unroll
  for (int m = 0; m < FM; ++m)
#pragma unroll
    for (int f = 0; f < FN; ++f)
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int n = sn * T + wave * (T / 4) + m * 16 + (lane >> 4) * 4 + j;
        float* dst = dWr + static_cast<int64_t>(n) * K + sk * T + f * 16 + (lane & 15);
        if (solo)
          *dst = accum ? *dst + acc[m][f][j] : acc[m][f][j];
        else if (cslot)
          *dst = acc[m][f][j];
        else
          atomicAdd(dst, acc[m][f][j]);
      }
}

// deterministic dW of the multi-chunk relations: dW[rel] (+)= sum of its partial slots in
// chunk order (slots rp[i] .. rp[i + 1] of the i-th multi-chunk relation mrel[i])
__global__ __launch_bounds__(256) void rel_dw_reduce_kernel(const float* __restrict__ part,
                                                            const int32_t* __restrict__ mrel,
                                                            const int32_t* __restrict__ rp, int nm, int64_t NK,
                                                            float* __restrict__ dW, int accum) {
  const int64_t total = static_cast<int64_t>(nm) * (NK >> 2);
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < total;
       t += static_cast<int64_t>(gridDim.x) * blockDim.x) {
    const int i = static_cast<int>(t / (NK >> 2));
    const int64_t e = (t - static_cast<int64_t>(i) * (NK >> 2)) * 4;
    float4_t v = float4_t{0.f, 0.f, 0.f, 0.f};
    const int s0 = rp[i], s1 = rp[i + 1];
    int sl = s0;
    for (; sl + 8 <= s1; sl += 8) {  // 8 slab loads in flight, added in slot order
      float4_t u[8];
#pragma unroll
      for (int k = 0; k < 8; ++k) u[k] = *reinterpret_cast<const float4_t*>(part + (sl + k) * NK + e);
#pragma unroll
      for (int k = 0; k < 8; ++k) v += u[k];
    }
    for (; sl < s1; ++sl) v += *reinterpret_cast<const float4_t*>(part + sl * NK + e);
    float4_t* d = reinterpret_cast<float4_t*>(dW + static_cast<int64_t>(mrel[i]) * NK + e);
    *d = accum ? *d + v : v;
  }
}

// bf16 operands of the relation weights for one step: wb[r] = bf16(W[r]) ([N][K], the
// forward B) and wt[r] = bf16(W[r])^T ([K][N], the backward B) from one read of the fp32
// weights; 64 x 64 tiles, the transpose through LDS (padded rows: conflict-free columns)
__global__ __launch_bounds__(256) void rel_weight_bf16_kernel(const float* __restrict__ W, int N, int K,
                                                              bf16_t* __restrict__ wb, bf16_t* __restrict__ wt) {
  __shared__ bf16_t t_s[64][66];
  const int tk = K >> 6, tn = N >> 6;
  const int64_t b = blockIdx.x;
  const int64_t r = b / (static_cast<int64_t>(tn) * tk);
  const int rem = static_cast<int>(b - r * tn * tk);
  const int n0 = (rem / tk) * 64, k0 = (rem % tk) * 64;
  const int tid = threadIdx.x, row = tid >> 2, c0 = (tid & 3) * 16;
  const int64_t base = r * static_cast<int64_t>(N) * K;
  const float* src = W + base + static_cast<int64_t>(n0 + row) * K + k0 + c0;
  float v[16];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const float4_t f = *reinterpret_cast<const float4_t*>(src + q * 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) v[q * 4 + j] = f[j];
  }
  bf16_t* dst = wb + base + static_cast<int64_t>(n0 + row) * K + k0 + c0;
  *reinterpret_cast<uint4_t*>(dst) = pack_bf16x8(v);
  *reinterpret_cast<uint4_t*>(dst + 8) = pack_bf16x8(v + 8);
#pragma unroll
  for (int j = 0; j < 16; ++j) t_s[row][c0 + j] = f2bf(v[j]);
  __syncthreads();
  // transposed: output row k0 + row (an input column), columns n0 + c0 .. + 15
  float u[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) u[j] = bf2f(t_s[c0 + j][row]);
  bf16_t* dT = wt + base + static_cast<int64_t>(k0 + row) * N + n0 + c0;
  *reinterpret_cast<uint4_t*>(dT) = pack_bf16x8(u);
  *reinterpret_cast<uint4_t*>(dT + 8) = pack_bf16x8(u + 8);
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

size_t eh_rel_gemm_lds(int K, int N, int mode, int tm) {
  return static_cast<size_t>(tm) * ((K + 8) + (mode == 0 ? N + 8 : 0)) * sizeof(bf16_t);
}

int eh_rel_gemm_tile() { return RG_TM; }

hipError_t eh_rel_gemm(const void* A, int K, const int32_t* a_idx, const int32_t* trel, const int32_t* tstart,
                       const int32_t* tlen, int n_tiles, const void* B, int N, const float* scale,
                       const int32_t* o_idx, int mode, int tm, void* Y, hipStream_t s) {
  if (n_tiles == 0) return hipSuccess;
  if (K % 32 != 0 || N % 16 != 0 || K > 1024 || N <= 0 || tm % 16 != 0 || tm < 16 || tm > RG_TM)
    return hipErrorInvalidValue;
  const size_t lds = eh_rel_gemm_lds(K, N, mode, tm);
  if (lds > 160 * 1024 - 2048) return hipErrorInvalidValue;
  EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(rel_gemm_kernel),
                                      hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  hipLaunchKernelGGL(rel_gemm_kernel, dim3(n_tiles), dim3(256), lds, s, static_cast<const bf16_t*>(A), K, a_idx, trel,
                     tstart, tlen, static_cast<const bf16_t*>(B), N, scale, o_idx, mode, tm, Y);
  return hipGetLastError();
}

hipError_t eh_rel_gemm_dw(const void* G, int N, const int32_t* g_idx, const void* X, int K, const int32_t* x_idx,
                          const float* scale, const int32_t* crel, const int32_t* cstart, const int32_t* clen,
                          const int32_t* csolo, int n_chunks, float* dW, int accum, hipStream_t s,
                          const int32_t* cslot, float* part, const int32_t* mrel, const int32_t* mrp, int n_multi) {
  if (n_chunks == 0) return hipSuccess;
  if (N % 64 != 0 || K % 64 != 0) return hipErrorInvalidValue;
  static const int t_max = [] {  // EULER_AMD_RG_DW_T=64: 64 x 64 slabs only (tuning knob)
    const char* e = std::getenv("EULER_AMD_RG_DW_T");
    return e ? std::atoi(e) : 128;
  }();
  const int T = (t_max >= 128 && N % 128 == 0 && K % 128 == 0) ? 128 : 64;
  const int64_t blocks = static_cast<int64_t>(n_chunks) * (N / T) * (K / T);
  if (blocks >= (1ll << 31)) return hipErrorInvalidValue;
  if (cslot && (!csolo || !part || !mrel || !mrp)) return hipErrorInvalidValue;
  if (T == 128)
    hipLaunchKernelGGL(rel_gemm_dw_kernel<128>, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s,
                       static_cast<const bf16_t*>(G), N, g_idx, static_cast<const bf16_t*>(X), K, x_idx, scale, crel,
                       cstart, clen, csolo, dW, accum, cslot, part);
  else
    hipLaunchKernelGGL(rel_gemm_dw_kernel<64>, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s,
                       static_cast<const bf16_t*>(G), N, g_idx, static_cast<const bf16_t*>(X), K, x_idx, scale, crel,
                       cstart, clen, csolo, dW, accum, cslot, part);
  if (cslot && n_multi > 0) {
    const int64_t NK = static_cast<int64_t>(N) * K;
    const int64_t items = static_cast<int64_t>(n_multi) * (NK >> 2);
    const uint32_t g = static_cast<uint32_t>(std::min<int64_t>((items + 255) / 256, 4096));
    hipLaunchKernelGGL(rel_dw_reduce_kernel, dim3(g), dim3(256), 0, s, part, mrel, mrp, n_multi, NK, dW, accum);
  }
  return hipGetLastError();
}

int eh_rel_gemm_dw_chunk() { return RG_CH; }

hipError_t eh_rel_weight_bf16(const float* W, int64_t R, int N, int K, void* wb, void* wt, hipStream_t s) {
  if (R <= 0) return hipSuccess;
  if (N % 64 != 0 || K % 64 != 0) return hipErrorInvalidValue;
  const int64_t blocks = R * (N / 64) * (K / 64);
  if (blocks >= (1ll << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rel_weight_bf16_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s, W, N, K,
                     static_cast<bf16_t*>(wb), static_cast<bf16_t*>(wt));
  return hipGetLastError();
}

}  // extern "C"
