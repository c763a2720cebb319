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
//   rel_gemm_dw : dW[rel] += sum_e (scale[e] * G[g_idx[e]])^T X[x_idx[e]]  (per-tile
//                 outer-product GEMM over the 64 edges, fp32 atomics into [R][N][K])
#include "hip/common.h"
#include "hip/launchers.h"

namespace euler_hip {

typedef __bf16 rg_bf16x8 __attribute__((ext_vector_type(8)));

__device__ __forceinline__ float4_t rg_mfma(uint4_t a, uint4_t b, float4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(rg_bf16x8, a), __builtin_bit_cast(rg_bf16x8, b),
                                                 c, 0, 0, 0);
}

constexpr int RG_BM = 64;  // edges per tile

__global__ __launch_bounds__(256) void rel_gemm_kernel(const bf16_t* __restrict__ A, int K,
                                                       const int32_t* __restrict__ a_idx,
                                                       const int32_t* __restrict__ trel,
                                                       const int32_t* __restrict__ tstart,
                                                       const int32_t* __restrict__ tlen, const bf16_t* __restrict__ B,
                                                       int N, const float* __restrict__ scale,
                                                       const int32_t* __restrict__ o_idx, int mode, void* Y) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int t = xcd_remap(blockIdx.x, gridDim.x);
  const int r = trel[t], e0 = tstart[t], ne = tlen[t];
  const int ldk = K + 8;
  const int cpr = K >> 3;
  // prologue: gather the tile's A rows (zero rows past the tile / for padding ids)
  for (int it = threadIdx.x; it < RG_BM * cpr; it += 256) {
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
  bf16_t* otile = lds + RG_BM * ldk;  // mode 0 output tile [64][N + 8]
  // epilogue bookkeeping for the 16 rows this lane owns in C (row = m*16 + (lane>>4)*4 + j)
  int64_t orow[4][4];
  float osc[4][4];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int row = m * 16 + (lane >> 4) * 4 + j;
      orow[m][j] = row < ne ? static_cast<int64_t>(o_idx[e0 + row]) : -1;
      osc[m][j] = (row < ne && scale) ? scale[e0 + row] : 1.f;
    }
  for (int n0 = wave * 16; n0 < N; n0 += 64) {
    float4_t acc[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) acc[m] = float4_t{0.f, 0.f, 0.f, 0.f};
    uint4_t b = *reinterpret_cast<const uint4_t*>(Br + static_cast<int64_t>(n0 + lr) * K + lk);
    for (int k0 = 0; k0 < K; k0 += 32) {
      const bool more = k0 + 32 < K;
      const uint4_t bn = more ? *reinterpret_cast<const uint4_t*>(Br + static_cast<int64_t>(n0 + lr) * K + k0 + 32 + lk)
                              : uint4_t{0u, 0u, 0u, 0u};
      uint4_t a[4];
#pragma unroll
      for (int m = 0; m < 4; ++m) a[m] = *reinterpret_cast<const uint4_t*>(lds + (m * 16 + lr) * ldk + k0 + lk);
#pragma unroll
      for (int m = 0; m < 4; ++m) acc[m] = rg_mfma(a[m], b, acc[m]);
      b = bn;
    }
    const int col = n0 + lr;
    if (mode == 0) {
      // stage the bf16 tile in LDS; rows leave as 16-byte stores below
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int row = m * 16 + (lane >> 4) * 4 + j;
          otile[row * ldn + col] = f2bf(acc[m][j] * osc[m][j]);
        }
    } else {
#pragma unroll
      for (int m = 0; m < 4; ++m)
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t o = orow[m][j];
          if (o >= 0) atomicAdd(static_cast<float*>(Y) + o * N + col, acc[m][j] * osc[m][j]);
        }
    }
  }
  if (mode == 0) {
    __syncthreads();
    const int cpn = N >> 3;
    for (int it = threadIdx.x; it < ne * cpn; it += 256) {
      const int row = it / cpn, c = it - row * cpn;
      const int64_t o = o_idx[e0 + row];
      if (o >= 0)
        *reinterpret_cast<uint4_t*>(static_cast<bf16_t*>(Y) + o * N + c * 8) =
            *reinterpret_cast<const uint4_t*>(otile + row * ldn + c * 8);
    }
  }
}

// dW for one (chunk of <= RG_CH edges of ONE relation, 64 x 64 slab of dW[rel]) per workgroup:
// the chunk's 64-edge sub-tiles are staged transposed in LDS and accumulated in registers
// (wave w: slab rows w*16..+16, four 16-column fragments), so each dW element receives one
// atomic per chunk instead of one per 64-edge tile (the atomics were the dW kernel's floor).
constexpr int RG_CH = 1024;  // edges per dW chunk

__global__ __launch_bounds__(256) void rel_gemm_dw_kernel(const bf16_t* __restrict__ G, int N,
                                                          const int32_t* __restrict__ g_idx,
                                                          const bf16_t* __restrict__ X, int K,
                                                          const int32_t* __restrict__ x_idx,
                                                          const float* __restrict__ scale,
                                                          const int32_t* __restrict__ crel,
                                                          const int32_t* __restrict__ cstart,
                                                          const int32_t* __restrict__ clen, float* __restrict__ dW) {
  constexpr int LDT = RG_BM + 8;  // transposed tiles: [col][edge], 144-byte rows
  __shared__ __attribute__((aligned(16))) bf16_t gT[64 * LDT];
  __shared__ __attribute__((aligned(16))) bf16_t xT[64 * LDT];
  const int SN = N >> 6, SK = K >> 6;
  const int b = xcd_remap(blockIdx.x, gridDim.x);
  const int chunk = b / (SN * SK), s = b - chunk * (SN * SK);
  const int sn = s / SK, sk = s - sn * SK;
  const int r = crel[chunk], c0 = cstart[chunk], clen_ = clen[chunk];
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  float4_t acc[4];
#pragma unroll
  for (int f = 0; f < 4; ++f) acc[f] = float4_t{0.f, 0.f, 0.f, 0.f};
  // item = (edge e = it & 63, 8-column chunk c = it >> 6): the 64 lanes of a wave take 64
  // consecutive edges of one chunk, so the transposed LDS writes hit consecutive bytes
  // (no bank conflicts); 2 items per thread and operand.  The next sub-tile's rows are
  // loaded into registers while the MFMAs of the current one run.
  uint4_t gv[2], xv[2];
  float gs[2];
  auto prefetch = [&](int sub) {
    const int ne = min(RG_BM, clen_ - sub);
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int it = threadIdx.x + h * 256;
      const int e = it & 63, c = it >> 6;
      gv[h] = uint4_t{0u, 0u, 0u, 0u};
      xv[h] = uint4_t{0u, 0u, 0u, 0u};
      gs[h] = 0.f;
      if (e < ne) {
        const int64_t gi = g_idx[c0 + sub + e];
        const int64_t xi = x_idx[c0 + sub + e];
        if (gi >= 0) {
          gv[h] = *reinterpret_cast<const uint4_t*>(G + gi * N + sn * 64 + c * 8);
          gs[h] = scale ? scale[c0 + sub + e] : 1.f;
        }
        if (xi >= 0) xv[h] = *reinterpret_cast<const uint4_t*>(X + xi * K + sk * 64 + c * 8);
      }
    }
  };
  prefetch(0);
  for (int sub = 0; sub < clen_; sub += RG_BM) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int it = threadIdx.x + h * 256;
      const int e = it & 63, c = it >> 6;
      float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      acc_bf16x8(v, gv[h], gs[h]);
#pragma unroll
      for (int q = 0; q < 8; ++q) gT[(c * 8 + q) * LDT + e] = f2bf(v[q]);
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        xT[(c * 8 + 2 * q) * LDT + e] = static_cast<bf16_t>(xv[h][q] & 0xffffu);
        xT[(c * 8 + 2 * q + 1) * LDT + e] = static_cast<bf16_t>(xv[h][q] >> 16);
      }
    }
    __syncthreads();
    if (sub + RG_BM < clen_) prefetch(sub + RG_BM);
#pragma unroll
    for (int k0 = 0; k0 < RG_BM; k0 += 32) {
      const uint4_t a = *reinterpret_cast<const uint4_t*>(gT + (wave * 16 + lr) * LDT + k0 + lk);
#pragma unroll
      for (int f = 0; f < 4; ++f) {
        const uint4_t bb = *reinterpret_cast<const uint4_t*>(xT + (f * 16 + lr) * LDT + k0 + lk);
        acc[f] = rg_mfma(a, bb, acc[f]);
      }
    }
    __syncthreads();
  }
  float* __restrict__ dWr = dW + static_cast<int64_t>(r) * N * K;
#pragma unroll
  for (int f = 0; f < 4; ++f)
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int n = sn * 64 + wave * 16 + (lane >> 4) * 4 + j;
      atomicAdd(dWr + static_cast<int64_t>(n) * K + sk * 64 + f * 16 + lr, acc[f][j]);
    }
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

size_t eh_rel_gemm_lds(int K, int N, int mode) {
  return static_cast<size_t>(RG_BM) * ((K + 8) + (mode == 0 ? N + 8 : 0)) * sizeof(bf16_t);
}

hipError_t eh_rel_gemm(const void* A, int K, const int32_t* a_idx, const int32_t* trel, const int32_t* tstart,
                       const int32_t* tlen, int n_tiles, const void* B, int N, const float* scale,
                       const int32_t* o_idx, int mode, void* Y, hipStream_t s) {
  if (n_tiles == 0) return hipSuccess;
  if (K % 32 != 0 || N % 16 != 0 || K > 1024 || N <= 0) return hipErrorInvalidValue;
  const size_t lds = eh_rel_gemm_lds(K, N, mode);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rel_gemm_kernel, dim3(n_tiles), dim3(256), lds, s, static_cast<const bf16_t*>(A), K, a_idx, trel,
                     tstart, tlen, static_cast<const bf16_t*>(B), N, scale, o_idx, mode, Y);
  return hipGetLastError();
}

hipError_t eh_rel_gemm_dw(const void* G, int N, const int32_t* g_idx, const void* X, int K, const int32_t* x_idx,
                          const float* scale, const int32_t* crel, const int32_t* cstart, const int32_t* clen,
                          int n_chunks, float* dW, hipStream_t s) {
  if (n_chunks == 0) return hipSuccess;
  if (N % 64 != 0 || K % 64 != 0) return hipErrorInvalidValue;
  const int64_t blocks = static_cast<int64_t>(n_chunks) * (N / 64) * (K / 64);
  if (blocks >= (1ll << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(rel_gemm_dw_kernel, dim3(static_cast<uint32_t>(blocks)), dim3(256), 0, s,
                     static_cast<const bf16_t*>(G), N, g_idx, static_cast<const bf16_t*>(X), K, x_idx, scale, crel,
                     cstart, clen, dW);
  return hipGetLastError();
}

int eh_rel_gemm_dw_chunk() { return RG_CH; }

}  // extern "C"
