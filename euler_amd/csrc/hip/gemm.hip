// Tiled MFMA GEMM for the skinny products of the model code around the fused kernels
// (unsupervised GraphSAGE tower heads, the R-GCN self-loop, ...): hipBLASLt picks one
// 256 x 128 tile for an [6144 x 256] x [256 x 128] product (24 workgroups, 34 us on
// MI355X, profiles/r3_unsup/); here 64 x 64 tiles, bf16 MFMA with fp32 accumulation, the
// next k-step's operands loaded into registers while the current one runs, fused
// epilogues, and split-K (deterministic partial slabs + one reduce) for the [R]-row
// reductions of weight gradients.
//
//   C[M][N] = rscale[M] * (op(A) op(B)) (+ bias[N]) (+ Add[M][N]) (relu) (* relu'(Rm[M][N]))
//   A: a_t = 0: [M][K] row-major (lda);  a_t = 1: [K][M] (lda)  -> op(A) = A or A^T
//   B: b_t = 0: [N][K] (ldb) (C = A B^T, "NT");  b_t = 1: [K][N] (ldb) ("NN")
//   A, B fp32 or bf16 (staged in LDS as bf16); C fp32 or bf16 (ldc); Rm bf16 or fp32
//   splits > 1: grid.z splits the K range; partial slabs [splits][M][N] fp32 in `part`,
//   then gemm_reduce sums them into C with the epilogue.
#include "hip/common.h"
#include "hip/launchers.h"
#include "hip/tile.h"

namespace euler_hip {

constexpr int kGmT = 64, kGmK = 64, kGmLd = kGmK + 8;  // tile, k step, LDS row (bf16, +16 B pad)

struct GemmArgs {
  const void* A;
  const void* B;
  void* C;
  const float* bias;   // [N] or null
  const void* rmask;   // [M][N] (ldr): multiply by relu'(rmask) (rmask > 0), or null
  float* part;         // split-K slabs [splits][M][N]
  int64_t M, N, K;
  int64_t lda, ldb, ldc, ldr;
  int32_t a_t, b_t, a_bf16, b_bf16, c_bf16, r_bf16;
  int32_t relu, splits, kps;  // kps: k per split (multiple of kGmK)
  float alpha;
  const void* addend;  // [M][N] (ld_add) added before relu / rmask, or null (may alias C)
  int64_t ld_add;
  int32_t add_bf16;
  const float* rscale;  // [M]: the product row r is scaled by rscale[r] before bias / addend
};

__device__ __forceinline__ float gm_addend(const GemmArgs& a, int64_t row, int64_t col) {
  return a.add_bf16 ? bf2f(static_cast<const bf16_t*>(a.addend)[row * a.ld_add + col])
                    : static_cast<const float*>(a.addend)[row * a.ld_add + col];
}

// 8 consecutive k of row r of op(X) (X [rows][k] if !t, [k][rows] if t) -> 8 floats;
// out-of-range elements read 0
__device__ __forceinline__ void gm_load8(const void* X, int bf, int t, int64_t ld, int64_t rows, int64_t K,
                                         int64_t r, int64_t k0, float* v) {
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = 0.f;
  if (r >= rows) return;
  if (!t) {
    if (k0 + 8 <= K && ((ld | k0) & 7) == 0) {  // one (or two) vector loads
      if (bf) {
        const uint4_t q = *reinterpret_cast<const uint4_t*>(static_cast<const bf16_t*>(X) + r * ld + k0);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[2 * j] = bf2f(static_cast<bf16_t>(q[j] & 0xffffu));
          v[2 * j + 1] = bf2f(static_cast<bf16_t>(q[j] >> 16));
        }
      } else {
        const float4_t a = *reinterpret_cast<const float4_t*>(static_cast<const float*>(X) + r * ld + k0);
        const float4_t b = *reinterpret_cast<const float4_t*>(static_cast<const float*>(X) + r * ld + k0 + 4);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[j] = a[j];
          v[4 + j] = b[j];
        }
      }
      return;
    }
#pragma unroll
    for (int j = 0; j < 8; ++j)
      if (k0 + j < K) v[j] = bf ? bf2f(static_cast<const bf16_t*>(X)[r * ld + k0 + j]) : static_cast<const float*>(X)[r * ld + k0 + j];
    return;
  }
#pragma unroll
  for (int j = 0; j < 8; ++j)
    if (k0 + j < K) v[j] = bf ? bf2f(static_cast<const bf16_t*>(X)[(k0 + j) * ld + r]) : static_cast<const float*>(X)[(k0 + j) * ld + r];
}

// one 64 x 64 output tile (a K range for split-K); 4 waves, wave w: rows (w >> 1) * 32,
// columns (w & 1) * 32 as 2 x 2 MFMA tiles, two 32-deep MFMA k-steps per 64-deep stage.
// Operand staging: thread t owns row t >> 2, k chunk (t & 3) * 16 of both the A and the B
// tile (4 x 8 values in flight per thread and stage).
__global__ __launch_bounds__(256) void gemm_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t As[2][kGmT * kGmLd];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][kGmT * kGmLd];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t m0 = static_cast<int64_t>(blockIdx.x) * kGmT, n0 = static_cast<int64_t>(blockIdx.y) * kGmT;
  const int split = blockIdx.z;
  const int64_t kb = static_cast<int64_t>(split) * a.kps;
  const int64_t ke = kb + a.kps < a.K ? kb + a.kps : a.K;
  const int sr = tid >> 2, sk = (tid & 3) * 16;
  float va[16], vb[16];
  auto fetch = [&](int64_t k0) {
    gm_load8(a.A, a.a_bf16, a.a_t, a.lda, a.M, ke, m0 + sr, k0 + sk, va);
    gm_load8(a.A, a.a_bf16, a.a_t, a.lda, a.M, ke, m0 + sr, k0 + sk + 8, va + 8);
    gm_load8(a.B, a.b_bf16, a.b_t, a.ldb, a.N, ke, n0 + sr, k0 + sk, vb);
    gm_load8(a.B, a.b_bf16, a.b_t, a.ldb, a.N, ke, n0 + sr, k0 + sk + 8, vb + 8);
  };
  auto stage = [&](int buf) {
    *reinterpret_cast<uint4_t*>(&As[buf][sr * kGmLd + sk]) = pack_bf16x8(va);
    *reinterpret_cast<uint4_t*>(&As[buf][sr * kGmLd + sk + 8]) = pack_bf16x8(va + 8);
    *reinterpret_cast<uint4_t*>(&Bs[buf][sr * kGmLd + sk]) = pack_bf16x8(vb);
    *reinterpret_cast<uint4_t*>(&Bs[buf][sr * kGmLd + sk + 8]) = pack_bf16x8(vb + 8);
  };
  float4_t acc[2][2];
  tl_zero(acc);
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  if (kb < ke) {
    fetch(kb);
    stage(0);
    __syncthreads();
    int buf = 0;
    for (int64_t k0 = kb; k0 < ke; k0 += kGmK) {
      const bool more = k0 + kGmK < ke;
      if (more) fetch(k0 + kGmK);  // next k step in flight during this one's MFMAs
#pragma unroll
      for (int ks = 0; ks < kGmK; ks += 32) {
        uint4_t fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          fa[i] = *reinterpret_cast<const uint4_t*>(&As[buf][(wr + i * 16 + lr) * kGmLd + ks + lk]);
          fb[i] = *reinterpret_cast<const uint4_t*>(&Bs[buf][(wc + i * 16 + lr) * kGmLd + ks + lk]);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
      }
      if (more) {
        stage(buf ^ 1);
        __syncthreads();
        buf ^= 1;
      }
    }
  }
  // epilogue: C/D lane map col = lane & 15, row = (lane >> 4) * 4 + j
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wc + j * 16 + lr;
      if (col >= a.N) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = m0 + wr + i * 16 + (lane >> 4) * 4 + q;
        if (row >= a.M) continue;
        float v = acc[i][j][q] * a.alpha;
        if (a.splits > 1) {
          a.part[(static_cast<int64_t>(split) * a.M + row) * a.N + col] = v;
          continue;
        }
        if (a.rscale) v *= a.rscale[row];
        if (a.bias) v += a.bias[col];
        if (a.addend) v += gm_addend(a, row, col);
        if (a.relu) v = fmaxf(v, 0.f);
        if (a.rmask) {
          const float rv = a.r_bf16 ? bf2f(static_cast<const bf16_t*>(a.rmask)[row * a.ldr + col])
                                    : static_cast<const float*>(a.rmask)[row * a.ldr + col];
          if (!(rv > 0.f)) v = 0.f;
        }
        if (a.c_bf16) static_cast<bf16_t*>(a.C)[row * a.ldc + col] = f2bf(v);
        else static_cast<float*>(a.C)[row * a.ldc + col] = v;
      }
    }
}

// C = alpha A^T B for k-major operands (A [K][M], B [K][N], row-major: the weight gradients
// dW = dY^T X of row-batched layers): 64-row k sub-tiles of both operands are staged in LDS
// as they lie in memory ([k][64 columns], contiguous 16-value row segments per thread, fp32
// rounded to bf16 on the way) and the MFMA fragments come out of the gfx950 transposing
// read (tl_tr_frag) — the generic kernel's transposed path loads every operand element
// with its own strided scalar load.  Split-K over grid.z (kps rows per split) into the
// partial slabs, summed by gemm_reduce_kernel.
constexpr int kTnLd = kGmT + 16;  // LDS row (halfwords): 40 dwords, conflict-free tr reads

__device__ __forceinline__ void tn_load16(const void* X, int bf, int64_t ld, int64_t rows, int64_t cols, int64_t k,
                                          int64_t c, float* v) {
#pragma unroll
  for (int j = 0; j < 16; ++j) v[j] = 0.f;
  if (k >= rows) return;
  if (c + 16 <= cols && (ld & 7) == 0 && (c & 7) == 0 && (reinterpret_cast<uintptr_t>(X) & 31) == 0) {
    if (bf) {
      const bf16_t* p = static_cast<const bf16_t*>(X) + k * ld + c;
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        const uint4_t q = *reinterpret_cast<const uint4_t*>(p + 8 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          v[8 * h + 2 * j] = bf2f(static_cast<bf16_t>(q[j] & 0xffffu));
          v[8 * h + 2 * j + 1] = bf2f(static_cast<bf16_t>(q[j] >> 16));
        }
      }
    } else {
      const float* p = static_cast<const float*>(X) + k * ld + c;
#pragma unroll
      for (int h = 0; h < 4; ++h) {
        const float4_t f = *reinterpret_cast<const float4_t*>(p + 4 * h);
#pragma unroll
        for (int j = 0; j < 4; ++j) v[4 * h + j] = f[j];
      }
    }
    return;
  }
  for (int j = 0; j < 16; ++j)
    if (c + j < cols)
      v[j] = bf ? bf2f(static_cast<const bf16_t*>(X)[k * ld + c + j]) : static_cast<const float*>(X)[k * ld + c + j];
}

__global__ __launch_bounds__(256) void gemm_tn_kernel(GemmArgs a) {
  __shared__ __attribute__((aligned(16))) bf16_t As[2][kGmK * kTnLd];
  __shared__ __attribute__((aligned(16))) bf16_t Bs[2][kGmK * kTnLd];
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int64_t m0 = static_cast<int64_t>(blockIdx.x) * kGmT, n0 = static_cast<int64_t>(blockIdx.y) * kGmT;
  const int split = blockIdx.z;
  const int64_t kb = static_cast<int64_t>(split) * a.kps;
  const int64_t ke = kb + a.kps < a.K ? kb + a.kps : a.K;
  const int sr = tid >> 2, sc = (tid & 3) * 16;  // staged k row, 16-column segment
  float va[16], vb[16];
  auto fetch = [&](int64_t k0) {
    tn_load16(a.A, a.a_bf16, a.lda, ke, a.M, k0 + sr, m0 + sc, va);
    tn_load16(a.B, a.b_bf16, a.ldb, ke, a.N, k0 + sr, n0 + sc, vb);
  };
  auto stage = [&](int buf) {
    *reinterpret_cast<uint4_t*>(&As[buf][sr * kTnLd + sc]) = pack_bf16x8(va);
    *reinterpret_cast<uint4_t*>(&As[buf][sr * kTnLd + sc + 8]) = pack_bf16x8(va + 8);
    *reinterpret_cast<uint4_t*>(&Bs[buf][sr * kTnLd + sc]) = pack_bf16x8(vb);
    *reinterpret_cast<uint4_t*>(&Bs[buf][sr * kTnLd + sc + 8]) = pack_bf16x8(vb + 8);
  };
  float4_t acc[2][2];
  tl_zero(acc);
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  if (kb < ke) {
    fetch(kb);
    stage(0);
    __syncthreads();
    int buf = 0;
    for (int64_t k0 = kb; k0 < ke; k0 += kGmK) {
      const bool more = k0 + kGmK < ke;
      if (more) fetch(k0 + kGmK);
#pragma unroll
      for (int ks = 0; ks < kGmK; ks += 32) {
        uint4_t fa[2], fb[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) {
          fa[i] = tl_tr_frag<kTnLd>(As[buf], ks, wr + i * 16, lane);
          fb[i] = tl_tr_frag<kTnLd>(Bs[buf], ks, wc + i * 16, lane);
        }
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 2; ++j) acc[i][j] = mfma16(fa[i], fb[j], acc[i][j]);
      }
      if (more) {
        stage(buf ^ 1);  // buf ^ 1 was last read before the previous step's barrier
        __syncthreads();
        buf ^= 1;
      }
    }
  }
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int64_t col = n0 + wc + j * 16 + (lane & 15);
      if (col >= a.N) continue;
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int64_t row = m0 + wr + i * 16 + (lane >> 4) * 4 + q;
        if (row >= a.M) continue;
        float v = acc[i][j][q] * a.alpha;
        if (a.splits > 1) {
          a.part[(static_cast<int64_t>(split) * a.M + row) * a.N + col] = v;
          continue;
        }
        if (a.rscale) v *= a.rscale[row];
        if (a.addend) v += gm_addend(a, row, col);
        if (a.c_bf16) static_cast<bf16_t*>(a.C)[row * a.ldc + col] = f2bf(v);
        else static_cast<float*>(a.C)[row * a.ldc + col] = v;
      }
    }
}

// sum of the split-K slabs + the epilogue
__global__ __launch_bounds__(256) void gemm_reduce_kernel(GemmArgs a) {

  grid_stride(a.M * a.N, [&](int64_t i) {
    const int64_t row = i / a.N, col = i - row * a.N;
    float v = 0.f;
    const int64_t MN = a.M * a.N;
    int s = 0;
    for (; s + 8 <= a.splits; s += 8) {  // 8 slab loads in flight
      float t[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) t[u] = a.part[(s + u) * MN + i];
#pragma unroll
      for (int u = 0; u < 8; ++u) v += t[u];
    }
    for (; s < a.splits; ++s) v += a.part[s * MN + i];
    if (a.rscale) v *= a.rscale[row];
    if (a.bias) v += a.bias[col];
    if (a.addend) v += gm_addend(a, row, col);
    if (a.relu) v = fmaxf(v, 0.f);
    if (a.rmask) {
      const float rv = a.r_bf16 ? bf2f(static_cast<const bf16_t*>(a.rmask)[row * a.ldr + col])
                                : static_cast<const float*>(a.rmask)[row * a.ldr + col];
      if (!(rv > 0.f)) v = 0.f;
    }
    if (a.c_bf16) static_cast<bf16_t*>(a.C)[row * a.ldc + col] = f2bf(v);
    else static_cast<float*>(a.C)[row * a.ldc + col] = v;
  });
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

hipError_t eh_gemm(const void* A, const void* B, void* C, const float* bias, const void* rmask, float* part,
                   int64_t M, int64_t N, int64_t K, int64_t lda, int64_t ldb, int64_t ldc, int64_t ldr, int a_t,
                   int b_t, int a_bf16, int b_bf16, int c_bf16, int r_bf16, int relu, int splits, float alpha,
                   const void* addend, int64_t ld_add, int add_bf16, const float* rscale, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1 || (splits > 1 && !part)) return hipErrorInvalidValue;
  GemmArgs g{A, B, C, bias, rmask, part, M, N, K, lda, ldb, ldc, ldr, a_t, b_t, a_bf16, b_bf16, c_bf16, r_bf16,
             relu, splits, 0, alpha, addend, ld_add, add_bf16, rscale};
  const int64_t ksteps = ceil_div(K, kGmK);
  g.kps = static_cast<int32_t>(ceil_div(ksteps, splits) * kGmK);
  const dim3 grid(static_cast<uint32_t>(ceil_div(M, kGmT)), static_cast<uint32_t>(ceil_div(N, kGmT)),
                  static_cast<uint32_t>(splits));
  hipLaunchKernelGGL(gemm_kernel, grid, dim3(256), 0, s, g);
  if (splits > 1)
    hipLaunchKernelGGL(gemm_reduce_kernel, grid_for(M * N), dim3(256), 0, s, g);
  return hipGetLastError();
}

// C [M][N] = alpha A^T B, A [K][M] (lda), B [K][N] (ldb), split over K in `splits` slabs
hipError_t eh_gemm_tn(const void* A, const void* B, void* C, float* part, int64_t M, int64_t N, int64_t K, int64_t lda,
                      int64_t ldb, int64_t ldc, int a_bf16, int b_bf16, int c_bf16, int splits, float alpha,
                      const void* addend, int64_t ld_add, int add_bf16, const float* rscale, hipStream_t s) {
  if (M <= 0 || N <= 0 || K <= 0 || splits < 1 || (splits > 1 && !part)) return hipErrorInvalidValue;
  GemmArgs g{A, B, C, nullptr, nullptr, part, M, N, K, lda, ldb, ldc, 0, 1, 1, a_bf16, b_bf16, c_bf16, 0,
             0, splits, 0, alpha, addend, ld_add, add_bf16, rscale};
  const int64_t ksteps = ceil_div(K, kGmK);
  g.kps = static_cast<int32_t>(ceil_div(ksteps, splits) * kGmK);
  const dim3 grid(static_cast<uint32_t>(ceil_div(M, kGmT)), static_cast<uint32_t>(ceil_div(N, kGmT)),
                  static_cast<uint32_t>(splits));
  hipLaunchKernelGGL(gemm_tn_kernel, grid, dim3(256), 0, s, g);
  if (splits > 1)
    hipLaunchKernelGGL(gemm_reduce_kernel, grid_for(M * N), dim3(256), 0, s, g);
  return hipGetLastError();
}

}  // extern "C"
