// Fused GraphSAGE / GCN-style layer for fixed-fanout neighbor tiles.
//
//   A[m]   = [ x[self[m]] | (sum_k x[nbr[m,k]] + include_self * x[self[m]]) * inv_cnt ]   (bf16, [M, 2D])
//   out[m] = act( A[m] @ W^T + bias )                                                    (bf16, [M, H])
//
// W is stored as torch.nn.Linear stores it, [H, 2D] (= [W_self | W_neigh]), which is
// exactly the k-contiguous B-operand layout of v_mfma_f32_16x16x32_bf16, so B
// fragments are single 16-byte loads straight from L2 (W is shared by all blocks).
//
// One workgroup = 4 waves = 64 target rows.  Phase 1 gathers the neighbor rows with
// 16-byte loads (all fanout loads in flight per lane), reduces in fp32 and writes the
// bf16 A tile into LDS (row stride padded by 16 B: conflict-free ds_read_b128 for the
// A fragments) and, optionally, to HBM for the backward pass.  Phase 2 runs the MFMA
// GEMM out of LDS; each wave owns a 64-column slab and loops over the column chunks,
// so the gathered tile is reused for every output chunk.
//
// Reference semantics: SAGEConv = self_fc(x) + neigh_fc(scatter_mean(gather(x)))
// (reference tf_euler/python/convolution/sage_conv.py:33-44) with the self-loop edges
// UniqueDataFlow adds (tf_euler/python/dataflow/neighbor_dataflow.py:84-110).
#include "hip/common.h"

namespace euler_hip {

typedef __bf16 bf16x8_t __attribute__((ext_vector_type(8)));

__device__ __forceinline__ bf16x8_t as_bf16x8(uint4_t v) { return __builtin_bit_cast(bf16x8_t, v); }

constexpr int SAGE_BM = 64;
constexpr int SAGE_THREADS = 256;

// ---------------------------------------------------------------------------
// phase 1: gather + mean into the LDS A tile (and optionally HBM)
// ---------------------------------------------------------------------------
__device__ __forceinline__ void sage_gather_tile(const bf16_t* __restrict__ x, int D,
                                                 const int32_t* __restrict__ self_idx,
                                                 const int32_t* __restrict__ nbr_idx, int F, int include_self,
                                                 float inv_cnt, int64_t M, int64_t row0, bf16_t* lds, int ldsw,
                                                 bf16_t* __restrict__ a_save) {
  const int cpr = D >> 3;  // 16-byte chunks per half-row
  const int items = SAGE_BM * cpr;
  const int K2 = 2 * D;
  for (int it = threadIdx.x; it < items; it += SAGE_THREADS) {
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
      const int32_t* nb = nbr_idx + grow * F;
      int k = 0;
      for (; k + 8 <= F; k += 8) {
        int32_t j[8];
        uint4_t v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) j[u] = nb[k + u];
#pragma unroll
        for (int u = 0; u < 8; ++u)
          v[u] = j[u] >= 0 ? *reinterpret_cast<const uint4_t*>(x + static_cast<int64_t>(j[u]) * D + c * 8)
                           : uint4_t{0u, 0u, 0u, 0u};
#pragma unroll
        for (int u = 0; u < 8; ++u) acc_bf16x8(acc, v[u]);
      }
      for (; k < F; ++k) {
        const int32_t j = nb[k];
        if (j >= 0) acc_bf16x8(acc, *reinterpret_cast<const uint4_t*>(x + static_cast<int64_t>(j) * D + c * 8));
      }
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) acc[i] *= inv_cnt;
    const uint4_t mv = pack_bf16x8(acc);
    *reinterpret_cast<uint4_t*>(lds + r * ldsw + c * 8) = sv;
    *reinterpret_cast<uint4_t*>(lds + r * ldsw + D + c * 8) = mv;
    if (a_save && grow < M) {
      *reinterpret_cast<uint4_t*>(a_save + grow * K2 + c * 8) = sv;
      *reinterpret_cast<uint4_t*>(a_save + grow * K2 + D + c * 8) = mv;
    }
  }
}

// ---------------------------------------------------------------------------
// phase 2: out[rows, :] = act(A_lds @ W^T + b) with v_mfma_f32_16x16x32_bf16
// ---------------------------------------------------------------------------
template <int BN>
__device__ __forceinline__ void sage_gemm_tile(const bf16_t* lds, int ldsw, int K2, const bf16_t* __restrict__ W,
                                               const float* __restrict__ bias, int H, int64_t M, int64_t row0,
                                               int relu, bf16_t* __restrict__ out) {
  constexpr int WN = BN / 64;      // waves along N
  constexpr int WM = 4 / WN;       // waves along M
  constexpr int RW = SAGE_BM / WM; // rows per wave
  constexpr int FM = RW / 16;      // 16-row fragments per wave
  constexpr int FN = 4;            // 16-col fragments per wave (64 columns)
  const int wave = threadIdx.x >> 6;
  const int lane = threadIdx.x & 63;
  const int wm = wave / WN, wn = wave % WN;
  const int lr = lane & 15, lk = (lane >> 4) * 8;
  for (int cchunk = 0; cchunk < H; cchunk += BN) {
    const int cb = cchunk + wn * 64;
    if (cb >= H) continue;  // wave-uniform
    float4_t acc[FM][FN];
#pragma unroll
    for (int m = 0; m < FM; ++m)
#pragma unroll
      for (int n = 0; n < FN; ++n) acc[m][n] = float4_t{0.f, 0.f, 0.f, 0.f};
    const bf16_t* wrow[FN];
    bool wok[FN];
#pragma unroll
    for (int n = 0; n < FN; ++n) {
      const int col = cb + n * 16 + lr;
      wok[n] = col < H;
      wrow[n] = W + static_cast<int64_t>(wok[n] ? col : 0) * K2 + lk;
    }
    uint4_t bcur[FN];
#pragma unroll
    for (int n = 0; n < FN; ++n)
      bcur[n] = wok[n] ? *reinterpret_cast<const uint4_t*>(wrow[n]) : uint4_t{0u, 0u, 0u, 0u};
    for (int k0 = 0; k0 < K2; k0 += 32) {
      uint4_t bnext[FN];
      const bool more = k0 + 32 < K2;
#pragma unroll
      for (int n = 0; n < FN; ++n)
        bnext[n] = (more && wok[n]) ? *reinterpret_cast<const uint4_t*>(wrow[n] + k0 + 32)
                                    : uint4_t{0u, 0u, 0u, 0u};
      uint4_t a[FM];
#pragma unroll
      for (int m = 0; m < FM; ++m)
        a[m] = *reinterpret_cast<const uint4_t*>(lds + (wm * RW + m * 16 + lr) * ldsw + k0 + lk);
#pragma unroll
      for (int m = 0; m < FM; ++m)
#pragma unroll
        for (int n = 0; n < FN; ++n)
          acc[m][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(as_bf16x8(a[m]), as_bf16x8(bcur[n]), acc[m][n], 0, 0, 0);
#pragma unroll
      for (int n = 0; n < FN; ++n) bcur[n] = bnext[n];
    }
    // epilogue: C/D map col = lane&15, row = (lane>>4)*4 + j
#pragma unroll
    for (int n = 0; n < FN; ++n) {
      const int col = cb + n * 16 + lr;
      if (col >= H) continue;
      const float b = bias ? bias[col] : 0.f;
#pragma unroll
      for (int m = 0; m < FM; ++m) {
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int64_t row = row0 + wm * RW + m * 16 + (lane >> 4) * 4 + j;
          if (row < M) {
            float v = acc[m][n][j] + b;
            if (relu) v = fmaxf(v, 0.f);
            out[row * H + col] = f2bf(v);
          }
        }
      }
    }
  }
}

template <int BN>
__global__ __launch_bounds__(SAGE_THREADS) void sage_fwd_kernel(
    const bf16_t* __restrict__ x, int D, const int32_t* __restrict__ self_idx, const int32_t* __restrict__ nbr_idx,
    int F, int include_self, float inv_cnt, const bf16_t* __restrict__ W, const float* __restrict__ bias, int H,
    int64_t M, bf16_t* __restrict__ out, bf16_t* __restrict__ a_save, int relu) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int ldsw = 2 * D + 8;
  const int nblk = gridDim.x;
  const int tile = xcd_remap(blockIdx.x, nblk);
  const int64_t row0 = static_cast<int64_t>(tile) * SAGE_BM;
  sage_gather_tile(x, D, self_idx, nbr_idx, F, include_self, inv_cnt, M, row0, lds, ldsw, a_save);
  __syncthreads();
  sage_gemm_tile<BN>(lds, ldsw, 2 * D, W, bias, H, M, row0, relu, out);
}

// Plain MFMA linear on a materialised A (used by the backward recompute-free
// path and by the dense tower): out = act(A @ W^T + b), A [M, K] bf16, W [H, K].
template <int BN>
__global__ __launch_bounds__(SAGE_THREADS) void linear_fwd_kernel(const bf16_t* __restrict__ A, int K,
                                                                  const bf16_t* __restrict__ W,
                                                                  const float* __restrict__ bias, int H, int64_t M,
                                                                  bf16_t* __restrict__ out, int relu) {
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  const int ldsw = K + 8;
  const int tile = xcd_remap(blockIdx.x, gridDim.x);
  const int64_t row0 = static_cast<int64_t>(tile) * SAGE_BM;
  const int cpr = K >> 3;
  for (int it = threadIdx.x; it < SAGE_BM * cpr; it += SAGE_THREADS) {
    const int r = it / cpr, c = it - r * cpr;
    const int64_t g = row0 + r;
    uint4_t v = {0u, 0u, 0u, 0u};
    if (g < M) v = *reinterpret_cast<const uint4_t*>(A + g * K + c * 8);
    *reinterpret_cast<uint4_t*>(lds + r * ldsw + c * 8) = v;
  }
  __syncthreads();
  sage_gemm_tile<BN>(lds, ldsw, K, W, bias, H, M, row0, relu, out);
}

// ---------------------------------------------------------------------------
// backward: route dA = dPre @ W ([M, 2D]) back to the gathered input rows.
//   dx[self[m]] += dA[m, :D] + include_self * dA[m, D:] * inv_cnt
//   dx[nbr[m,k]] += dA[m, D:] * inv_cnt
// `disjoint` = every input row is referenced at most once (tree-layout blocks):
// plain stores, deterministic, no atomics.  Otherwise fp32 atomics.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void sage_bwd_scatter_kernel(const bf16_t* __restrict__ dA, int D,
                                                               const int32_t* __restrict__ self_idx,
                                                               const int32_t* __restrict__ nbr_idx, int F,
                                                               int include_self, float inv_cnt, int64_t M,
                                                               int disjoint, float* __restrict__ dx) {
  const int cpr = D >> 3;
  const int64_t it = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (it >= M * cpr) return;
  const int64_t m = it / cpr;
  const int c = static_cast<int>(it - m * cpr);
  const uint4_t vs = *reinterpret_cast<const uint4_t*>(dA + m * 2 * D + c * 8);
  const uint4_t vn = *reinterpret_cast<const uint4_t*>(dA + m * 2 * D + D + c * 8);
  float gs[8], gn[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) gs[i] = gn[i] = 0.f;
  acc_bf16x8(gs, vs);
  acc_bf16x8(gn, vn, inv_cnt);
  if (include_self) {
#pragma unroll
    for (int i = 0; i < 8; ++i) gs[i] += gn[i];
  }
  const int64_t s = self_idx[m];
  if (s >= 0) {
    float* p = dx + s * D + c * 8;
    if (disjoint) {
      *reinterpret_cast<float4_t*>(p) = float4_t{gs[0], gs[1], gs[2], gs[3]};
      *reinterpret_cast<float4_t*>(p + 4) = float4_t{gs[4], gs[5], gs[6], gs[7]};
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) atomicAdd(p + i, gs[i]);
    }
  }
  for (int k = 0; k < F; ++k) {
    const int64_t j = nbr_idx[m * F + k];
    if (j < 0) continue;
    float* p = dx + j * D + c * 8;
    if (disjoint) {
      *reinterpret_cast<float4_t*>(p) = float4_t{gn[0], gn[1], gn[2], gn[3]};
      *reinterpret_cast<float4_t*>(p + 4) = float4_t{gn[4], gn[5], gn[6], gn[7]};
    } else {
#pragma unroll
      for (int i = 0; i < 8; ++i) atomicAdd(p + i, gn[i]);
    }
  }
}

// gradient through ReLU, in place on a bf16 grad given the bf16 post-activation output
__global__ __launch_bounds__(256) void relu_bwd_kernel(bf16_t* __restrict__ g, const bf16_t* __restrict__ y,
                                                       int64_t n8) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n8) return;
  uint4_t gv = reinterpret_cast<uint4_t*>(g)[i];
  const uint4_t yv = reinterpret_cast<const uint4_t*>(y)[i];
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    uint32_t m = 0;
    // keep the grad half-word where y > 0 (sign bit clear and non-zero)
    if ((yv[q] & 0x8000u) == 0 && (yv[q] & 0x7fffu) != 0) m |= 0xffffu;
    if ((yv[q] & 0x80000000u) == 0 && (yv[q] & 0x7fff0000u) != 0) m |= 0xffff0000u;
    gv[q] &= m;
  }
  reinterpret_cast<uint4_t*>(g)[i] = gv;
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

static int sage_pick_bn(int H) { return H >= 256 ? 256 : (H > 64 ? 128 : 64); }

hipError_t eh_sage_fwd(const void* x, int D, const int32_t* self_idx, const int32_t* nbr_idx, int F,
                       int include_self, float inv_cnt, const void* W, const float* bias, int H, int64_t M, void* out,
                       void* a_save, int relu, hipStream_t s) {
  if (M == 0) return hipSuccess;
  if (D % 16 != 0 || D > 512) return hipErrorInvalidValue;
  const size_t lds = static_cast<size_t>(SAGE_BM) * (2 * D + 8) * sizeof(bf16_t);
  const dim3 grid(static_cast<uint32_t>(ceil_div(M, SAGE_BM)));
  const int bn = sage_pick_bn(H);
#define EH_LAUNCH(BNV)                                                                                           \
  do { if (lds > 65536) EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(sage_fwd_kernel<BNV>),     \
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
  hipLaunchKernelGGL(sage_fwd_kernel<BNV>, grid, dim3(SAGE_THREADS), lds, s, static_cast<const bf16_t*>(x), D,  \
                     self_idx, nbr_idx, F, include_self, inv_cnt, static_cast<const bf16_t*>(W), bias, H, M,     \
                     static_cast<bf16_t*>(out), static_cast<bf16_t*>(a_save), relu); } while (0)
  if (bn == 256) EH_LAUNCH(256);
  else if (bn == 128) EH_LAUNCH(128);
  else EH_LAUNCH(64);
#undef EH_LAUNCH
  return hipGetLastError();
}

hipError_t eh_linear_fwd(const void* A, int K, const void* W, const float* bias, int H, int64_t M, void* out,
                         int relu, hipStream_t s) {
  if (M == 0) return hipSuccess;
  if (K % 32 != 0 || K > 1024) return hipErrorInvalidValue;
  const size_t lds = static_cast<size_t>(SAGE_BM) * (K + 8) * sizeof(bf16_t);
  const dim3 grid(static_cast<uint32_t>(ceil_div(M, SAGE_BM)));
  const int bn = sage_pick_bn(H);
#define EH_LAUNCH(BNV)                                                                                         \
  do { if (lds > 65536) EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(linear_fwd_kernel<BNV>), \
                                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds)); \
  hipLaunchKernelGGL(linear_fwd_kernel<BNV>, grid, dim3(SAGE_THREADS), lds, s, static_cast<const bf16_t*>(A), \
                     K, static_cast<const bf16_t*>(W), bias, H, M, static_cast<bf16_t*>(out), relu); } while (0)
  if (bn == 256) EH_LAUNCH(256);
  else if (bn == 128) EH_LAUNCH(128);
  else EH_LAUNCH(64);
#undef EH_LAUNCH
  return hipGetLastError();
}

hipError_t eh_sage_bwd_scatter(const void* dA, int D, const int32_t* self_idx, const int32_t* nbr_idx, int F,
                               int include_self, float inv_cnt, int64_t M, int disjoint, float* dx, hipStream_t s) {
  if (M == 0) return hipSuccess;
  if (D % 8 != 0) return hipErrorInvalidValue;
  const int64_t items = M * (D / 8);
  hipLaunchKernelGGL(sage_bwd_scatter_kernel, dim3(static_cast<uint32_t>(ceil_div(items, 256))), dim3(256), 0, s,
                     static_cast<const bf16_t*>(dA), D, self_idx, nbr_idx, F, include_self, inv_cnt, M, disjoint,
                     dx);
  return hipGetLastError();
}

hipError_t eh_relu_bwd(void* g, const void* y, int64_t n, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (n % 8 != 0) return hipErrorInvalidValue;
  const int64_t n8 = n / 8;
  hipLaunchKernelGGL(relu_bwd_kernel, dim3(static_cast<uint32_t>(ceil_div(n8, 256))), dim3(256), 0, s,
                     static_cast<bf16_t*>(g), static_cast<const bf16_t*>(y), n8);
  return hipGetLastError();
}

}  // extern "C"
