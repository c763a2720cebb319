// Fused sigmoid cross-entropy over (source, context) embedding pairs — the unsupervised
// GraphSAGE objective (reference tf_euler/python/mp_utils/base.py:80-91: logits of the B
// positives and B x K negatives, mean sigmoid CE) in two launches instead of ~20 torch
// elementwise / reduction kernels (profiles/r3_unsup/).
//
//   pair_fwd : one wave per source b: x_s = <es[b], ec[row(b, s)]> for s = 0 (positive,
//              row b) and s = 1..K (negatives, rows B + b K + s - 1); part[b] =
//              (sum_s softplus(x_s) - x_0) * inv_n, part[B + b] = reciprocal rank of the
//              positive; logits [B, 1 + K]
//   pair_sum : one workgroup: loss[0] = sum_b part[b]; mrr[0] += sum_b part[B + b] (a
//              fixed-order tree sum: deterministic, no same-address atomics)
//   pair_bwd : g_s = (sigmoid(x_s) - [s == 0]) * dloss[0] * inv_n; des[b] = sum_s g_s ec_s,
//              dec[row(b, s)] = g_s es[b]
#include "hip/common.h"
#include "hip/launchers.h"
#include "hip/tile.h"

namespace euler_hip {

constexpr int PL_MAXK = 15;  // negatives per source (larger K: the torch composition)

__device__ __forceinline__ float pl_softplus(float x) { return x > 20.f ? x : log1pf(__expf(x)); }

__global__ __launch_bounds__(256) void pair_fwd_kernel(const float* __restrict__ es, const float* __restrict__ ec,
                                                       int B, int K, int E, float inv_n, float* __restrict__ logits,
                                                       float* __restrict__ part) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  const int d = lane * 4;
  float4_t s = {0.f, 0.f, 0.f, 0.f};
  if (d < E) s = *reinterpret_cast<const float4_t*>(es + static_cast<int64_t>(b) * E + d);
  float x[PL_MAXK + 1];
#pragma unroll
  for (int k = 0; k <= PL_MAXK; ++k) {
    if (k > K) break;
    const int64_t row = k == 0 ? b : static_cast<int64_t>(B) + static_cast<int64_t>(b) * K + k - 1;
    float p = 0.f;
    if (d < E) {
      const float4_t c = *reinterpret_cast<const float4_t*>(ec + row * E + d);
      p = s[0] * c[0] + s[1] * c[1] + s[2] * c[2] + s[3] * c[3];
    }
    x[k] = wave_sum(p);
  }
  if (lane == 0) {
    float l = -x[0];
    int rank = 1;
#pragma unroll
    for (int k = 0; k <= PL_MAXK; ++k) {
      if (k > K) break;
      l += pl_softplus(x[k]);
      logits[static_cast<int64_t>(b) * (K + 1) + k] = x[k];
      if (k > 0 && x[k] >= x[0]) ++rank;
    }
    part[b] = l * inv_n;
    part[B + b] = 1.f / static_cast<float>(rank);
  }
}

__global__ __launch_bounds__(1024) void pair_sum_kernel(const float* __restrict__ part, int B, float* __restrict__ loss,
                                                        float* __restrict__ mrr) {
  __shared__ float red[2][16];
  float l = 0.f, r = 0.f;
  for (int b = threadIdx.x; b < B; b += 1024) {
    l += part[b];
    r += part[B + b];
  }
  l = wave_sum(l);
  r = wave_sum(r);
  const int w = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    red[0][w] = l;
    red[1][w] = r;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    float sl = 0.f, sr = 0.f;
    for (int i = 0; i < 16; ++i) {
      sl += red[0][i];
      sr += red[1][i];
    }
    loss[0] = sl;
    if (mrr) mrr[0] += sr;
  }
}

__global__ __launch_bounds__(256) void pair_bwd_kernel(const float* __restrict__ es, const float* __restrict__ ec,
                                                       int B, int K, int E, float inv_n,
                                                       const float* __restrict__ logits, const float* __restrict__ dloss,
                                                       float* __restrict__ des, float* __restrict__ dec) {
  const int b = blockIdx.x * 4 + (threadIdx.x >> 6), lane = threadIdx.x & 63;
  if (b >= B) return;
  const int d = lane * 4;
  if (d >= E) return;
  const float sc = dloss[0] * inv_n;
  const float4_t s = *reinterpret_cast<const float4_t*>(es + static_cast<int64_t>(b) * E + d);
  float4_t acc = {0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k <= K; ++k) {
    const float x = logits[static_cast<int64_t>(b) * (K + 1) + k];
    const float g = (1.f / (1.f + __expf(-x)) - (k == 0 ? 1.f : 0.f)) * sc;
    const int64_t row = k == 0 ? b : static_cast<int64_t>(B) + static_cast<int64_t>(b) * K + k - 1;
    const float4_t c = *reinterpret_cast<const float4_t*>(ec + row * E + d);
    acc += g * c;
    *reinterpret_cast<float4_t*>(dec + row * E + d) = g * s;
  }
  *reinterpret_cast<float4_t*>(des + static_cast<int64_t>(b) * E + d) = acc;
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

// part: [2 B] scratch; loss [1] is written, mrr [1] (optional) accumulated
hipError_t eh_pair_fwd(const float* es, const float* ec, int B, int K, int E, float inv_n, float* logits, float* part,
                       float* loss, float* mrr, hipStream_t s) {
  if (B == 0) return hipSuccess;
  if (E % 4 != 0 || E > 256 || K < 0 || K > PL_MAXK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pair_fwd_kernel, dim3(static_cast<uint32_t>(ceil_div(B, 4))), dim3(256), 0, s, es, ec, B, K, E,
                     inv_n, logits, part);
  hipLaunchKernelGGL(pair_sum_kernel, dim3(1), dim3(1024), 0, s, part, B, loss, mrr);
  return hipGetLastError();
}

hipError_t eh_pair_bwd(const float* es, const float* ec, int B, int K, int E, float inv_n, const float* logits,
                       const float* dloss, float* des, float* dec, hipStream_t s) {
  if (B == 0) return hipSuccess;
  if (E % 4 != 0 || E > 256 || K < 0 || K > PL_MAXK) return hipErrorInvalidValue;
  hipLaunchKernelGGL(pair_bwd_kernel, dim3(static_cast<uint32_t>(ceil_div(B, 4))), dim3(256), 0, s, es, ec, B, K, E,
                     inv_n, logits, dloss, des, dec);
  return hipGetLastError();
}

}  // extern "C"
