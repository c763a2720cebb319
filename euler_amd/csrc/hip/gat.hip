// K5: multi-head GAT edge-softmax fused with the weighted neighbour
// aggregation, forward and backward, for every head in one launch.
//
// Reference computation (tf_euler/python/convolution/gat_conv.py:41-78 + mp_ops.py:76-79,
// one GATConv object per head, examples/gat/gat.py:56-70):
//   z_ij   = al[j, h] + ar[i, h]             (al = <a_src, h_j>, ar = <a_dst, h_i> per head)
//   s_ij   = leaky_relu(z_ij, slope)
//   p_ij   = softmax_{j in N(i)} s_ij        (scatter_max, exp, scatter_add, divide: 4 passes)
//   out_i  = sum_j p_ij * h_j[h, :]          (gather + multiply + scatter_add: 3 passes)
// Here that is ONE pass over the destination CSR: each destination row is owned by a
// group of lanes (8 bf16 / 4 fp32 columns per lane), the neighbour rows stream through
// registers with an online (flash-style) max / sum-exp rescale, and only out [S, H*C]
// plus the per-head log-sum-exp [S, H] are written.  Nothing of size [E, *] is ever
// materialised.
//
// Backward (no atomics, deterministic):
//   Dv_i   = <dout_i, out_i>  per head    (= sum_j p_ij dp_ij)
//   dp_ij  = <dout_i, h_j>,  ds = p (dp - Dv),  dz = ds * (z > 0 ? 1 : slope)
//   dar_i  = sum_j dz_ij                         <- destination pass (CSR)
//   dh_j   = sum_i p_ij dout_i,  dal_j = sum_i dz <- source pass (CSC), p recomputed
//                                                   from al/ar and the saved lse
#include "hip/common.h"
#include "hip/launchers.h"

namespace euler_hip {

template <typename T>
struct GV;  // 16-byte vector of T <-> fp32 registers
template <>
struct GV<bf16_t> {
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
struct GV<float> {
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

// sum over aligned groups of g lanes (g a power of two <= 64); every lane of a group
// takes the same control path (same row, same chunk slot), so the exchange is safe
__device__ __forceinline__ float gat_group_sum(float v, int g) {
  for (int o = g >> 1; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ float lrelu(float z, float slope) { return z > 0.f ? z : z * slope; }

constexpr int GAT_U = 4;  // neighbour rows in flight per lane

// row of this lane group, its lane-in-row and whether the row exists
struct GatLane {
  int64_t row;
  int sub;
  bool ok;
};
__device__ __forceinline__ GatLane gat_lane(int lp, int64_t S) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  GatLane g;
  g.row = wave * (64 / lp) + lane / lp;
  g.sub = lane & (lp - 1);
  g.ok = g.row < S;
  return g;
}

// ----------------------------------------------------------------------------- forward
template <typename T, int MAXCH>
__global__ __launch_bounds__(256) void gat_fwd_kernel(const int64_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ col, int64_t S,
                                                      const T* __restrict__ h, const float* __restrict__ al,
                                                      const float* __restrict__ ar, int H, int C, float slope, int lp,
                                                      T* __restrict__ out, float* __restrict__ lse) {
  constexpr int V = GV<T>::N;
  const int HC = H * C, nch = HC / V;
  const GatLane L = gat_lane(lp, S);
  bool ok[MAXCH];
  int hd[MAXCH];
  float ari[MAXCH], m[MAXCH], l[MAXCH], acc[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    const int c = L.sub + k * lp;
    ok[k] = L.ok && c < nch;
    hd[k] = ok[k] ? (c * V) / C : 0;
    ari[k] = ok[k] ? ar[L.row * H + hd[k]] : 0.f;
    m[k] = -INFINITY;
    l[k] = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) acc[k][v] = 0.f;
  }
  const int64_t a = L.ok ? indptr[L.row] : 0, b = L.ok ? indptr[L.row + 1] : 0;
  for (int64_t e = a; e < b; e += GAT_U) {
    int32_t j[GAT_U];
#pragma unroll
    for (int u = 0; u < GAT_U; ++u) j[u] = (e + u < b) ? col[e + u] : -1;
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      if (!ok[k]) continue;
      const int c0 = (L.sub + k * lp) * V;
      float z[GAT_U], x[GAT_U][V];
#pragma unroll
      for (int u = 0; u < GAT_U; ++u) {
        if (j[u] >= 0) {
          z[u] = al[static_cast<int64_t>(j[u]) * H + hd[k]] + ari[k];
          GV<T>::load(h + static_cast<int64_t>(j[u]) * HC + c0, x[u]);
        }
      }
#pragma unroll
      for (int u = 0; u < GAT_U; ++u) {
        if (j[u] < 0) continue;
        const float s = lrelu(z[u], slope);
        const float nm = fmaxf(m[k], s);
        const float sc = __expf(m[k] - nm);
        const float p = __expf(s - nm);
        l[k] = l[k] * sc + p;
#pragma unroll
        for (int v = 0; v < V; ++v) acc[k][v] = acc[k][v] * sc + p * x[u][v];
        m[k] = nm;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    if (!ok[k]) continue;
    const int c0 = (L.sub + k * lp) * V;
    const float inv = l[k] > 0.f ? 1.f / l[k] : 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) acc[k][v] *= inv;
    GV<T>::store(out + L.row * HC + c0, acc[k]);
    if (c0 % C == 0) lse[L.row * H + hd[k]] = l[k] > 0.f ? m[k] + __logf(l[k]) : 0.f;
  }
}

// ----------------------------------------------------------------------------- backward, destination pass
template <typename T, int MAXCH>
__global__ __launch_bounds__(256) void gat_bwd_dst_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ col, int64_t S, const T* __restrict__ h,
    const float* __restrict__ al, const float* __restrict__ ar, int H, int C, float slope, int lp,
    const T* __restrict__ out, const T* __restrict__ dout, const float* __restrict__ lse, float* __restrict__ dar,
    float* __restrict__ dv) {
  constexpr int V = GV<T>::N;
  const int HC = H * C, nch = HC / V, g = C / V;
  const GatLane L = gat_lane(lp, S);
  bool ok[MAXCH];
  int hd[MAXCH];
  float ari[MAXCH], lsei[MAXCH], Dv[MAXCH], dacc[MAXCH], dO[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    const int c = L.sub + k * lp;
    ok[k] = L.ok && c < nch;
    hd[k] = ok[k] ? (c * V) / C : 0;
    dacc[k] = 0.f;
    Dv[k] = 0.f;
    if (ok[k]) {
      ari[k] = ar[L.row * H + hd[k]];
      lsei[k] = lse[L.row * H + hd[k]];
      float o[V];
      GV<T>::load(dout + L.row * HC + c * V, dO[k]);
      GV<T>::load(out + L.row * HC + c * V, o);
      float part = 0.f;
#pragma unroll
      for (int v = 0; v < V; ++v) part += dO[k][v] * o[v];
      Dv[k] = gat_group_sum(part, g);
    }
  }
  const int64_t a = L.ok ? indptr[L.row] : 0, b = L.ok ? indptr[L.row + 1] : 0;
  for (int64_t e = a; e < b; e += GAT_U) {
    int32_t j[GAT_U];
#pragma unroll
    for (int u = 0; u < GAT_U; ++u) j[u] = (e + u < b) ? col[e + u] : -1;
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      if (!ok[k]) continue;
      const int c0 = (L.sub + k * lp) * V;
      float z[GAT_U], part[GAT_U];
#pragma unroll
      for (int u = 0; u < GAT_U; ++u) {
        part[u] = 0.f;
        z[u] = 0.f;
        if (j[u] >= 0) {
          float x[V];
          z[u] = al[static_cast<int64_t>(j[u]) * H + hd[k]] + ari[k];
          GV<T>::load(h + static_cast<int64_t>(j[u]) * HC + c0, x);
#pragma unroll
          for (int v = 0; v < V; ++v) part[u] += dO[k][v] * x[v];
        }
      }
#pragma unroll
      for (int u = 0; u < GAT_U; ++u) {
        if (j[u] < 0) continue;
        const float dp = gat_group_sum(part[u], g);
        const float p = __expf(lrelu(z[u], slope) - lsei[k]);
        const float ds = p * (dp - Dv[k]);
        dacc[k] += z[u] > 0.f ? ds : ds * slope;
      }
    }
  }
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    if (!ok[k]) continue;
    if (((L.sub + k * lp) * V) % C == 0) {
      dar[L.row * H + hd[k]] = dacc[k];
      dv[L.row * H + hd[k]] = Dv[k];
    }
  }
}

// ----------------------------------------------------------------------------- backward, source pass
// cindptr/crow: CSC (edges grouped by source); crow holds the destination row.
template <typename T, int MAXCH>
__global__ __launch_bounds__(256) void gat_bwd_src_kernel(
    const int64_t* __restrict__ cindptr, const int32_t* __restrict__ crow, int64_t N, const T* __restrict__ h,
    const float* __restrict__ al, const float* __restrict__ ar, int H, int C, float slope, int lp,
    const T* __restrict__ dout, const float* __restrict__ lse, const float* __restrict__ dv, T* __restrict__ dh,
    float* __restrict__ dal) {
  constexpr int V = GV<T>::N;
  const int HC = H * C, nch = HC / V, g = C / V;
  const GatLane L = gat_lane(lp, N);
  bool ok[MAXCH];
  int hd[MAXCH];
  float alj[MAXCH], dalacc[MAXCH], hj[MAXCH][V], acc[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    const int c = L.sub + k * lp;
    ok[k] = L.ok && c < nch;
    hd[k] = ok[k] ? (c * V) / C : 0;
    dalacc[k] = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) acc[k][v] = 0.f;
    if (ok[k]) {
      alj[k] = al[L.row * H + hd[k]];
      GV<T>::load(h + L.row * HC + c * V, hj[k]);
    }
  }
  const int64_t a = L.ok ? cindptr[L.row] : 0, b = L.ok ? cindptr[L.row + 1] : 0;
  for (int64_t e = a; e < b; e += GAT_U) {
    int32_t i[GAT_U];
#pragma unroll
    for (int u = 0; u < GAT_U; ++u) i[u] = (e + u < b) ? crow[e + u] : -1;
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      if (!ok[k]) continue;
      const int c0 = (L.sub + k * lp) * V;
      float z[GAT_U], ls[GAT_U], D[GAT_U], part[GAT_U], dO[GAT_U][V];
#pragma unroll
      for (int u = 0; u < GAT_U; ++u) {
        part[u] = 0.f;
        if (i[u] >= 0) {
          const int64_t ih = static_cast<int64_t>(i[u]) * H + hd[k];
          z[u] = alj[k] + ar[ih];
          ls[u] = lse[ih];
          D[u] = dv[ih];
          GV<T>::load(dout + static_cast<int64_t>(i[u]) * HC + c0, dO[u]);
#pragma unroll
          for (int v = 0; v < V; ++v) part[u] += dO[u][v] * hj[k][v];
        }
      }
#pragma unroll
      for (int u = 0; u < GAT_U; ++u) {
        if (i[u] < 0) continue;
        const float dp = gat_group_sum(part[u], g);
        const float p = __expf(lrelu(z[u], slope) - ls[u]);
        const float ds = p * (dp - D[u]);
        dalacc[k] += z[u] > 0.f ? ds : ds * slope;
#pragma unroll
        for (int v = 0; v < V; ++v) acc[k][v] += p * dO[u][v];
      }
    }
  }
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    if (!ok[k]) continue;
    const int c0 = (L.sub + k * lp) * V;
    GV<T>::store(dh + L.row * HC + c0, acc[k]);
    if (c0 % C == 0) dal[L.row * H + hd[k]] = dalacc[k];
  }
}

// lanes per row (power of two <= 64) and chunk slots per lane for H*C columns
struct GatShape {
  int lp, maxch;
};
inline GatShape gat_shape(int HC, int V) {
  const int nch = HC / V;
  int lp = 1;
  while (lp < nch && lp < 64) lp <<= 1;
  return GatShape{lp, static_cast<int>((nch + lp - 1) / lp)};
}

inline dim3 gat_grid(int64_t rows, int lp) {
  const int64_t rpw = 64 / lp;
  const int64_t waves = (rows + rpw - 1) / rpw;
  return dim3(static_cast<uint32_t>((waves + 3) / 4));
}

}  // namespace euler_hip

using namespace euler_hip;

#define GAT_DISPATCH(T, MAXCH_RT, KERNEL, ...)                                                     \
  switch (MAXCH_RT) {                                                                              \
    case 1: hipLaunchKernelGGL((KERNEL<T, 1>), __VA_ARGS__); break;                                \
    case 2: hipLaunchKernelGGL((KERNEL<T, 2>), __VA_ARGS__); break;                                \
    case 3:                                                                                        \
    case 4: hipLaunchKernelGGL((KERNEL<T, 4>), __VA_ARGS__); break;                                \
    default: return hipErrorInvalidValue;                                                          \
  }

extern "C" {

int eh_gat_supported(int H, int C, int is_bf16) {
  const int V = is_bf16 ? 8 : 4;
  if (H <= 0 || C <= 0 || C % V != 0) return 0;
  const int g = C / V;
  if (g > 64 || (g & (g - 1)) != 0) return 0;
  return gat_shape(H * C, V).maxch <= 4 ? 1 : 0;
}

hipError_t eh_gat_fwd(const int64_t* indptr, const int32_t* col, int64_t S, const void* h, int is_bf16,
                      const float* al, const float* ar, int H, int C, float slope, void* out, float* lse,
                      hipStream_t s) {
  if (S == 0) return hipSuccess;
  if (!eh_gat_supported(H, C, is_bf16)) return hipErrorInvalidValue;
  const GatShape sh = gat_shape(H * C, is_bf16 ? 8 : 4);
  const dim3 grid = gat_grid(S, sh.lp);
  if (is_bf16) {
    GAT_DISPATCH(bf16_t, sh.maxch, gat_fwd_kernel, grid, dim3(256), 0, s, indptr, col, S,
                 static_cast<const bf16_t*>(h), al, ar, H, C, slope, sh.lp, static_cast<bf16_t*>(out), lse)
  } else {
    GAT_DISPATCH(float, sh.maxch, gat_fwd_kernel, grid, dim3(256), 0, s, indptr, col, S,
                 static_cast<const float*>(h), al, ar, H, C, slope, sh.lp, static_cast<float*>(out), lse)
  }
  return hipGetLastError();
}

hipError_t eh_gat_bwd(const int64_t* indptr, const int32_t* col, int64_t S, const int64_t* cindptr,
                      const int32_t* crow, int64_t N, const void* h, int is_bf16, const float* al, const float* ar,
                      int H, int C, float slope, const void* out, const void* dout, const float* lse, float* dv,
                      void* dh, float* dal, float* dar, hipStream_t s) {
  if (!eh_gat_supported(H, C, is_bf16)) return hipErrorInvalidValue;
  const GatShape sh = gat_shape(H * C, is_bf16 ? 8 : 4);
  if (S > 0) {
    const dim3 grid = gat_grid(S, sh.lp);
    if (is_bf16) {
      GAT_DISPATCH(bf16_t, sh.maxch, gat_bwd_dst_kernel, grid, dim3(256), 0, s, indptr, col, S,
                   static_cast<const bf16_t*>(h), al, ar, H, C, slope, sh.lp, static_cast<const bf16_t*>(out),
                   static_cast<const bf16_t*>(dout), lse, dar, dv)
    } else {
      GAT_DISPATCH(float, sh.maxch, gat_bwd_dst_kernel, grid, dim3(256), 0, s, indptr, col, S,
                   static_cast<const float*>(h), al, ar, H, C, slope, sh.lp, static_cast<const float*>(out),
                   static_cast<const float*>(dout), lse, dar, dv)
    }
    EULER_HIP_CHECK(hipGetLastError());
  }
  if (N > 0) {
    const dim3 grid = gat_grid(N, sh.lp);
    if (is_bf16) {
      GAT_DISPATCH(bf16_t, sh.maxch, gat_bwd_src_kernel, grid, dim3(256), 0, s, cindptr, crow, N,
                   static_cast<const bf16_t*>(h), al, ar, H, C, slope, sh.lp, static_cast<const bf16_t*>(dout),
                   lse, dv, static_cast<bf16_t*>(dh), dal)
    } else {
      GAT_DISPATCH(float, sh.maxch, gat_bwd_src_kernel, grid, dim3(256), 0, s, cindptr, crow, N,
                   static_cast<const float*>(h), al, ar, H, C, slope, sh.lp, static_cast<const float*>(dout), lse,
                   dv, static_cast<float*>(dh), dal)
    }
    EULER_HIP_CHECK(hipGetLastError());
  }
  return hipSuccess;
}

}  // extern "C"
