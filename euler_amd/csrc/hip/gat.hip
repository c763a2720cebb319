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
// registers with an online (flash-style) max / sum-exp rescale done once per batch of U
// rows, and only out [S, H*C] plus the per-head log-sum-exp [S, H] are written.  Nothing
// of size [E, *] is ever materialised.
//
// Backward (no atomics, deterministic):
//   Dv_i   = <dout_i, out_i>  per head    (= sum_j p_ij dp_ij)
//   dp_ij  = <dout_i, h_j>,  ds = p (dp - Dv),  dz = ds * (z > 0 ? 1 : slope)
//   dar_i  = sum_j dz_ij                         <- destination pass (CSR); also packs
//                                                   (ar, lse, Dv) per (i, head) into one
//                                                   16-byte record for the next pass
//   dh_j   = sum_i p_ij dout_i,  dal_j = sum_i dz <- source pass (CSC), p recomputed
//                                                   from al/ar and the saved lse
//
// Scheduling: rows are visited in an optional `order` (the host passes rows sorted by
// degree, longest first), so the 64/lp rows sharing a wave have similar lengths (a wave
// runs as long as its longest row) and the heaviest rows start first.  The next batch's
// column indices are loaded before the current batch's rows are consumed, so each batch
// costs one memory round trip instead of two.  al of a neighbour is recomputed from its
// gathered row when a_src is given (one row fetch per edge instead of row + al line).
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

#ifndef GAT_FWD_U
#define GAT_FWD_U 2
#endif
#ifndef GAT_BWD_U
#define GAT_BWD_U 2
#endif
// neighbour rows in flight per lane group.  Measured on the ogbn-products-shaped graph
// (tools/gat_kernels.py, profiles/r2_gat/): 2 beats 4/8/16 — the gathers are latency-bound
// and fewer live rows per lane buys more resident waves than the unroll buys in-flight loads
// (fwd 5.3 ms at U=2 vs 8.4 ms at U=8; bwd 13.1 vs 15.9 ms).
#ifndef GAT_BWD_SRC_U
#define GAT_BWD_SRC_U GAT_BWD_U
#endif
constexpr int GAT_UF = GAT_FWD_U;
constexpr int GAT_UB = GAT_BWD_U;
constexpr int GAT_UBS = GAT_BWD_SRC_U;  // source (CSC) pass of the backward

// row of this lane group, its lane-in-row and whether the row exists
struct GatLane {
  int64_t row;
  int sub;
  bool ok;
};
__device__ __forceinline__ GatLane gat_lane(int lp, int64_t S, const int32_t* __restrict__ order) {
  const int lane = threadIdx.x & 63;
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t slot = wave * (64 / lp) + lane / lp;
  GatLane g;
  g.ok = slot < S;
  g.row = g.ok ? (order ? static_cast<int64_t>(order[slot]) : slot) : 0;
  g.sub = lane & (lp - 1);
  return g;
}

template <int U>
__device__ __forceinline__ void gat_load_idx(const int32_t* __restrict__ col, int64_t e, int64_t b, int32_t (&j)[U]) {
#pragma unroll
  for (int u = 0; u < U; ++u) j[u] = (e + u < b) ? col[e + u] : -1;
}

// ----------------------------------------------------------------------------- forward
template <typename T, int MAXCH>
__global__ __launch_bounds__(256) void gat_fwd_kernel(const int64_t* __restrict__ indptr,
                                                      const int32_t* __restrict__ col,
                                                      const int32_t* __restrict__ order, int64_t S,
                                                      const T* __restrict__ h, const float* __restrict__ al,
                                                      const float* __restrict__ ar, int H, int C, float slope, int lp,
                                                      T* __restrict__ out, float* __restrict__ lse,
                                                      const float* __restrict__ a_src) {
  constexpr int V = GV<T>::N;
  constexpr int U = GAT_UF;
  const int HC = H * C, nch = HC / V, g = C / V;
  const GatLane L = gat_lane(lp, S, order);
  // a_src given: al[j, h] = <h_j, a_src[h]> is recomputed from the neighbour row already in
  // registers (same per-lane partial + group sum as gat_att_fwd) instead of gathered, so an
  // edge costs one row fetch, not a row plus a 32-byte al line
  const bool rc = a_src != nullptr;
  bool ok[MAXCH];
  int hd[MAXCH];
  float ari[MAXCH], m[MAXCH], l[MAXCH], acc[MAXCH][V], asv[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    const int c = L.sub + k * lp;
    ok[k] = L.ok && c < nch;
    hd[k] = ok[k] ? (c * V) / C : 0;
    ari[k] = ok[k] ? ar[L.row * H + hd[k]] : 0.f;
    m[k] = -INFINITY;
    l[k] = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      acc[k][v] = 0.f;
      asv[k][v] = (rc && c < nch) ? a_src[c * V + v] : 0.f;
    }
  }
  const int64_t a = L.ok ? indptr[L.row] : 0, b = L.ok ? indptr[L.row + 1] : 0;
  int32_t jn[U];
  gat_load_idx<U>(col, a, b, jn);
  for (int64_t e = a; e < b; e += U) {
    int32_t j[U];
#pragma unroll
    for (int u = 0; u < U; ++u) j[u] = jn[u];
    gat_load_idx<U>(col, e + U, b, jn);  // next batch's indices, in flight with this batch's rows
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      if (!ok[k]) continue;
      const int c0 = (L.sub + k * lp) * V;
      float s[U], x[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        s[u] = -INFINITY;
        if (j[u] >= 0) {
          if (!rc) s[u] = al[static_cast<int64_t>(j[u]) * H + hd[k]];
          GV<T>::load(h + static_cast<int64_t>(j[u]) * HC + c0, x[u]);
        } else {
#pragma unroll
          for (int v = 0; v < V; ++v) x[u][v] = 0.f;
        }
      }
      if (rc) {
#pragma unroll
        for (int u = 0; u < U; ++u) {
          float d = 0.f;
#pragma unroll
          for (int v = 0; v < V; ++v) d += x[u][v] * asv[k][v];
          d = gat_group_sum(d, g);
          if (j[u] >= 0) s[u] = d;
        }
      }
      // one rescale per batch: nm = max(m, max_u s_u)
      float bm = m[k];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (j[u] >= 0) s[u] = lrelu(s[u] + ari[k], slope);
        bm = fmaxf(bm, s[u]);
      }
      const float sc = bm == -INFINITY ? 1.f : __expf(m[k] - bm);  // all-padding batch so far
      l[k] *= sc;
#pragma unroll
      for (int v = 0; v < V; ++v) acc[k][v] *= sc;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const float p = j[u] >= 0 ? __expf(s[u] - bm) : 0.f;
        l[k] += p;
#pragma unroll
        for (int v = 0; v < V; ++v) acc[k][v] += p * x[u][v];
      }
      m[k] = bm;
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
// writes dar [S, H] and the packed per-(row, head) record stat [S, H] = (ar, lse, Dv, 0)
template <typename T, int MAXCH>
__global__ __launch_bounds__(256) void gat_bwd_dst_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ col, const int32_t* __restrict__ order,
    int64_t S, const T* __restrict__ h, const float* __restrict__ al, const float* __restrict__ ar, int H, int C,
    float slope, int lp, const T* __restrict__ out, const T* __restrict__ dout, const float* __restrict__ lse,
    float* __restrict__ dar, float4_t* __restrict__ stat, const float* __restrict__ a_src) {
  constexpr int V = GV<T>::N;
  constexpr int U = GAT_UB;
  const int HC = H * C, nch = HC / V, g = C / V;
  const GatLane L = gat_lane(lp, S, order);
  const bool rc = a_src != nullptr;  // recompute al from the gathered row (see the forward)
  bool ok[MAXCH];
  int hd[MAXCH];
  float ari[MAXCH], lsei[MAXCH], Dv[MAXCH], dacc[MAXCH], dO[MAXCH][V], asv[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    const int c = L.sub + k * lp;
#pragma unroll
    for (int v = 0; v < V; ++v) asv[k][v] = (rc && c < nch) ? a_src[c * V + v] : 0.f;
    ok[k] = L.ok && c < nch;
    hd[k] = ok[k] ? (c * V) / C : 0;
    dacc[k] = 0.f;
    Dv[k] = 0.f;
    ari[k] = 0.f;
    lsei[k] = 0.f;
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
  int32_t jn[U];
  gat_load_idx<U>(col, a, b, jn);
  for (int64_t e = a; e < b; e += U) {
    int32_t j[U];
#pragma unroll
    for (int u = 0; u < U; ++u) j[u] = jn[u];
    gat_load_idx<U>(col, e + U, b, jn);
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      if (!ok[k]) continue;
      const int c0 = (L.sub + k * lp) * V;
      float z[U], part[U], alp[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        part[u] = 0.f;
        alp[u] = 0.f;
        z[u] = 0.f;
        if (j[u] >= 0) {
          float x[V];
          if (!rc) z[u] = al[static_cast<int64_t>(j[u]) * H + hd[k]] + ari[k];
          GV<T>::load(h + static_cast<int64_t>(j[u]) * HC + c0, x);
#pragma unroll
          for (int v = 0; v < V; ++v) {
            part[u] += dO[k][v] * x[v];
            alp[u] += x[v] * asv[k][v];
          }
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (j[u] < 0) continue;
        if (rc) z[u] = gat_group_sum(alp[u], g) + ari[k];
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
      stat[L.row * H + hd[k]] = float4_t{ari[k], lsei[k], Dv[k], 0.f};
    }
  }
}

// ----------------------------------------------------------------------------- backward, source pass
// cindptr/crow: CSC (edges grouped by source); crow holds the destination row.
template <typename T, int MAXCH>
__global__ __launch_bounds__(256) void gat_bwd_src_kernel(
    const int64_t* __restrict__ cindptr, const int32_t* __restrict__ crow, const int32_t* __restrict__ order,
    int64_t N, const T* __restrict__ h, const float* __restrict__ al, int H, int C, float slope, int lp,
    const T* __restrict__ dout, const float4_t* __restrict__ stat, T* __restrict__ dh, float* __restrict__ dal) {
  constexpr int V = GV<T>::N;
  constexpr int U = GAT_UBS;
  const int HC = H * C, nch = HC / V, g = C / V;
  const GatLane L = gat_lane(lp, N, order);
  bool ok[MAXCH];
  int hd[MAXCH];
  float alj[MAXCH], dalacc[MAXCH], hj[MAXCH][V], acc[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    const int c = L.sub + k * lp;
    ok[k] = L.ok && c < nch;
    hd[k] = ok[k] ? (c * V) / C : 0;
    dalacc[k] = 0.f;
    alj[k] = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) acc[k][v] = 0.f;
    if (ok[k]) {
      alj[k] = al[L.row * H + hd[k]];
      GV<T>::load(h + L.row * HC + c * V, hj[k]);
    }
  }
  const int64_t a = L.ok ? cindptr[L.row] : 0, b = L.ok ? cindptr[L.row + 1] : 0;
  int32_t in_[U];
  gat_load_idx<U>(crow, a, b, in_);
  for (int64_t e = a; e < b; e += U) {
    int32_t i[U];
#pragma unroll
    for (int u = 0; u < U; ++u) i[u] = in_[u];
    gat_load_idx<U>(crow, e + U, b, in_);
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      if (!ok[k]) continue;
      const int c0 = (L.sub + k * lp) * V;
      float4_t st[U];
      float part[U], dO[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        part[u] = 0.f;
        if (i[u] >= 0) {
          st[u] = stat[static_cast<int64_t>(i[u]) * H + hd[k]];
          GV<T>::load(dout + static_cast<int64_t>(i[u]) * HC + c0, dO[u]);
#pragma unroll
          for (int v = 0; v < V; ++v) part[u] += dO[u][v] * hj[k][v];
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (i[u] < 0) continue;
        const float dp = gat_group_sum(part[u], g);
        const float z = alj[k] + st[u][0];
        const float p = __expf(lrelu(z, slope) - st[u][1]);
        const float ds = p * (dp - st[u][2]);
        dalacc[k] += z > 0.f ? ds : ds * slope;
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

// ----------------------------------------------------------------------------- attention terms
// al[n, h] = <z[n, h, :], a_src[h, :]>,  ar[n, h] = <z[n, h, :], a_dst[h, :]>  (fp32 out; one read
// of z instead of an fp32 copy, two multiplies and two row reductions)
template <typename T, int MAXCH>
__global__ __launch_bounds__(256) void gat_att_fwd_kernel(const T* __restrict__ z, int64_t N, int H, int C, int lp,
                                                          const float* __restrict__ a_src,
                                                          const float* __restrict__ a_dst, float* __restrict__ al,
                                                          float* __restrict__ ar) {
  constexpr int V = GV<T>::N;
  const int HC = H * C, nch = HC / V, g = C / V;
  const GatLane L = gat_lane(lp, N, nullptr);
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    const int c = L.sub + k * lp;
    if (!(L.ok && c < nch)) continue;
    float x[V];
    GV<T>::load(z + L.row * HC + c * V, x);
    float ps = 0.f, pd = 0.f;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      ps += x[v] * a_src[c * V + v];
      pd += x[v] * a_dst[c * V + v];
    }
    ps = gat_group_sum(ps, g);
    pd = gat_group_sum(pd, g);
    if ((c * V) % C == 0) {
      al[L.row * H + (c * V) / C] = ps;
      ar[L.row * H + (c * V) / C] = pd;
    }
  }
}

// dz[n, :] += dal[n, h] a_src[h, :] + dar[n, h] a_dst[h, :]   (in place on the aggregation's dz)
// da_src[h, c] += sum_n dal[n, h] z[n, h, c]  (and da_dst): rows are visited grid-stride, each
// lane keeps its column partials in registers, one fp32 atomic per column per wave at the end.
template <typename T, int MAXCH>
__global__ __launch_bounds__(256) void gat_att_bwd_kernel(const T* __restrict__ z, int64_t N, int H, int C, int lp,
                                                          const float* __restrict__ a_src,
                                                          const float* __restrict__ a_dst,
                                                          const float* __restrict__ dal,
                                                          const float* __restrict__ dar, T* __restrict__ dz,
                                                          float* __restrict__ da_src, float* __restrict__ da_dst) {
  constexpr int V = GV<T>::N;
  const int HC = H * C, nch = HC / V;
  const int lane = threadIdx.x & 63;
  const int rpw = 64 / lp;
  const int sub = lane & (lp - 1);
  const int64_t wave = (static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x) >> 6;
  const int64_t nwaves = (static_cast<int64_t>(gridDim.x) * blockDim.x) >> 6;
  float ps[MAXCH][V], pd[MAXCH][V], as[MAXCH][V], ad[MAXCH][V];
#pragma unroll
  for (int k = 0; k < MAXCH; ++k) {
    const int c = sub + k * lp;
#pragma unroll
    for (int v = 0; v < V; ++v) {
      ps[k][v] = pd[k][v] = 0.f;
      as[k][v] = c < nch ? a_src[c * V + v] : 0.f;  // this lane's columns, loaded once
      ad[k][v] = c < nch ? a_dst[c * V + v] : 0.f;
    }
  }
  const int64_t stride = nwaves * rpw;
  // RR rows per lane group per iteration: all of their loads are issued before any use
  constexpr int RR = 4;
  for (int64_t r0 = wave * rpw + lane / lp; r0 < N; r0 += RR * stride) {
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      const int c = sub + k * lp;
      if (c >= nch) continue;
      const int h = (c * V) / C;
      float x[RR][V], d[RR][V], gs[RR], gd[RR];
#pragma unroll
      for (int q = 0; q < RR; ++q) {
        const int64_t r = r0 + q * stride;
        if (r < N) {
          gs[q] = dal[r * H + h];
          gd[q] = dar[r * H + h];
          GV<T>::load(z + r * HC + c * V, x[q]);
          GV<T>::load(dz + r * HC + c * V, d[q]);
        } else {
          gs[q] = gd[q] = 0.f;
#pragma unroll
          for (int v = 0; v < V; ++v) x[q][v] = d[q][v] = 0.f;
        }
      }
#pragma unroll
      for (int q = 0; q < RR; ++q) {
#pragma unroll
        for (int v = 0; v < V; ++v) {
          d[q][v] += gs[q] * as[k][v] + gd[q] * ad[k][v];
          ps[k][v] += gs[q] * x[q][v];
          pd[k][v] += gd[q] * x[q][v];
        }
        const int64_t r = r0 + q * stride;
        if (r < N) GV<T>::store(dz + r * HC + c * V, d[q]);
      }
    }
  }
  // the rpw row groups of the wave hold partials of the same columns: fold them
#pragma unroll
  for (int k = 0; k < MAXCH; ++k)
#pragma unroll
    for (int v = 0; v < V; ++v) {
      for (int o = lp; o < 64; o <<= 1) {
        ps[k][v] += __shfl_xor(ps[k][v], o, 64);
        pd[k][v] += __shfl_xor(pd[k][v], o, 64);
      }
    }
  // fold the block's 4 waves through LDS ([4][2*HC] floats, dynamic), then ONE plain store
  // of the block partial per column into [grid][HC] slabs summed on the host side (no
  // contended atomics: every block would otherwise add into the same 2*HC words)
  extern __shared__ float red[];
  const int w = threadIdx.x >> 6;
  if (lane < lp) {
#pragma unroll
    for (int k = 0; k < MAXCH; ++k) {
      const int c = sub + k * lp;
      if (c >= nch) continue;
#pragma unroll
      for (int v = 0; v < V; ++v) {
        red[w * 2 * HC + c * V + v] = ps[k][v];
        red[w * 2 * HC + HC + c * V + v] = pd[k][v];
      }
    }
  }
  __syncthreads();
  for (int c = threadIdx.x; c < 2 * HC; c += blockDim.x) {
    const float s = red[c] + red[2 * HC + c] + red[4 * HC + c] + red[6 * HC + c];
    if (c < HC)
      da_src[static_cast<int64_t>(blockIdx.x) * HC + c] = s;
    else
      da_dst[static_cast<int64_t>(blockIdx.x) * HC + c - HC] = s;
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

hipError_t eh_gat_fwd(const int64_t* indptr, const int32_t* col, const int32_t* order, int64_t S, const void* h,
                      int is_bf16, const float* al, const float* ar, int H, int C, float slope, void* out, float* lse,
                      const float* a_src, hipStream_t s) {
  if (S == 0) return hipSuccess;
  if (!eh_gat_supported(H, C, is_bf16)) return hipErrorInvalidValue;
  const GatShape sh = gat_shape(H * C, is_bf16 ? 8 : 4);
  const dim3 grid = gat_grid(S, sh.lp);
  if (is_bf16) {
    GAT_DISPATCH(bf16_t, sh.maxch, gat_fwd_kernel, grid, dim3(256), 0, s, indptr, col, order, S,
                 static_cast<const bf16_t*>(h), al, ar, H, C, slope, sh.lp, static_cast<bf16_t*>(out), lse, a_src)
  } else {
    GAT_DISPATCH(float, sh.maxch, gat_fwd_kernel, grid, dim3(256), 0, s, indptr, col, order, S,
                 static_cast<const float*>(h), al, ar, H, C, slope, sh.lp, static_cast<float*>(out), lse, a_src)
  }
  return hipGetLastError();
}

hipError_t eh_gat_att_fwd(const void* z, int is_bf16, int64_t N, int H, int C, const float* a_src,
                          const float* a_dst, float* al, float* ar, hipStream_t s) {
  if (N == 0) return hipSuccess;
  if (!eh_gat_supported(H, C, is_bf16)) return hipErrorInvalidValue;
  const GatShape sh = gat_shape(H * C, is_bf16 ? 8 : 4);
  const dim3 grid = gat_grid(N, sh.lp);
  if (is_bf16) {
    GAT_DISPATCH(bf16_t, sh.maxch, gat_att_fwd_kernel, grid, dim3(256), 0, s, static_cast<const bf16_t*>(z), N, H, C,
                 sh.lp, a_src, a_dst, al, ar)
  } else {
    GAT_DISPATCH(float, sh.maxch, gat_att_fwd_kernel, grid, dim3(256), 0, s, static_cast<const float*>(z), N, H, C,
                 sh.lp, a_src, a_dst, al, ar)
  }
  return hipGetLastError();
}

int eh_gat_att_bwd_blocks(int64_t N, int H, int C, int is_bf16) {
  // grid-stride: partials stay in registers across rows; <= 2048 block partials (8 waves
  // per CU of row streams)
  const GatShape sh = gat_shape(H * C, is_bf16 ? 8 : 4);
  const dim3 grid = gat_grid(N > 0 ? N : 1, sh.lp);
  return static_cast<int>(grid.x > 2048 ? 2048 : grid.x);
}

hipError_t eh_gat_att_bwd(const void* z, int is_bf16, int64_t N, int H, int C, const float* a_src, const float* a_dst,
                          const float* dal, const float* dar, void* dz, float* da_src, float* da_dst, hipStream_t s) {
  if (N == 0) return hipSuccess;
  if (!eh_gat_supported(H, C, is_bf16)) return hipErrorInvalidValue;
  const GatShape sh = gat_shape(H * C, is_bf16 ? 8 : 4);
  const dim3 grid(static_cast<uint32_t>(eh_gat_att_bwd_blocks(N, H, C, is_bf16)));
  const size_t lds = static_cast<size_t>(8) * H * C * sizeof(float);
  if (is_bf16) {
    GAT_DISPATCH(bf16_t, sh.maxch, gat_att_bwd_kernel, grid, dim3(256), lds, s, static_cast<const bf16_t*>(z), N, H,
                 C, sh.lp, a_src, a_dst, dal, dar, static_cast<bf16_t*>(dz), da_src, da_dst)
  } else {
    GAT_DISPATCH(float, sh.maxch, gat_att_bwd_kernel, grid, dim3(256), lds, s, static_cast<const float*>(z), N, H, C,
                 sh.lp, a_src, a_dst, dal, dar, static_cast<float*>(dz), da_src, da_dst)
  }
  return hipGetLastError();
}

hipError_t eh_gat_bwd(const int64_t* indptr, const int32_t* col, const int32_t* order, int64_t S,
                      const int64_t* cindptr, const int32_t* crow, const int32_t* corder, int64_t N, const void* h,
                      int is_bf16, const float* al, const float* ar, int H, int C, float slope, const void* out,
                      const void* dout, const float* lse, float* stat, void* dh, float* dal, float* dar,
                      const float* a_src, hipStream_t s) {
  if (!eh_gat_supported(H, C, is_bf16)) return hipErrorInvalidValue;
  const GatShape sh = gat_shape(H * C, is_bf16 ? 8 : 4);
  float4_t* st = reinterpret_cast<float4_t*>(stat);
  if (S > 0) {
    const dim3 grid = gat_grid(S, sh.lp);
    if (is_bf16) {
      GAT_DISPATCH(bf16_t, sh.maxch, gat_bwd_dst_kernel, grid, dim3(256), 0, s, indptr, col, order, S,
                   static_cast<const bf16_t*>(h), al, ar, H, C, slope, sh.lp, static_cast<const bf16_t*>(out),
                   static_cast<const bf16_t*>(dout), lse, dar, st, a_src)
    } else {
      GAT_DISPATCH(float, sh.maxch, gat_bwd_dst_kernel, grid, dim3(256), 0, s, indptr, col, order, S,
                   static_cast<const float*>(h), al, ar, H, C, slope, sh.lp, static_cast<const float*>(out),
                   static_cast<const float*>(dout), lse, dar, st, a_src)
    }
    EULER_HIP_CHECK(hipGetLastError());
  }
  if (N > 0) {
    const dim3 grid = gat_grid(N, sh.lp);
    if (is_bf16) {
      GAT_DISPATCH(bf16_t, sh.maxch, gat_bwd_src_kernel, grid, dim3(256), 0, s, cindptr, crow, corder, N,
                   static_cast<const bf16_t*>(h), al, H, C, slope, sh.lp, static_cast<const bf16_t*>(dout), st,
                   static_cast<bf16_t*>(dh), dal)
    } else {
      GAT_DISPATCH(float, sh.maxch, gat_bwd_src_kernel, grid, dim3(256), 0, s, cindptr, crow, corder, N,
                   static_cast<const float*>(h), al, H, C, slope, sh.lp, static_cast<const float*>(dout), st,
                   static_cast<float*>(dh), dal)
    }
    EULER_HIP_CHECK(hipGetLastError());
  }
  return hipSuccess;
}

}  // extern "C"
