// Message-passing primitives:
//   gather_rows      out[e]  = x[idx[e]]                         (K1; idx < 0 -> zero row)
//   segment_reduce   out[s]  = reduce_{e in seg s} src[perm[e]]  (K2; sum | mean | max + argmax)
//   index_add_rows   out[idx[e]] += src[e]                       (atomic fp32, gather backward)
//   scatter_rows     out[idx[e]]  = src[e]                       (max backward, unique positions)
//   edge_softmax     per-destination online softmax over [E, H] logits (K5)
//
// Segments come from a CSR over *destination* indices built once per block
// (sorted by destination), so sum/mean/max are deterministic and atomic-free
// (reference used tf.tensor_scatter_add / a serial loop: mp_ops.py:27-79,
// tf_euler/kernels/scatter_op.cc:27-105).
#include "hip/common.h"

namespace euler_hip {

// rows are moved in 16-byte vectors when possible, else 4-byte words
template <int VB>  // vector bytes: 16 or 4
struct Vec;
template <>
struct Vec<16> { using T = uint4_t; };
template <>
struct Vec<4> { using T = uint32_t; };
template <>
struct Vec<2> { using T = uint16_t; };  // rows of an odd number of bf16 values (e.g. 1433-d)

template <int VB, typename IdxT>
__global__ __launch_bounds__(256) void gather_rows_kernel(const uint8_t* __restrict__ x, int64_t n_rows,
                                                          int64_t row_bytes, const IdxT* __restrict__ idx,
                                                          int64_t n, uint8_t* __restrict__ out) {
  using V = typename Vec<VB>::T;
  const int64_t vpr = row_bytes / VB;
  grid_stride(n * vpr, [&](int64_t t) {
    const int64_t e = t / vpr, c = t - e * vpr;
    const int64_t r = static_cast<int64_t>(idx[e]);
    V v{};
    if (r >= 0 && r < n_rows) v = reinterpret_cast<const V*>(x + r * row_bytes)[c];
    reinterpret_cast<V*>(out + e * row_bytes)[c] = v;
  });
}

// out[e, :] = sum_f x[idx[e, f], :] in fp32 (idx < 0: skipped).  One thread per (row e,
// 16-byte column chunk); the F row loads are issued 4 at a time before they are summed, in
// f order (the same order as a gather followed by a sum over f).
template <bool BF>
__global__ __launch_bounds__(256) void gather_sum_kernel(const uint8_t* __restrict__ x, int64_t n_rows,
                                                         int64_t row_bytes, const int64_t* __restrict__ idx,
                                                         int64_t n, int F, float* __restrict__ out) {
  constexpr int V = BF ? 8 : 4;  // columns per 16-byte chunk
  const int64_t cpr = row_bytes / 16;
  grid_stride(n * cpr, [&](int64_t t) {
    const int64_t e = t / cpr, c = t - e * cpr;
    const int64_t* ie = idx + e * F;
    float acc[V];
#pragma unroll
    for (int v = 0; v < V; ++v) acc[v] = 0.f;
    for (int f0 = 0; f0 < F; f0 += 4) {
      uint4_t raw[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t r = f0 + u < F ? ie[f0 + u] : -1;
        raw[u] = uint4_t{0u, 0u, 0u, 0u};
        if (r >= 0 && r < n_rows) raw[u] = reinterpret_cast<const uint4_t*>(x + r * row_bytes)[c];
      }
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        if constexpr (BF) {
          acc_bf16x8(acc, raw[u]);
        } else {
#pragma unroll
          for (int v = 0; v < 4; ++v) acc[v] += __uint_as_float(raw[u][v]);
        }
      }
    }
    float4_t* o = reinterpret_cast<float4_t*>(out + e * (cpr * V) + c * V);
    o[0] = float4_t{acc[0], acc[1], acc[2], acc[3]};
    if constexpr (BF) o[1] = float4_t{acc[4], acc[5], acc[6], acc[7]};
  });
}

template <typename T>
__device__ __forceinline__ float ld(const T* p);
template <>
__device__ __forceinline__ float ld<float>(const float* p) { return *p; }
template <>
__device__ __forceinline__ float ld<bf16_t>(const bf16_t* p) { return bf2f(*p); }
template <typename T>
__device__ __forceinline__ void st(T* p, float v);
template <>
__device__ __forceinline__ void st<float>(float* p, float v) { *p = v; }
template <>
__device__ __forceinline__ void st<bf16_t>(bf16_t* p, float v) { *p = f2bf(v); }

// op: 0 sum, 1 mean, 2 max.  One thread per (segment, 4-column group).
template <typename T>
__global__ __launch_bounds__(256) void segment_reduce_kernel(const T* __restrict__ src, int D,
                                                             const int64_t* __restrict__ indptr,
                                                             const int64_t* __restrict__ perm, int64_t S, int op,
                                                             float empty_val, T* __restrict__ out,
                                                             int64_t* __restrict__ argmax) {
  const int groups = (D + 3) / 4;
  grid_stride(S * groups, [&](int64_t t) {
    const int64_t s = t / groups;
    const int d0 = static_cast<int>(t - s * groups) * 4;
    const int nd = min(4, D - d0);
    const int64_t a = indptr[s], b = indptr[s + 1];
    float acc[4];
    int64_t am[4] = {-1, -1, -1, -1};
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] = op == 2 ? -INFINITY : 0.f;
    // 4 source rows in flight per thread: the perm loads, then the row loads, are issued
    // back to back instead of one dependent pair per edge
    constexpr int U = 4;
    for (int64_t e0 = a; e0 < b; e0 += U) {
      int64_t row[U];
      float v[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) row[u] = (e0 + u < b) ? (perm ? perm[e0 + u] : e0 + u) : -1;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) v[u][i] = (row[u] >= 0 && i < nd) ? ld<T>(src + row[u] * D + d0 + i) : 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (row[u] < 0) continue;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (i < nd) {
            if (op == 2) {
              if (v[u][i] > acc[i]) { acc[i] = v[u][i]; am[i] = row[u]; }
            } else {
              acc[i] += v[u][i];
            }
          }
        }
      }
    }
    const float inv = (op == 1 && b > a) ? 1.f / static_cast<float>(b - a) : 1.f;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      if (i < nd) {
        float v = acc[i] * inv;
        if (b == a) v = (op == 2) ? empty_val : 0.f;
        st<T>(out + s * D + d0 + i, v);
        if (argmax) argmax[s * D + d0 + i] = am[i];
      }
    }
  });
}

// 16-byte-vector form of segment_reduce for D % V == 0 (V = 8 bf16 / 4 fp32 columns per
// thread): one vector load per source row instead of V scalar loads, 8 rows in flight.
template <typename T>
struct SegVec;
template <>
struct SegVec<bf16_t> {
  static constexpr int V = 8;
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
struct SegVec<float> {
  static constexpr int V = 4;
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

template <typename T>
__global__ __launch_bounds__(256) void segment_reduce_vec_kernel(const T* __restrict__ src, int D,
                                                                 const int64_t* __restrict__ indptr,
                                                                 const int64_t* __restrict__ perm, int64_t S,
                                                                 int op, float empty_val, T* __restrict__ out,
                                                                 int64_t* __restrict__ argmax) {
  constexpr int V = SegVec<T>::V;
  const int groups = D / V;
  grid_stride(S * groups, [&](int64_t t) {
    const int64_t s = t / groups;
    const int d0 = static_cast<int>(t - s * groups) * V;
    const int64_t a = indptr[s], b = indptr[s + 1];
    float acc[V];
    int64_t am[V];
#pragma unroll
    for (int i = 0; i < V; ++i) {
      acc[i] = op == 2 ? -INFINITY : 0.f;
      am[i] = -1;
    }
    constexpr int U = 8;
    for (int64_t e0 = a; e0 < b; e0 += U) {
      int64_t row[U];
      float v[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) row[u] = (e0 + u < b) ? (perm ? perm[e0 + u] : e0 + u) : -1;
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (row[u] >= 0) {
          SegVec<T>::load(src + row[u] * D + d0, v[u]);
        } else {
#pragma unroll
          for (int i = 0; i < V; ++i) v[u][i] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (row[u] < 0) continue;
#pragma unroll
        for (int i = 0; i < V; ++i) {
          if (op == 2) {
            if (v[u][i] > acc[i]) {
              acc[i] = v[u][i];
              am[i] = row[u];
            }
          } else {
            acc[i] += v[u][i];
          }
        }
      }
    }
    const float inv = (op == 1 && b > a) ? 1.f / static_cast<float>(b - a) : 1.f;
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = b == a ? (op == 2 ? empty_val : 0.f) : acc[i] * inv;
    SegVec<T>::store(out + s * D + d0, acc);
    if (argmax) {
#pragma unroll
      for (int i = 0; i < V; ++i) argmax[s * D + d0 + i] = am[i];
    }
  });
}

// wave-per-segment sum / mean for skewed segment lengths (power-law in-degrees: a hot
// destination's long segment is no longer one lane group's serial chain).  A wave covers one
// segment: LP = D / V lanes per row, 64 / LP rows side by side, U row steps in flight, then
// a butterfly over the row slots.  op 0 sum, 1 mean; D / V a power of two <= 64.
template <typename T>
__global__ __launch_bounds__(256) void segment_reduce_wave_kernel(const T* __restrict__ src, int D,
                                                                  const int64_t* __restrict__ indptr,
                                                                  const int64_t* __restrict__ perm, int64_t S, int op,
                                                                  T* __restrict__ out) {
  constexpr int V = SegVec<T>::V;
  const int LP = D / V, R = 64 / LP;
  const int lane = threadIdx.x & 63, slot = lane / LP, d0 = (lane - slot * LP) * V;
  // one segment per wave and iteration (uniform per wave); capped grid, see grid_for
  for (int64_t s = static_cast<int64_t>(blockIdx.x) * 4 + (threadIdx.x >> 6); s < S;
       s += static_cast<int64_t>(gridDim.x) * 4) {
    const int64_t a = indptr[s], b = indptr[s + 1];
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    constexpr int U = 4;
    for (int64_t e0 = a + slot; e0 < b; e0 += static_cast<int64_t>(R) * U) {
      int64_t row[U];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        const int64_t e = e0 + static_cast<int64_t>(u) * R;
        row[u] = e < b ? (perm ? perm[e] : e) : -1;
      }
      float v[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (row[u] >= 0) {
          SegVec<T>::load(src + row[u] * D + d0, v[u]);
        } else {
#pragma unroll
          for (int i = 0; i < V; ++i) v[u][i] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] += v[u][i];
    }
    for (int off = LP; off < 64; off <<= 1)
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] += __shfl_xor(acc[i], off, 64);
    if (slot == 0) {
      const float inv = (op == 1 && b > a) ? 1.f / static_cast<float>(b - a) : 1.f;
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] *= inv;
      SegVec<T>::store(out + s * D + d0, acc);
    }
  }
}

template <typename T>
__global__ __launch_bounds__(256) void index_add_rows_kernel(const T* __restrict__ src, int D,
                                                             const int64_t* __restrict__ idx, int64_t n,
                                                             float* __restrict__ out, int64_t n_out) {
  grid_stride(n * D, [&](int64_t t) {
    const int64_t e = t / D;
    const int d = static_cast<int>(t - e * D);
    const int64_t r = idx[e];
    if (r < 0 || r >= n_out) return;
    atomicAdd(out + r * D + d, ld<T>(src + t));
  });
}

// max backward: grad_src[argmax[s,d], d] = grad_out[s,d]  (argmax positions are unique)
template <typename T>
__global__ __launch_bounds__(256) void max_bwd_kernel(const T* __restrict__ gout, const int64_t* __restrict__ argmax,
                                                      int64_t S, int D, T* __restrict__ gsrc) {
  grid_stride(S * D, [&](int64_t t) {
    const int64_t r = argmax[t];
    if (r < 0) return;
    const int d = static_cast<int>(t % D);
    gsrc[r * D + d] = gout[t];
  });
}

// ---------------------------------------------------------------------------
// K5: edge softmax over destination segments, H heads packed per edge.
//   logits [E, H] (edge order = perm over destination CSR), out [E, H]
// One thread per (segment, head): online max / sum-exp in a single pass, then
// a normalising pass (two reads of the segment's logits, one write).
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void edge_softmax_kernel(const T* __restrict__ logits, int H,
                                                           const int64_t* __restrict__ indptr,
                                                           const int64_t* __restrict__ perm, int64_t S,
                                                           T* __restrict__ out) {
  grid_stride(S * H, [&](int64_t t) {
    const int64_t s = t / H;
    const int h = static_cast<int>(t - s * H);
    const int64_t a = indptr[s], b = indptr[s + 1];
    float m = -INFINITY, l = 0.f;
    for (int64_t e = a; e < b; ++e) {
      const int64_t row = perm ? perm[e] : e;
      const float v = ld<T>(logits + row * H + h);
      const float nm = fmaxf(m, v);
      l = l * __expf(m - nm) + __expf(v - nm);
      m = nm;
    }
    const float inv = l > 0.f ? 1.f / l : 0.f;
    for (int64_t e = a; e < b; ++e) {
      const int64_t row = perm ? perm[e] : e;
      st<T>(out + row * H + h, __expf(ld<T>(logits + row * H + h) - m) * inv);
    }
  });
}

// softmax backward: g_in = p * (g - sum_seg(p * g))
template <typename T>
__global__ __launch_bounds__(256) void edge_softmax_bwd_kernel(const T* __restrict__ p, const T* __restrict__ g,
                                                               int H, const int64_t* __restrict__ indptr,
                                                               const int64_t* __restrict__ perm, int64_t S,
                                                               T* __restrict__ gin) {
  grid_stride(S * H, [&](int64_t t) {
    const int64_t s = t / H;
    const int h = static_cast<int>(t - s * H);
    const int64_t a = indptr[s], b = indptr[s + 1];
    float dot = 0.f;
    for (int64_t e = a; e < b; ++e) {
      const int64_t row = perm ? perm[e] : e;
      dot += ld<T>(p + row * H + h) * ld<T>(g + row * H + h);
    }
    for (int64_t e = a; e < b; ++e) {
      const int64_t row = perm ? perm[e] : e;
      const float pv = ld<T>(p + row * H + h);
      st<T>(gin + row * H + h, pv * (ld<T>(g + row * H + h) - dot));
    }
  });
}

// ---------------------------------------------------------------------------
// K4: CSR SpMM  out[s, :] = sum_{e in seg s} w[e] * x[col[e], :]  (row-split, one
// thread per (row, 4-column group), fp32 accumulation).  x may be bf16 or fp32.
// ---------------------------------------------------------------------------
template <typename T>
__global__ __launch_bounds__(256) void spmm_csr_kernel(const int64_t* __restrict__ indptr,
                                                       const int64_t* __restrict__ col,
                                                       const float* __restrict__ w, const T* __restrict__ x, int D,
                                                       int64_t S, T* __restrict__ out) {
  const int groups = (D + 3) / 4;
  grid_stride(S * groups, [&](int64_t t) {
    const int64_t s = t / groups;
    const int d0 = static_cast<int>(t - s * groups) * 4;
    const int nd = min(4, D - d0);
    float acc[4] = {0.f, 0.f, 0.f, 0.f};
    const int64_t a = indptr[s], b = indptr[s + 1];
    // 4 neighbour rows in flight per thread (index + weight loads, then the row loads)
    constexpr int U = 4;
    for (int64_t e0 = a; e0 < b; e0 += U) {
      int64_t c[U];
      float we[U], v[U][4];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        c[u] = (e0 + u < b) ? col[e0 + u] : -1;
        we[u] = (e0 + u < b && w) ? w[e0 + u] : 1.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) v[u][i] = (c[u] >= 0 && i < nd) ? ld<T>(x + c[u] * D + d0 + i) : 0.f;
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[i] += we[u] * v[u][i];
    }
#pragma unroll
    for (int i = 0; i < 4; ++i)
      if (i < nd) st<T>(out + s * D + d0 + i, acc[i]);
  });
}

// 16-byte-vector form of spmm_csr for D % V == 0 (SegVec: 8 bf16 / 4 fp32 columns per
// thread), 8 neighbour rows in flight
template <typename T>
__global__ __launch_bounds__(256) void spmm_csr_vec_kernel(const int64_t* __restrict__ indptr,
                                                           const int64_t* __restrict__ col,
                                                           const float* __restrict__ w, const T* __restrict__ x,
                                                           int D, int64_t S, T* __restrict__ out) {
  constexpr int V = SegVec<T>::V;
  const int groups = D / V;
  grid_stride(S * groups, [&](int64_t t) {
    const int64_t s = t / groups;
    const int d0 = static_cast<int>(t - s * groups) * V;
    float acc[V];
#pragma unroll
    for (int i = 0; i < V; ++i) acc[i] = 0.f;
    const int64_t a = indptr[s], b = indptr[s + 1];
    constexpr int U = 8;
    for (int64_t e0 = a; e0 < b; e0 += U) {
      int64_t c[U];
      float we[U], v[U][V];
#pragma unroll
      for (int u = 0; u < U; ++u) {
        c[u] = (e0 + u < b) ? col[e0 + u] : -1;
        we[u] = (e0 + u < b && w) ? w[e0 + u] : 1.f;
      }
#pragma unroll
      for (int u = 0; u < U; ++u) {
        if (c[u] >= 0) {
          SegVec<T>::load(x + c[u] * D + d0, v[u]);
        } else {
#pragma unroll
          for (int i = 0; i < V; ++i) v[u][i] = 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < U; ++u)
#pragma unroll
        for (int i = 0; i < V; ++i) acc[i] += we[u] * v[u][i];
    }
    SegVec<T>::store(out + s * D + d0, acc);
  });
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

hipError_t eh_gather_rows(const void* x, int64_t n_rows, int64_t row_bytes, const void* idx, int idx_is64, int64_t n,
                          void* out, hipStream_t s) {
  if (n == 0 || row_bytes == 0) return hipSuccess;
  const bool v16 = (row_bytes % 16 == 0) && (reinterpret_cast<uintptr_t>(x) % 16 == 0) &&
                   (reinterpret_cast<uintptr_t>(out) % 16 == 0);
  const bool v4 = !v16 && row_bytes % 4 == 0 && reinterpret_cast<uintptr_t>(x) % 4 == 0 &&
                  reinterpret_cast<uintptr_t>(out) % 4 == 0;
  if (!v16 && !v4 && row_bytes % 2 != 0) return hipErrorInvalidValue;
  const int vb = v16 ? 16 : (v4 ? 4 : 2);
  const int64_t total = n * (row_bytes / vb);
  const dim3 grid = grid_for(total);
  const uint8_t* xb = static_cast<const uint8_t*>(x);
  uint8_t* ob = static_cast<uint8_t*>(out);
  if (v16) {
    if (idx_is64)
      hipLaunchKernelGGL((gather_rows_kernel<16, int64_t>), grid, dim3(256), 0, s, xb, n_rows, row_bytes,
                         static_cast<const int64_t*>(idx), n, ob);
    else
      hipLaunchKernelGGL((gather_rows_kernel<16, int32_t>), grid, dim3(256), 0, s, xb, n_rows, row_bytes,
                         static_cast<const int32_t*>(idx), n, ob);
  } else if (v4) {
    if (idx_is64)
      hipLaunchKernelGGL((gather_rows_kernel<4, int64_t>), grid, dim3(256), 0, s, xb, n_rows, row_bytes,
                         static_cast<const int64_t*>(idx), n, ob);
    else
      hipLaunchKernelGGL((gather_rows_kernel<4, int32_t>), grid, dim3(256), 0, s, xb, n_rows, row_bytes,
                         static_cast<const int32_t*>(idx), n, ob);
  } else {
    if (idx_is64)
      hipLaunchKernelGGL((gather_rows_kernel<2, int64_t>), grid, dim3(256), 0, s, xb, n_rows, row_bytes,
                         static_cast<const int64_t*>(idx), n, ob);
    else
      hipLaunchKernelGGL((gather_rows_kernel<2, int32_t>), grid, dim3(256), 0, s, xb, n_rows, row_bytes,
                         static_cast<const int32_t*>(idx), n, ob);
  }
  return hipGetLastError();
}


hipError_t eh_gather_sum(const void* x, int is_bf16, int64_t n_rows, int64_t row_bytes, const int64_t* idx, int64_t n,
                         int F, float* out, hipStream_t s) {
  if (n == 0 || row_bytes == 0) return hipSuccess;
  if (row_bytes % 16 != 0 || reinterpret_cast<uintptr_t>(x) % 16 != 0 || reinterpret_cast<uintptr_t>(out) % 16 != 0 ||
      F < 0)
    return hipErrorInvalidValue;
  const dim3 grid = grid_for(n * (row_bytes / 16));
  const uint8_t* xb = static_cast<const uint8_t*>(x);
  if (is_bf16)
    hipLaunchKernelGGL((gather_sum_kernel<true>), grid, dim3(256), 0, s, xb, n_rows, row_bytes, idx, n, F, out);
  else
    hipLaunchKernelGGL((gather_sum_kernel<false>), grid, dim3(256), 0, s, xb, n_rows, row_bytes, idx, n, F, out);
  return hipGetLastError();
}

hipError_t eh_segment_reduce_wave(const void* src, int is_bf16, int D, const int64_t* indptr, const int64_t* perm,
                                  int64_t S, int op, void* out, hipStream_t s) {
  if (S == 0 || D == 0) return hipSuccess;
  const int V = is_bf16 ? 8 : 4;
  const int LP = D / V;
  if (D % V != 0 || LP > 64 || (LP & (LP - 1)) != 0 || op < 0 || op > 1) return hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(src) % 16 != 0 || reinterpret_cast<uintptr_t>(out) % 16 != 0)
    return hipErrorInvalidValue;
  const dim3 grid = grid_for(S, 4);
  if (is_bf16)
    hipLaunchKernelGGL(segment_reduce_wave_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(src), D,
                       indptr, perm, S, op, static_cast<bf16_t*>(out));
  else
    hipLaunchKernelGGL(segment_reduce_wave_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(src), D,
                       indptr, perm, S, op, static_cast<float*>(out));
  return hipGetLastError();
}

hipError_t eh_segment_reduce(const void* src, int is_bf16, int D, const int64_t* indptr, const int64_t* perm,
                             int64_t S, int op, float empty_val, void* out, int64_t* argmax, hipStream_t s) {
  if (S == 0 || D == 0) return hipSuccess;
  const int V = is_bf16 ? 8 : 4;
  if (D % V == 0 && reinterpret_cast<uintptr_t>(src) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0) {
    const dim3 vgrid = grid_for(S * (D / V));
    if (is_bf16)
      hipLaunchKernelGGL(segment_reduce_vec_kernel<bf16_t>, vgrid, dim3(256), 0, s, static_cast<const bf16_t*>(src),
                         D, indptr, perm, S, op, empty_val, static_cast<bf16_t*>(out), argmax);
    else
      hipLaunchKernelGGL(segment_reduce_vec_kernel<float>, vgrid, dim3(256), 0, s, static_cast<const float*>(src), D,
                         indptr, perm, S, op, empty_val, static_cast<float*>(out), argmax);
    return hipGetLastError();
  }
  const dim3 grid = grid_for(S * ((D + 3) / 4));
  if (is_bf16)
    hipLaunchKernelGGL(segment_reduce_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(src), D,
                       indptr, perm, S, op, empty_val, static_cast<bf16_t*>(out), argmax);
  else
    hipLaunchKernelGGL(segment_reduce_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(src), D,
                       indptr, perm, S, op, empty_val, static_cast<float*>(out), argmax);
  return hipGetLastError();
}

hipError_t eh_index_add_rows(const void* src, int is_bf16, int D, const int64_t* idx, int64_t n, float* out,
                             int64_t n_out, hipStream_t s) {
  if (n == 0 || D == 0) return hipSuccess;
  const dim3 grid = grid_for(n * D);
  if (is_bf16)
    hipLaunchKernelGGL(index_add_rows_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(src), D, idx,
                       n, out, n_out);
  else
    hipLaunchKernelGGL(index_add_rows_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(src), D, idx, n,
                       out, n_out);
  return hipGetLastError();
}

hipError_t eh_max_bwd(const void* gout, int is_bf16, const int64_t* argmax, int64_t S, int D, void* gsrc,
                      hipStream_t s) {
  if (S == 0 || D == 0) return hipSuccess;
  const dim3 grid = grid_for(S * D);
  if (is_bf16)
    hipLaunchKernelGGL(max_bwd_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(gout), argmax, S, D,
                       static_cast<bf16_t*>(gsrc));
  else
    hipLaunchKernelGGL(max_bwd_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(gout), argmax, S, D,
                       static_cast<float*>(gsrc));
  return hipGetLastError();
}

hipError_t eh_edge_softmax(const void* logits, int is_bf16, int H, const int64_t* indptr, const int64_t* perm,
                           int64_t S, void* out, hipStream_t s) {
  if (S == 0 || H == 0) return hipSuccess;
  const dim3 grid = grid_for(S * H);
  if (is_bf16)
    hipLaunchKernelGGL(edge_softmax_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(logits), H,
                       indptr, perm, S, static_cast<bf16_t*>(out));
  else
    hipLaunchKernelGGL(edge_softmax_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(logits), H,
                       indptr, perm, S, static_cast<float*>(out));
  return hipGetLastError();
}

hipError_t eh_edge_softmax_bwd(const void* p, const void* g, int is_bf16, int H, const int64_t* indptr,
                               const int64_t* perm, int64_t S, void* gin, hipStream_t s) {
  if (S == 0 || H == 0) return hipSuccess;
  const dim3 grid = grid_for(S * H);
  if (is_bf16)
    hipLaunchKernelGGL(edge_softmax_bwd_kernel<bf16_t>, grid, dim3(256), 0, s, static_cast<const bf16_t*>(p),
                       static_cast<const bf16_t*>(g), H, indptr, perm, S, static_cast<bf16_t*>(gin));
  else
    hipLaunchKernelGGL(edge_softmax_bwd_kernel<float>, grid, dim3(256), 0, s, static_cast<const float*>(p),
                       static_cast<const float*>(g), H, indptr, perm, S, static_cast<float*>(gin));
  return hipGetLastError();
}

hipError_t eh_spmm_csr(const int64_t* indptr, const int64_t* col, const float* w, const void* x, int is_bf16, int D,
                       int64_t S, void* out, hipStream_t s) {
  if (S == 0 || D == 0) return hipSuccess;
  const int V = is_bf16 ? 8 : 4;
  if (D % V == 0 && reinterpret_cast<uintptr_t>(x) % 16 == 0 && reinterpret_cast<uintptr_t>(out) % 16 == 0) {
    const dim3 vgrid = grid_for(S * (D / V));
    if (is_bf16)
      hipLaunchKernelGGL(spmm_csr_vec_kernel<bf16_t>, vgrid, dim3(256), 0, s, indptr, col, w,
                         static_cast<const bf16_t*>(x), D, S, static_cast<bf16_t*>(out));
    else
      hipLaunchKernelGGL(spmm_csr_vec_kernel<float>, vgrid, dim3(256), 0, s, indptr, col, w,
                         static_cast<const float*>(x), D, S, static_cast<float*>(out));
    return hipGetLastError();
  }
  const dim3 grid = grid_for(S * ((D + 3) / 4));
  if (is_bf16)
    hipLaunchKernelGGL(spmm_csr_kernel<bf16_t>, grid, dim3(256), 0, s, indptr, col, w,
                       static_cast<const bf16_t*>(x), D, S, static_cast<bf16_t*>(out));
  else
    hipLaunchKernelGGL(spmm_csr_kernel<float>, grid, dim3(256), 0, s, indptr, col, w, static_cast<const float*>(x), D,
                       S, static_cast<float*>(out));
  return hipGetLastError();
}

}  // extern "C"
