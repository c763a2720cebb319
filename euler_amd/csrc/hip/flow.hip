// Device-side full-neighbourhood expansion for the GCN-family dataflows (SURVEY P3/K4/K7;
// reference tf_euler/python/dataflow/gcn_dataflow.py:26-48: per hop, get_full_neighbor of
// every node of the current set, euler/core/kernels/get_nb_node_op.cc semantics: a node's
// out-edges of the requested types, type by type, in storage order).
//
// Capacity-padded and capturable: the target set is a fixed-size int64 array of rows
// (-1 = padding), the output edge arrays have a fixed capacity and every slot past the
// real edge count is -1, so one hipGraph replays the expansion for any batch.
//   flow_degree : deg[i] = out-degree of rows[i] over the type mask (0 for padding)
//   (scan)      : offs = inclusive prefix sum of deg (torch.cumsum, rocPRIM)
//   flow_expand : edge e -> target i by binary search in offs, then the (type, index)
//                 inside the target's segments; nbr[e] = neighbour row, src[e] = i
// The edges come out target-major (all of target 0's, then target 1's, ...), i.e. the
// reference's flat SparseTensor value order of get_full_neighbor.
#include "hip/common.h"
#include "hip/launchers.h"

namespace euler_hip {

__global__ __launch_bounds__(256) void flow_degree_kernel(const int64_t* __restrict__ indptr, int64_t num_rows,
                                                          int num_types, uint32_t mask,
                                                          const int64_t* __restrict__ rows, int64_t n,
                                                          int64_t* __restrict__ deg) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t r = rows[i];
  int64_t d = 0;
  if (r >= 0 && r < num_rows) {
    const int64_t base = r * num_types;
    for (int t = 0; t < num_types; ++t)
      if ((mask >> t) & 1u) d += indptr[base + t + 1] - indptr[base + t];
  }
  deg[i] = d;
}

__global__ __launch_bounds__(256) void flow_expand_kernel(const int64_t* __restrict__ indptr,
                                                          const int32_t* __restrict__ nbr, int64_t num_rows,
                                                          int num_types, uint32_t mask,
                                                          const int64_t* __restrict__ rows, int64_t n,
                                                          const int64_t* __restrict__ offs, int64_t cap,
                                                          int64_t* __restrict__ out_nbr,
                                                          int64_t* __restrict__ out_src,
                                                          int32_t* __restrict__ overflow) {
  const int64_t e = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (e >= cap) return;
  const int64_t total = n > 0 ? offs[n - 1] : 0;
  if (e == 0 && total > cap) atomicOr(overflow, 1);
  if (e >= total) {
    out_nbr[e] = -1;
    out_src[e] = -1;
    return;
  }
  // first target whose inclusive offset exceeds e
  int64_t lo = 0, hi = n - 1;
  while (lo < hi) {
    const int64_t m = (lo + hi) >> 1;
    if (offs[m] > e) hi = m;
    else lo = m + 1;
  }
  const int64_t r = rows[lo];
  int64_t k = e - (lo > 0 ? offs[lo - 1] : 0);  // edge index inside the target's edges
  const int64_t base = r * num_types;
  int64_t pos = -1;
  for (int t = 0; t < num_types; ++t) {
    if (!((mask >> t) & 1u)) continue;
    const int64_t a = indptr[base + t], len = indptr[base + t + 1] - a;
    if (k < len) {
      pos = a + k;
      break;
    }
    k -= len;
  }
  out_nbr[e] = pos >= 0 ? static_cast<int64_t>(nbr[pos]) : -1;
  out_src[e] = pos >= 0 ? lo : -1;
}

// One hop's block assembly after the expansion and the dedup (dataflow/device_flow.py
// DeviceFullFlow.produce, whose torch composition this replaces with one launch):
//   new set        new_n_id[j] = uniq[j] (j < cap_n), last_new[j] = j < min(cnt, cap_n) ? j : -1
//   positions      inv' = inv < cap_n ? inv : -1;  res_n_id = inv'[cap_e:]
//   edges          [neighbour edges..., self loops...]: target src[k] / last_idx[k - cap_e],
//                  source inv'[k]; an edge whose source is -1 gets target -1
//   dest. CSR      indptr[t] = min(offs[t-1], cap_e) + (self loops ? min(t, n_targets) : 0),
//                  perm[new_pos(k)] = k (the stable destination order, no sort), counts
// perm is zeroed by the caller: after a capacity overflow positions may collide and every
// entry must still be a valid edge index.
struct FlowBlockArgs {
  const int64_t *src, *offs, *uniq, *inv, *cnt, *last_idx, *n_targets;
  int64_t cap_e, cap_prev, cap_n, L, E;
  int32_t self_loops;
  int64_t *new_n_id, *res_n_id, *edge_t, *edge_s, *perm, *indptr, *counts, *last_new, *cnt_new;
  int32_t* overflow;
};

__device__ __forceinline__ int64_t fb_excl(const FlowBlockArgs& a, int64_t t) {  // exclusive offset of target t
  if (t <= 0) return 0;
  const int64_t o = a.offs[t - 1];
  return o < a.cap_e ? o : a.cap_e;
}

__global__ __launch_bounds__(256) void flow_block_kernel(FlowBlockArgs a) {
  const int64_t cnt = a.cnt[0];
  const int64_t nt = a.n_targets[0];
  const int64_t live = cnt < a.cap_n ? cnt : a.cap_n;
  int64_t n_items = a.E > a.cap_n ? a.E : a.cap_n;
  if (a.cap_prev + 1 > n_items) n_items = a.cap_prev + 1;
  grid_stride(n_items, [&](int64_t i) {
    if (i == 0) {
      a.cnt_new[0] = live;
      if (cnt > a.cap_n) atomicOr(a.overflow, 1);
    }
    if (i < a.cap_n) {
      a.new_n_id[i] = i < a.L ? a.uniq[i] : -1;
      a.last_new[i] = i < live ? i : -1;
    }
    if (i < a.cap_prev) {
      const int64_t v = a.inv[a.cap_e + i];
      a.res_n_id[i] = (v >= 0 && v < a.cap_n) ? v : -1;
    }
    if (i <= a.cap_prev) {
      const int64_t loops = a.self_loops ? (i < nt ? i : nt) : 0;
      const int64_t ip = fb_excl(a, i) + loops;
      a.indptr[i] = ip;
      if (i < a.cap_prev) {
        const int64_t loops1 = a.self_loops ? (i + 1 < nt ? i + 1 : nt) : 0;
        a.counts[i] = fb_excl(a, i + 1) + loops1 - ip;
      }
    }
    if (i < a.E) {
      const int64_t v = a.inv[i];
      const int64_t sv = (v >= 0 && v < a.cap_n) ? v : -1;
      int64_t t, pos;
      if (i < a.cap_e) {
        t = a.src[i];
        pos = a.self_loops ? (t >= 0 ? i + t : i + nt) : i;
      } else {
        const int64_t q = i - a.cap_e;
        t = a.last_idx[q];
        pos = q < nt ? fb_excl(a, q + 1) + q : a.cap_e + q;
      }
      a.edge_t[i] = sv >= 0 ? t : -1;
      a.edge_s[i] = sv;
      if (pos >= 0 && pos < a.E) a.perm[pos] = i;
    }
  });
}

// One hop's block of the fixed-fanout device SageDataFlow (dataflow/device_flow.py
// DeviceSageFlow.produce): neighbour edge k of target k / f, then one self loop per target;
// an edge whose source is -1 (no neighbour drawn, padding target) gets target -1.  Also the
// destination CSR the convolutions would otherwise sort for: counts here, indptr = their
// exclusive scan (the caller), perm from sage_place_kernel (valid edges of each target in
// order, its self loop last: the stable sort's order; padding edges are not placed).
struct SageBlockArgs {
  const int64_t *inv, *uniq, *cnt, *last_idx;
  int64_t cap_prev, f, cap_n, cap_e, L, E;
  int32_t self_loops;
  int64_t *new_n_id, *res_n_id, *edge_t, *edge_s, *counts, *last_new, *cnt_new;
  const int64_t* indptr;  // sage_place_kernel only
  int64_t* perm;
};

__device__ __forceinline__ bool sb_self_ok(const SageBlockArgs& a, int64_t t) {
  return a.self_loops && a.last_idx[t] >= 0 && a.inv[a.cap_e + t] >= 0;
}

__global__ __launch_bounds__(256) void sage_block_kernel(SageBlockArgs a) {
  const int64_t cnt = a.cnt[0];
  const int64_t live = cnt < a.cap_n ? cnt : a.cap_n;
  int64_t n_items = a.E > a.cap_n ? a.E : a.cap_n;
  if (a.cap_prev > n_items) n_items = a.cap_prev;
  grid_stride(n_items, [&](int64_t i) {
    if (i == 0) a.cnt_new[0] = live;
    if (i < a.cap_n) {
      a.new_n_id[i] = i < a.L ? a.uniq[i] : -1;
      a.last_new[i] = i < live ? i : -1;
    }
    if (i < a.cap_prev) {
      a.res_n_id[i] = a.inv[a.cap_e + i];
      int64_t c = sb_self_ok(a, i) ? 1 : 0;
      for (int64_t j = 0; j < a.f; ++j) c += a.inv[i * a.f + j] >= 0;
      a.counts[i] = c;
    }
    if (i < a.E) {
      const int64_t sv = a.inv[i];
      const int64_t t = i < a.cap_e ? i / a.f : a.last_idx[i - a.cap_e];
      a.edge_t[i] = sv >= 0 ? t : -1;
      a.edge_s[i] = sv;
    }
  });
}

__global__ __launch_bounds__(256) void sage_place_kernel(SageBlockArgs a) {
  grid_stride(a.cap_prev, [&](int64_t t) {
    int64_t p = a.indptr[t];
    for (int64_t j = 0; j < a.f; ++j) {
      const int64_t k = t * a.f + j;
      if (a.inv[k] >= 0) a.perm[p++] = k;
    }
    if (sb_self_ok(a, t)) a.perm[p] = a.cap_e + t;
  });
}

// symmetric GCN normalisation per edge (reference gcn_conv.py:32-40 + the edge product of
// convolution/convs.py Conv.edge_weight): w[e] = deg0[dst]^-1/2 * deg1[src]^-1/2 with the
// degrees clamped at 1e-12, 0 for a padding edge; one launch instead of ~9 torch ops
__global__ __launch_bounds__(256) void gcn_norm_weight_kernel(const int64_t* __restrict__ dst,
                                                              const int64_t* __restrict__ src, int64_t E,
                                                              const int64_t* __restrict__ c0, int64_t n0,
                                                              const int64_t* __restrict__ c1, int64_t n1,
                                                              float* __restrict__ w) {
  grid_stride(E, [&](int64_t e) {
    const int64_t d = dst[e], s = src[e];
    float v = 0.f;
    if (d >= 0 && d < n0 && s >= 0 && s < n1)
      v = rsqrtf(fmaxf(static_cast<float>(c0[d]), 1e-12f)) * rsqrtf(fmaxf(static_cast<float>(c1[s]), 1e-12f));
    w[e] = v;
  });
}

// cnt[v] += 1 for every 0 <= idx[i] < size (padding -1 skipped: no contended sentinel
// bin); cnt zeroed by the caller
__global__ __launch_bounds__(256) void seg_count_kernel(const int64_t* __restrict__ idx, int64_t n, int64_t size,
                                                        unsigned long long* __restrict__ cnt) {
  grid_stride(n, [&](int64_t i) {
    const int64_t v = idx[i];
    if (v >= 0 && v < size) atomicAdd(cnt + v, 1ull);
  });
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

hipError_t eh_flow_degree(const int64_t* indptr, int64_t num_rows, int num_types, uint32_t mask, const int64_t* rows,
                          int64_t n, int64_t* deg, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  if (num_types < 1 || num_types > 32) return hipErrorInvalidValue;
  hipLaunchKernelGGL(flow_degree_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, indptr,
                     num_rows, num_types, mask, rows, n, deg);
  return hipGetLastError();
}

hipError_t eh_flow_expand(const int64_t* indptr, const int32_t* nbr, int64_t num_rows, int num_types, uint32_t mask,
                          const int64_t* rows, int64_t n, const int64_t* offs, int64_t cap, int64_t* out_nbr,
                          int64_t* out_src, int32_t* overflow, hipStream_t s) {
  if (cap <= 0) return hipSuccess;
  if (num_types < 1 || num_types > 32) return hipErrorInvalidValue;
  hipLaunchKernelGGL(flow_expand_kernel, dim3(static_cast<uint32_t>(ceil_div(cap, 256))), dim3(256), 0, s, indptr,
                     nbr, num_rows, num_types, mask, rows, n, offs, cap, out_nbr, out_src, overflow);
  return hipGetLastError();
}


hipError_t eh_flow_block(const int64_t* src, const int64_t* offs, const int64_t* uniq, const int64_t* inv,
                         const int64_t* cnt, const int64_t* last_idx, const int64_t* n_targets, int64_t cap_e,
                         int64_t cap_prev, int64_t cap_n, int self_loops, int64_t* new_n_id, int64_t* res_n_id,
                         int64_t* edge_index, int64_t* perm, int64_t* indptr, int64_t* counts, int64_t* last_new,
                         int64_t* cnt_new, int32_t* overflow, hipStream_t s) {
  if (cap_e < 0 || cap_prev <= 0 || cap_n <= 0) return hipErrorInvalidValue;
  FlowBlockArgs a;
  a.src = src;
  a.offs = offs;
  a.uniq = uniq;
  a.inv = inv;
  a.cnt = cnt;
  a.last_idx = last_idx;
  a.n_targets = n_targets;
  a.cap_e = cap_e;
  a.cap_prev = cap_prev;
  a.cap_n = cap_n;
  a.L = cap_e + cap_prev;
  a.E = self_loops ? cap_e + cap_prev : cap_e;
  a.self_loops = self_loops;
  a.new_n_id = new_n_id;
  a.res_n_id = res_n_id;
  a.edge_t = edge_index;
  a.edge_s = edge_index + a.E;
  a.perm = perm;
  a.indptr = indptr;
  a.counts = counts;
  a.last_new = last_new;
  a.cnt_new = cnt_new;
  a.overflow = overflow;
  EULER_HIP_CHECK(eh_zero(perm, a.E * 8, s));
  int64_t n = a.E > cap_n ? a.E : cap_n;
  if (cap_prev + 1 > n) n = cap_prev + 1;
  hipLaunchKernelGGL(flow_block_kernel, grid_for(n), dim3(256), 0, s, a);
  return hipGetLastError();
}

static SageBlockArgs sage_block_args(const int64_t* inv, const int64_t* uniq, const int64_t* cnt,
                                     const int64_t* last_idx, int64_t cap_prev, int64_t f, int64_t cap_n,
                                     int self_loops) {
  SageBlockArgs a{};
  a.inv = inv;
  a.uniq = uniq;
  a.cnt = cnt;
  a.last_idx = last_idx;
  a.cap_prev = cap_prev;
  a.f = f;
  a.cap_n = cap_n;
  a.cap_e = cap_prev * f;
  a.L = a.cap_e + cap_prev;
  a.E = self_loops ? a.L : a.cap_e;
  a.self_loops = self_loops;
  return a;
}

hipError_t eh_sage_block(const int64_t* inv, const int64_t* uniq, const int64_t* cnt, const int64_t* last_idx,
                         int64_t cap_prev, int64_t f, int64_t cap_n, int self_loops, int64_t* new_n_id,
                         int64_t* res_n_id, int64_t* edge_index, int64_t* counts, int64_t* last_new, int64_t* cnt_new,
                         hipStream_t s) {
  if (cap_prev <= 0 || f <= 0 || cap_n <= 0) return hipErrorInvalidValue;
  SageBlockArgs a = sage_block_args(inv, uniq, cnt, last_idx, cap_prev, f, cap_n, self_loops);
  a.new_n_id = new_n_id;
  a.res_n_id = res_n_id;
  a.edge_t = edge_index;
  a.edge_s = edge_index + a.E;
  a.counts = counts;
  a.last_new = last_new;
  a.cnt_new = cnt_new;
  int64_t n = a.E > cap_n ? a.E : cap_n;
  if (cap_prev > n) n = cap_prev;
  hipLaunchKernelGGL(sage_block_kernel, grid_for(n), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t eh_sage_place(const int64_t* inv, const int64_t* last_idx, int64_t cap_prev, int64_t f, int self_loops,
                         const int64_t* indptr, int64_t* perm, hipStream_t s) {
  SageBlockArgs a = sage_block_args(inv, nullptr, nullptr, last_idx, cap_prev, f, 1, self_loops);
  a.indptr = indptr;
  a.perm = perm;
  EULER_HIP_CHECK(eh_zero(perm, a.E * 8, s));
  hipLaunchKernelGGL(sage_place_kernel, grid_for(cap_prev), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t eh_gcn_norm_weight(const int64_t* dst, const int64_t* src, int64_t E, const int64_t* c0, int64_t n0,
                              const int64_t* c1, int64_t n1, float* w, hipStream_t s) {
  if (E <= 0) return hipSuccess;
  hipLaunchKernelGGL(gcn_norm_weight_kernel, grid_for(E), dim3(256), 0, s, dst, src, E, c0, n0, c1, n1, w);
  return hipGetLastError();
}

hipError_t eh_seg_count(const int64_t* idx, int64_t n, int64_t size, int64_t* cnt, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(seg_count_kernel, grid_for(n), dim3(256), 0, s, idx, n, size,
                     reinterpret_cast<unsigned long long*>(cnt));
  return hipGetLastError();
}

}  // extern "C"
