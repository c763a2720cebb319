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


hipError_t eh_seg_count(const int64_t* idx, int64_t n, int64_t size, int64_t* cnt, hipStream_t s) {
  if (n <= 0) return hipSuccess;
  hipLaunchKernelGGL(seg_count_kernel, grid_for(n), dim3(256), 0, s, idx, n, size,
                     reinterpret_cast<unsigned long long*>(cnt));
  return hipGetLastError();
}

}  // extern "C"
