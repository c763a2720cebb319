// One weighted neighbour draw of a (row, type)-segmented CSR with per-segment cumulative
// weights, shared by sample_neighbor_kernel (sampling.hip) and the fused GCN step's
// layer-wise draw (gcn.hip): the edge-type group proportionally to its weight sum (u01 of
// r[0]), then the first position whose cumulative weight exceeds u01(r[1]) * total.
// Returns the neighbour row or default_row; *w / *t: its weight and type (-1: none).
#pragma once
#include "hip/common.h"

namespace euler_hip {

__device__ __forceinline__ int32_t sample_one_neighbor(const int64_t* __restrict__ indptr,
                                                       const int32_t* __restrict__ nbr,
                                                       const float* __restrict__ cumw, int num_types,
                                                       uint32_t type_mask, int64_t row, const uint4_t& r,
                                                       int32_t default_row, float* w_out, int32_t* t_out) {
  const int64_t base = row * num_types;
  int64_t lo = 0, hi = 0;
  float total = 0.f;
  int32_t t = -1;
  if (num_types == 1) {
    lo = indptr[base];
    hi = indptr[base + 1];
    total = hi > lo ? cumw[hi - 1] : 0.f;
    t = 0;
  } else {
    float tot = 0.f;
    for (int k = 0; k < num_types; ++k) {
      if (!((type_mask >> k) & 1u)) continue;
      const int64_t a = indptr[base + k], b = indptr[base + k + 1];
      if (b > a) tot += cumw[b - 1];
    }
    if (tot > 0.f) {
      float u = u01(r[0]) * tot;
      for (int k = 0; k < num_types; ++k) {
        if (!((type_mask >> k) & 1u)) continue;
        const int64_t a = indptr[base + k], b = indptr[base + k + 1];
        if (b <= a) continue;
        const float g = cumw[b - 1];
        lo = a;
        hi = b;
        total = g;
        t = k;
        if (u < g) break;
        u -= g;
      }
    }
  }
  int32_t res = default_row;
  float w = 0.f;
  if (hi > lo && total > 0.f) {
    const float u = u01(r[1]) * total;
    int64_t a = lo, b = hi - 1;  // first position with cumw > u
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      if (cumw[m] > u) b = m;
      else a = m + 1;
    }
    res = nbr[a];
    w = cumw[a] - (a > lo ? cumw[a - 1] : 0.f);
  } else {
    t = -1;
  }
  if (w_out) *w_out = w;
  if (t_out) *t_out = t;
  return res;
}

}  // namespace euler_hip
