// GPU-side graph sampling over an HBM-resident CSR shard.
//
// Layout of a device graph shard (see euler_amd/graph/device_graph.py):
//   indptr [N*T + 1] int64 : segment of (row n, edge type t) = [indptr[n*T+t], indptr[n*T+t+1])
//   nbr    [E]       int32 : neighbor row (dense row space, not raw ids)
//   cumw   [E]       fp32  : per-segment inclusive prefix sums of edge weights
//
// Semantics match the engine's weighted, with-replacement neighbor sampling
// (reference: euler/core/graph/node.cc:98-161 — pick an edge group by its
// weight sum, then binary-search the group's cumulative weights), with empty
// rows padded by `default_row` (reference: sample_neighbor_op.cc:37-145).
#include "hip/common.h"
#include "hip/sampling_math.h"

namespace euler_hip {

__global__ void rng_advance_kernel(int64_t* state, int64_t inc) { state[1] += inc; }

template <typename IdxT>
__global__ __launch_bounds__(256) void sample_neighbor_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ nbr, const float* __restrict__ cumw,
    int64_t num_rows, int num_types, uint32_t type_mask, const IdxT* __restrict__ nodes, int64_t n,
    int count, int32_t default_row, const int64_t* __restrict__ rng, uint64_t stream_id,
    int32_t* __restrict__ out, float* __restrict__ out_w, int32_t* __restrict__ out_t) {
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (tid >= n * count) return;
  const int64_t i = tid / count;
  const int64_t row = static_cast<int64_t>(nodes[i]);
  int32_t res = default_row;
  float w = 0.f;
  int32_t t_out = -1;
  if (row >= 0 && row < num_rows) {
    const uint4_t r = Philox::gen(static_cast<uint64_t>(rng[0]),
                                  (static_cast<uint64_t>(rng[1]) << 8) ^ stream_id,
                                  static_cast<uint64_t>(tid));
    res = sample_one_neighbor(indptr, nbr, cumw, num_types, type_mask, row, r, default_row, &w, &t_out);
  }
  out[tid] = res;
  if (out_w) out_w[tid] = w;
  if (out_t) out_t[tid] = t_out;
}

// Walker alias sampling of `count` rows from an (optionally sub-setted) population.
__global__ __launch_bounds__(256) void alias_sample_kernel(const float* __restrict__ prob,
                                                           const int32_t* __restrict__ alias,
                                                           const int32_t* __restrict__ rows, int64_t pop,
                                                           int64_t count, const int64_t* __restrict__ rng,
                                                           uint64_t stream_id, int32_t* __restrict__ out) {
  const int64_t tid = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (tid >= count) return;
  const uint4_t r = Philox::gen(static_cast<uint64_t>(rng[0]),
                                (static_cast<uint64_t>(rng[1]) << 8) ^ stream_id, static_cast<uint64_t>(tid));
  // 64-bit index from two words to avoid modulo bias on large populations
  const uint64_t x = (static_cast<uint64_t>(r[0]) << 32) | r[1];
  int64_t k = static_cast<int64_t>(__umul64hi(x, static_cast<uint64_t>(pop)));
  if (k >= pop) k = pop - 1;
  const int64_t pick = (u01(r[2]) < prob[k]) ? k : static_cast<int64_t>(alias[k]);
  out[tid] = rows ? rows[pick] : static_cast<int32_t>(pick);
}

// Random walks, out [n, walk_len + 1] (reference random_walk_op.cc:70-188).
// p = q = 1: chained weighted neighbour sampling (type group by weight, then a binary
// search of its prefix sums).  Otherwise node2vec: candidate weights of the current row
// times 1/p for the previous row, 1 for rows in the previous row's neighbour segments
// (previous step's edge types; binary search, segments are sorted by row), 1/q for the
// rest; two passes over the candidates (total, then the draw).  As in the reference the
// first step's "previous" row is the start itself with no neighbour set.
__device__ __forceinline__ bool rw_in_row(const int64_t* __restrict__ indptr, const int32_t* __restrict__ nbr,
                                          int num_types, uint32_t mask, int64_t row, int32_t v) {
  for (int t = 0; t < num_types; ++t) {
    if (!((mask >> t) & 1u)) continue;
    int64_t a = indptr[row * num_types + t], b = indptr[row * num_types + t + 1];
    while (a < b) {
      const int64_t m = (a + b) >> 1;
      const int32_t x = nbr[m];
      if (x == v) return true;
      if (x < v) a = m + 1;
      else b = m;
    }
  }
  return false;
}

__global__ __launch_bounds__(256) void random_walk_kernel(
    const int64_t* __restrict__ indptr, const int32_t* __restrict__ nbr, const float* __restrict__ cumw,
    int64_t num_rows, int num_types, const uint32_t* __restrict__ step_masks, const int32_t* __restrict__ starts,
    int64_t n, int walk_len, int32_t default_row, const int64_t* __restrict__ rng, uint64_t stream_id,
    float inv_p, float inv_q, int biased, int32_t* __restrict__ out) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  int64_t cur = starts[i];
  int64_t prev = cur;
  uint32_t prev_mask = 0u;  // no neighbour set before the first step
  out[i * (walk_len + 1)] = static_cast<int32_t>(cur);
  for (int s = 0; s < walk_len; ++s) {
    int32_t nxt = default_row;
    const uint32_t mask = step_masks[s];
    if (cur >= 0 && cur < num_rows) {
      const uint4_t r = Philox::gen(static_cast<uint64_t>(rng[0]),
                                    (static_cast<uint64_t>(rng[1]) << 8) ^ stream_id,
                                    static_cast<uint64_t>(i) * 1024u + s);
      const int64_t base = cur * num_types;
      if (biased) {
        const bool has_prev = prev >= 0 && prev < num_rows;
        float tot = 0.f;
        // `picked` (not nxt == default_row) marks a draw: the default may be a valid row
        bool picked = false;
        for (int pass = 0; pass < 2 && !picked; ++pass) {
          const float target = pass == 0 ? 0.f : u01(r[0]) * tot;
          float acc = 0.f;
          int32_t last = default_row;
          bool have_last = false;
          for (int t = 0; t < num_types && !picked; ++t) {
            if (!((mask >> t) & 1u)) continue;
            const int64_t a = indptr[base + t], b = indptr[base + t + 1];
            for (int64_t e = a; e < b; ++e) {
              const int32_t c = nbr[e];
              float w = e > a ? cumw[e] - cumw[e - 1] : cumw[e];
              if (c == prev) w *= inv_p;
              else if (!(has_prev && prev_mask && rw_in_row(indptr, nbr, num_types, prev_mask, prev, c))) w *= inv_q;
              acc += w;
              if (w > 0.f) {
                last = c;
                have_last = true;
              }
              if (pass == 1 && acc > target) {
                nxt = c;
                picked = true;
                break;
              }
            }
          }
          if (pass == 0) tot = acc;
          if (pass == 1 && !picked && have_last) {  // rounding at the top end
            nxt = last;
            picked = true;
          }
          if (pass == 0 && !(tot > 0.f)) break;
        }
      } else {
        float tot = 0.f;
        for (int t = 0; t < num_types; ++t) {
          if (!((mask >> t) & 1u)) continue;
          const int64_t a = indptr[base + t], b = indptr[base + t + 1];
          if (b > a) tot += cumw[b - 1];
        }
        if (tot > 0.f) {
          float u = u01(r[0]) * tot;
          int64_t lo = 0, hi = 0;
          float g = 0.f;
          for (int t = 0; t < num_types; ++t) {
            if (!((mask >> t) & 1u)) continue;
            const int64_t a = indptr[base + t], b = indptr[base + t + 1];
            if (b <= a) continue;
            g = cumw[b - 1];
            lo = a;
            hi = b;
            if (u < g) break;
            u -= g;
          }
          const float v = u01(r[1]) * g;
          int64_t a = lo, b = hi - 1;
          while (a < b) {
            const int64_t m = (a + b) >> 1;
            if (cumw[m] > v) b = m;
            else a = m + 1;
          }
          nxt = nbr[a];
        }
      }
    }
    out[i * (walk_len + 1) + s + 1] = nxt;
    prev = cur;
    prev_mask = mask;
    cur = nxt;
  }
}

// ---------------------------------------------------------------------------
// synthetic power-law CSR generator (device side, so a 100M-node / 1B-edge
// shard never has to exist in host RAM).  Two passes:
//   1. degree[n] ~ clipped discrete Pareto (mean avg_deg), exclusive scan -> indptr (torch.cumsum)
//   2. fill: neighbors uniform over rows with a locality bias, weights U(0.5,1.5),
//      per-row sorted neighbor ids (small insertion sort) and inclusive prefix sums.
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void synth_degree_kernel(int64_t n, float avg_deg, int max_deg, uint64_t seed,
                                                           int64_t* __restrict__ deg) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const uint4_t r = Philox::gen(seed, 0x5EEDull, static_cast<uint64_t>(i));
  // Pareto with alpha = 2 (finite mean) shifted so E[d] ~= avg_deg
  const float u = fmaxf(u01(r[0]), 1e-7f);
  const float xm = avg_deg * 0.5f;
  float d = xm / sqrtf(u);
  int di = static_cast<int>(d);
  if (di < 1) di = 1;
  if (di > max_deg) di = max_deg;
  deg[i] = di;
}

__global__ __launch_bounds__(256) void synth_fill_kernel(int64_t n, const int64_t* __restrict__ indptr,
                                                         uint64_t seed, int32_t* __restrict__ nbr,
                                                         float* __restrict__ cumw) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int64_t a = indptr[i], b = indptr[i + 1];
  float acc = 0.f;
  for (int64_t e = a; e < b; ++e) {
    const uint4_t r = Philox::gen(seed, 0xED6Eull, static_cast<uint64_t>(e));
    const uint64_t x = (static_cast<uint64_t>(r[0]) << 32) | r[1];
    int64_t v = static_cast<int64_t>(__umul64hi(x, static_cast<uint64_t>(n)));
    if (v == i) v = (v + 1) % n;  // no self loops in the synthetic graph
    // insertion into the sorted prefix of this row
    int64_t p = e;
    while (p > a && nbr[p - 1] > v) {
      nbr[p] = nbr[p - 1];
      cumw[p] = cumw[p - 1];  // temporarily holds raw weights
      --p;
    }
    nbr[p] = static_cast<int32_t>(v);
    cumw[p] = 0.5f + u01(r[2]);
  }
  for (int64_t e = a; e < b; ++e) {
    acc += cumw[e];
    cumw[e] = acc;
  }
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

hipError_t eh_rng_advance(int64_t* state, int64_t inc, hipStream_t s) {
  hipLaunchKernelGGL(rng_advance_kernel, dim3(1), dim3(1), 0, s, state, inc);
  return hipGetLastError();
}

hipError_t eh_sample_neighbor(const int64_t* indptr, const int32_t* nbr, const float* cumw, int64_t num_rows,
                              int num_types, uint32_t type_mask, const void* nodes, int nodes_is64, int64_t n,
                              int count, int32_t default_row, const int64_t* rng, uint64_t stream_id, int32_t* out,
                              float* out_w, int32_t* out_t, hipStream_t s) {
  const int64_t total = n * count;
  if (total == 0) return hipSuccess;
  const dim3 grid(static_cast<uint32_t>(ceil_div(total, 256)));
  if (nodes_is64)
    hipLaunchKernelGGL(sample_neighbor_kernel<int64_t>, grid, dim3(256), 0, s, indptr, nbr, cumw, num_rows,
                       num_types, type_mask, static_cast<const int64_t*>(nodes), n, count, default_row, rng,
                       stream_id, out, out_w, out_t);
  else
    hipLaunchKernelGGL(sample_neighbor_kernel<int32_t>, grid, dim3(256), 0, s, indptr, nbr, cumw, num_rows,
                       num_types, type_mask, static_cast<const int32_t*>(nodes), n, count, default_row, rng,
                       stream_id, out, out_w, out_t);
  return hipGetLastError();
}

hipError_t eh_alias_sample(const float* prob, const int32_t* alias, const int32_t* rows, int64_t pop, int64_t count,
                           const int64_t* rng, uint64_t stream_id, int32_t* out, hipStream_t s) {
  if (count == 0) return hipSuccess;
  hipLaunchKernelGGL(alias_sample_kernel, dim3(static_cast<uint32_t>(ceil_div(count, 256))), dim3(256), 0, s, prob,
                     alias, rows, pop, count, rng, stream_id, out);
  return hipGetLastError();
}

hipError_t eh_random_walk(const int64_t* indptr, const int32_t* nbr, const float* cumw, int64_t num_rows,
                          int num_types, const uint32_t* step_masks, const int32_t* starts, int64_t n, int walk_len,
                          int32_t default_row, const int64_t* rng, uint64_t stream_id, float p, float q, int32_t* out,
                          hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (!(p > 0.f) || !(q > 0.f)) return hipErrorInvalidValue;
  const int biased = (p != 1.f || q != 1.f) ? 1 : 0;
  hipLaunchKernelGGL(random_walk_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, indptr, nbr,
                     cumw, num_rows, num_types, step_masks, starts, n, walk_len, default_row, rng, stream_id, 1.f / p,
                     1.f / q, biased, out);
  return hipGetLastError();
}

hipError_t eh_synth_degree(int64_t n, float avg_deg, int max_deg, uint64_t seed, int64_t* deg, hipStream_t s) {
  hipLaunchKernelGGL(synth_degree_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, n,
                     avg_deg, max_deg, seed, deg);
  return hipGetLastError();
}

hipError_t eh_synth_fill(int64_t n, const int64_t* indptr, uint64_t seed, int32_t* nbr, float* cumw,
                         hipStream_t s) {
  hipLaunchKernelGGL(synth_fill_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, n, indptr,
                     seed, nbr, cumw);
  return hipGetLastError();
}

}  // extern "C"
