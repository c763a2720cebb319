// Owner routing of the fixed-capacity all-to-all exchanges (parallel/sparse_table.py
// lookup_static, graph/sharded_features.py): every id goes to the slot owner * C + r of
// the W * C exchange space, r = its rank among this rank's ids of the same owner in input
// order (stable, deterministic); ids that do not fit (r >= C) or are < 0 go to the trash
// slot W * C.  Replaces a sort by owner + a dozen index ops (~350 us per DeepWalk step at
// 700K ids, profiles/r2_mid/deepwalk_modes) with two passes over the ids:
//   count : per 2048-id chunk, ids per owner (LDS atomics)
//   scan  : per owner, the exclusive prefix of its counts over the chunks (in place): a
//           chunk's base for an owner is one load, not a sum over every earlier chunk (that
//           grew with the square of the chunk count)
//   place : per chunk, the owners' bases from the scan; then 8 rounds of 256 ids in order:
//           per wave and owner a ballot gives the lane prefix and the wave count, waves are
//           combined through LDS, the running count carries on.
// Owners W <= 63 (a ballot per owner bin per round).
// self_rank >= 0: the caller's own block goes LAST and the peers' blocks keep rank order
// (block of owner o: o < self ? o : o > self ? o - 1 : W - 1), so the peers' slots are one
// contiguous prefix that an uneven-split all-to-all sends as it is, and the caller's own
// ids never travel through the collective (no self-copy); self_rank < 0: block = owner.
#include "hip/common.h"
#include "hip/launchers.h"

namespace euler_hip {

constexpr int kRouteThreads = 256, kRouteRounds = 8, kRouteChunk = kRouteThreads * kRouteRounds;
constexpr int kRouteMaxBins = 64;  // W owners + the "none" bin

__device__ __forceinline__ int route_bin(int64_t id, int W) {
  return id >= 0 ? static_cast<int>(id % W) : W;
}

__global__ __launch_bounds__(kRouteThreads) void route_count_kernel(const int64_t* __restrict__ ids, int64_t n,
                                                                     int W, int32_t* __restrict__ cnt) {
  __shared__ int32_t c[kRouteMaxBins];
  const int NB = W + 1;
  if (threadIdx.x < NB) c[threadIdx.x] = 0;
  __syncthreads();
  const int64_t base = static_cast<int64_t>(blockIdx.x) * kRouteChunk;
  for (int r = 0; r < kRouteRounds; ++r) {
    const int64_t e = base + r * kRouteThreads + threadIdx.x;
    if (e < n) atomicAdd(&c[route_bin(ids[e], W)], 1);
  }
  __syncthreads();
  if (threadIdx.x < NB) cnt[static_cast<int64_t>(blockIdx.x) * NB + threadIdx.x] = c[threadIdx.x];
}

// one block per owner bin: exclusive prefix of cnt[.][q] over the chunks, in place
__global__ __launch_bounds__(kRouteThreads) void route_scan_kernel(int32_t* __restrict__ cnt, int64_t nchunks,
                                                                    int NB) {
  __shared__ int32_t part[kRouteThreads / 64];
  const int q = blockIdx.x, tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  int32_t running = 0;
  for (int64_t t0 = 0; t0 < nchunks; t0 += kRouteThreads) {
    const int64_t k = t0 + tid;
    const int32_t v = k < nchunks ? cnt[k * NB + q] : 0;
    int32_t x = v;  // inclusive wave scan
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
      const int32_t y = __shfl_up(x, o, 64);
      if (lane >= o) x += y;
    }
    if (lane == 63) part[wave] = x;
    __syncthreads();
    int32_t before = running;
    for (int w = 0; w < wave; ++w) before += part[w];
    if (k < nchunks) cnt[k * NB + q] = before + x - v;
    int32_t tile = 0;
    for (int w = 0; w < kRouteThreads / 64; ++w) tile += part[w];
    running += tile;
    __syncthreads();  // part[] is rewritten by the next tile
  }
}

__device__ __forceinline__ int64_t route_block(int b, int W, int self_rank) {
  if (self_rank < 0) return b;
  return b < self_rank ? b : (b > self_rank ? b - 1 : W - 1);
}

__global__ __launch_bounds__(kRouteThreads) void route_place_kernel(const int64_t* __restrict__ ids, int64_t n,
                                                                     int W, int64_t C, int self_rank,
                                                                     const int32_t* __restrict__ cnt,
                                                                     int64_t* __restrict__ pos,
                                                                     int64_t* __restrict__ send,
                                                                     int32_t* __restrict__ overflow) {
  __shared__ int32_t run[kRouteMaxBins];                       // ids placed so far per owner
  __shared__ int32_t wc[kRouteThreads / 64][kRouteMaxBins];    // this round's per-wave counts
  const int NB = W + 1;
  const int tid = threadIdx.x, wave = tid >> 6, lane = tid & 63;
  const int blk = static_cast<int>(blockIdx.x);
  // bases: the earlier chunks' counts of every owner (route_scan_kernel)
  if (tid < NB) run[tid] = cnt[static_cast<int64_t>(blk) * NB + tid];
  const int64_t trash = static_cast<int64_t>(W) * C;
  const uint64_t lt = (lane == 0) ? 0ull : (~0ull >> (64 - lane));
  bool over = false;
  const int64_t base = static_cast<int64_t>(blk) * kRouteChunk;
  for (int r = 0; r < kRouteRounds; ++r) {
    const int64_t e = base + r * kRouteThreads + tid;
    const bool in = e < n;
    const int64_t id = in ? ids[e] : -1;
    const int b = in ? route_bin(id, W) : -1;
    int pre = 0;
    for (int q = 0; q < NB; ++q) {
      const uint64_t m = __ballot(b == q);
      if (b == q) pre = __popcll(m & lt);
      if (lane == 0) wc[wave][q] = __popcll(m);
    }
    __syncthreads();  // bases (first round) and this round's wave counts are complete
    if (in) {
      int r0 = (b >= 0) ? run[b] : 0;
      for (int w = 0; w < wave; ++w) r0 += wc[w][b];
      const int64_t rank = r0 + pre;
      int64_t d = trash;
      if (b < W) {
        if (rank < C) {
          d = route_block(b, W, self_rank) * C + rank;
          send[d] = id;
        } else {
          over = true;
        }
      }
      pos[e] = d;
    }
    __syncthreads();  // every id of the round read run[]
    if (tid < NB) {
      int s = 0;
      for (int w = 0; w < kRouteThreads / 64; ++w) s += wc[w][tid];
      run[tid] += s;
    }
    __syncthreads();
  }
  if (over) overflow[0] = 1;
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

int64_t eh_route_chunks(int64_t n) { return ceil_div(n, kRouteChunk); }

hipError_t eh_route_by_owner(const int64_t* ids, int64_t n, int W, int64_t C, int self_rank, int32_t* cnt,
                             int64_t* pos, int64_t* send, int32_t* overflow, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (W < 1 || W + 1 > kRouteMaxBins || C < 1 || self_rank >= W) return hipErrorInvalidValue;
  const uint32_t nb = static_cast<uint32_t>(ceil_div(n, kRouteChunk));
  hipLaunchKernelGGL(route_count_kernel, dim3(nb), dim3(kRouteThreads), 0, s, ids, n, W, cnt);
  hipLaunchKernelGGL(route_scan_kernel, dim3(static_cast<uint32_t>(W + 1)), dim3(kRouteThreads), 0, s, cnt,
                     static_cast<int64_t>(nb), W + 1);
  hipLaunchKernelGGL(route_place_kernel, dim3(nb), dim3(kRouteThreads), 0, s, ids, n, W, C, self_rank, cnt, pos,
                     send, overflow);
  return hipGetLastError();
}

}  // extern "C"
