// K8: GPU unique with inverse indices, first-occurrence order (the
// semantics of tf.unique that every reference dataflow relies on: the previous hop's
// nodes keep their leading positions, neighbor_dataflow.py:96, sage_dataflow.py:49;
// engine ID_UNIQUE id_unique_op.cc:35-103).
//
// Open-addressing hash table in HBM (capacity = power of two >= 2n, linear probing,
// 64-bit CAS on the key slot) + an atomicMin of the element position per slot:
//   insert   : slot[i]   = slot of x[i];  minpos[slot] = min position of that key
//   mark     : flag[i]   = (minpos[slot[i]] == i)          (first occurrences)
//   (scan)   : pos       = inclusive prefix sum of flag     (rocPRIM scan via torch)
//   finalize : inv[i]    = pos[minpos[slot[i]]] - 1;  uniq[pos[i] - 1] = x[i] if flag[i]
// O(n) work, no sort.
#include "hip/common.h"
#include "hip/launchers.h"

namespace euler_hip {

constexpr unsigned long long kUniqEmpty = 0x8000000000000000ull;  // INT64_MIN: never a node id

__device__ __forceinline__ uint64_t fmix64(uint64_t k) {
  k ^= k >> 33;
  k *= 0xff51afd7ed558ccdull;
  k ^= k >> 33;
  k *= 0xc4ceb9fe1a85ec53ull;
  k ^= k >> 33;
  return k;
}

// empty table: keys = kUniqEmpty, minpos = INT32_MAX (one launch for both arrays)
__global__ __launch_bounds__(256) void unique_init_kernel(unsigned long long* __restrict__ keys,
                                                          int32_t* __restrict__ minpos, int64_t cap) {
  grid_stride(cap, [&](int64_t i) {
    keys[i] = kUniqEmpty;
    minpos[i] = 0x7fffffff;
  });
}

__global__ __launch_bounds__(256) void unique_insert_kernel(const int64_t* __restrict__ x, int64_t n,
                                                            unsigned long long* __restrict__ keys,
                                                            int32_t* __restrict__ minpos, int64_t cap,
                                                            int32_t* __restrict__ slot, int skip_neg) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  if (skip_neg && x[i] < 0) {  // padding ("no id"): not a key, inverse -1
    slot[i] = -1;
    return;
  }
  const unsigned long long k = static_cast<unsigned long long>(x[i]);
  uint64_t h = fmix64(k) & static_cast<uint64_t>(cap - 1);
  // cap >= 2n guarantees a free slot; the probe count is bounded by cap.  Repeated keys
  // (hub nodes) must not serialise on one address: a plain load finds a present key
  // without a CAS, and the position atomic is skipped once an earlier occurrence holds the
  // slot.  Padding ids (skip_neg: 67K copies of -1 in a sharded-feature exchange, all
  // inserted at once, 434 us of same-address CAS: profiles/r3_headline/shard_prof) never
  // reach the table.
  const volatile unsigned long long* vkeys = keys;
  const volatile int32_t* vmin = minpos;
  for (int64_t probe = 0; probe < cap; ++probe) {
    const unsigned long long cur = vkeys[h];
    bool mine = cur == k;
    if (!mine && cur == kUniqEmpty) {
      const unsigned long long prev = atomicCAS(keys + h, kUniqEmpty, k);
      mine = prev == kUniqEmpty || prev == k;
    }
    if (mine) {
      if (vmin[h] > static_cast<int32_t>(i)) atomicMin(minpos + h, static_cast<int32_t>(i));
      slot[i] = static_cast<int32_t>(h);
      return;
    }
    h = (h + 1) & static_cast<uint64_t>(cap - 1);
  }
  slot[i] = -1;  // unreachable with cap >= 2n
}

__global__ __launch_bounds__(256) void unique_mark_kernel(int64_t n, const int32_t* __restrict__ slot,
                                                          const int32_t* __restrict__ minpos,
                                                          int32_t* __restrict__ flag) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t s = slot[i];
  flag[i] = (s >= 0 && minpos[s] == static_cast<int32_t>(i)) ? 1 : 0;
}

__global__ __launch_bounds__(256) void unique_finalize_kernel(const int64_t* __restrict__ x, int64_t n,
                                                              const int32_t* __restrict__ slot,
                                                              const int32_t* __restrict__ minpos,
                                                              const int32_t* __restrict__ flag,
                                                              const int32_t* __restrict__ pos,
                                                              int64_t* __restrict__ inv, int64_t* __restrict__ uniq,
                                                              int64_t offset) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t s = slot[i];
  inv[i] = s >= 0 ? static_cast<int64_t>(pos[minpos[s]]) - 1 : -1;
  if (flag[i]) uniq[pos[i] - 1] = x[i] + offset;
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

hipError_t eh_unique_init(void* keys, int32_t* minpos, int64_t cap, hipStream_t s) {
  if (cap <= 0) return hipSuccess;
  hipLaunchKernelGGL(unique_init_kernel, grid_for(cap), dim3(256), 0, s, static_cast<unsigned long long*>(keys), minpos,
                     cap);
  return hipGetLastError();
}

hipError_t eh_unique_insert(const int64_t* x, int64_t n, void* keys, int32_t* minpos, int64_t cap, int32_t* slot,
                            int skip_neg, hipStream_t s) {
  if (n == 0) return hipSuccess;
  if (cap < 2 * n || (cap & (cap - 1)) != 0 || n >= (1ll << 31)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(unique_insert_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, x, n,
                     static_cast<unsigned long long*>(keys), minpos, cap, slot, skip_neg);
  return hipGetLastError();
}

hipError_t eh_unique_mark(int64_t n, const int32_t* slot, const int32_t* minpos, int32_t* flag, hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(unique_mark_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, n, slot,
                     minpos, flag);
  return hipGetLastError();
}

hipError_t eh_unique_finalize(const int64_t* x, int64_t n, const int32_t* slot, const int32_t* minpos,
                              const int32_t* flag, const int32_t* pos, int64_t* inv, int64_t* uniq, int64_t offset,
                              hipStream_t s) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(unique_finalize_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, x, n,
                     slot, minpos, flag, pos, inv, uniq, offset);
  return hipGetLastError();
}

}  // extern "C"
