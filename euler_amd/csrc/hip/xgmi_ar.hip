// Two-shot all-reduce over xGMI peer memory for the data-parallel gradient sync.
//
// The headline step's gradient is small (278 K parameters: 1.12 MB fp32 / 0.56 MB bf16), so a
// ring all-reduce is latency-bound: 2 (W - 1) dependent hops, each a flag round trip on one
// xGMI link.  MI355X's xGMI is point-to-point (every GPU has a direct link to each of its 7
// peers), so a rank can read every peer's memory directly and the whole reduction takes two
// phases with one cross-GPU barrier each:
//
//   A  stage: copy the local gradient into this rank's IPC buffer `in`;
//      barrier 1 (every block b signals block b of every peer, waits for all of them)
//   B  reduce-scatter: rank r sums shard r of every peer's `in` (7 remote reads in flight per
//      thread, one per link, fp32 accumulation) and writes it to `out` (and the local result);
//      barrier 2
//   D  all-gather: rank r reads shard s of peer s's `out` for every s != r.
//
// Each link carries 2 x (bytes / W) per rank instead of the ring's 2 (W - 1) / W x bytes
// serialised over W - 1 steps, and there are two barriers instead of 2 (W - 1) hops.
// Block b of every rank touches the same element chunks in every phase, so the barriers are
// per block (no grid-wide sync) and every block's waits depend only on block b of the peers.
//
// Memory model: per rank, the flags live in a small hipDeviceMallocUncached allocation and
// `in` / `out` in ordinary HBM (XAR_UNCACHED_DATA=1 puts them in uncached memory too, which
// measured ~25 us per one-rank call: profiles/r3_xgmi/); both are exported with
// hipIpcGetMemHandle and mapped by the peers.  Data stores are followed by a system-scope
// drain (vmcnt) in every wave and a block barrier, then one system-scope release store per
// peer from wave 0 (its L2 write-back makes the block's data visible over xGMI); flags are
// polled with system-scope loads and wave 0's system-scope acquire invalidates stale lines
// before the block reads the peers' data.  Every wait is
// bounded (wall clock); a timeout sets the error word and lets the grid drain, so a lost peer
// can never hang the GPU — the caller checks error() and falls back to RCCL.
//
// Epochs: block b keeps a private call counter; call k signals k (flags only grow), so the
// same buffers serve every call, also inside a hipGraph replayed any number of times.
//
// Reference: the reference's between-graph data parallelism all-reduces gradients through
// TF's collective ops (tf_euler/scripts/dist_tf_euler.sh:1-49,
// euler_estimator/python/base_estimator.py:164); this is the MI355X-native replacement for
// that gradient sync on one node.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "common.h"

namespace euler_hip {

constexpr int kArMaxRanks = 8;
constexpr int kArMaxBlocks = 64;
constexpr int kArThreads = 256;
constexpr int64_t kArSigBytes = 2 * kArMaxBlocks * kArMaxRanks * sizeof(uint32_t);
constexpr int kArVecPerThread = 4;  // 16-byte vectors per thread per shard sweep
#ifndef XAR_UNCACHED_DATA
#define XAR_UNCACHED_DATA 0
#endif

struct ArArgs {
  char* sig[kArMaxRanks];  // every rank's flag area (own included)
  char* buf[kArMaxRanks];  // every rank's data area: in [cap] then out [cap]
  void* data;              // local tensor: input and output, n elements
  int64_t n;               // elements; a multiple of the 16-byte vector width
  int64_t shard;           // elements per rank's shard (multiple of the vector width)
  int64_t cap;             // bytes of each of `in` and `out`
  int rank, world;
  int64_t in_off;          // >= 0: data IS this rank's `in` region at this byte offset (the
                           // producer wrote it there: no staging copy); -1: stage it
  uint32_t* epoch;         // [gridDim.x] call counters (this rank, ordinary memory)
  int* err;                // set to 1 by a wait that timed out
  long long timeout;       // wall_clock64 ticks per wait
};

__device__ __forceinline__ uint32_t* ar_sig(char* sig, int which, int b, int r) {
  return reinterpret_cast<uint32_t*>(sig) + (which * kArMaxBlocks + b) * kArMaxRanks + r;
}

// XAR_WT=1: the exchanged data never sits in an L2 — staged / reduced vectors are written
// with system-scope (write-through) stores and the peers' vectors read with system-scope
// loads — so a barrier needs neither the L2 write-back before the signal nor the
// invalidation after the wait: every wave drains its stores (vmcnt(0)), the flags are
// relaxed system-scope atomics.
#ifndef XAR_WT
#define XAR_WT 0
#endif
__device__ __forceinline__ void st_x(uint4_t* p, uint4_t v) {
  if (XAR_WT) {
    uint64_t* q = reinterpret_cast<uint64_t*>(p);
    __hip_atomic_store(q, (static_cast<uint64_t>(v[1]) << 32) | v[0], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    __hip_atomic_store(q + 1, (static_cast<uint64_t>(v[3]) << 32) | v[2], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_SYSTEM);
  } else {
    *p = v;
  }
}
__device__ __forceinline__ uint4_t ld_x(const uint4_t* p) {
  if (XAR_WT) {
    const uint64_t* q = reinterpret_cast<const uint64_t*>(p);
    const uint64_t a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint64_t b = __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM);
    uint4_t v;
    v[0] = static_cast<uint32_t>(a);
    v[1] = static_cast<uint32_t>(a >> 32);
    v[2] = static_cast<uint32_t>(b);
    v[3] = static_cast<uint32_t>(b >> 32);
    return v;
  }
  return *p;
}

// thread t < world (lanes of wave 0) signals peer t, then waits for peer t's signal.  The
// other waves only drain their own stores (vmcnt(0)) before the block barrier: wave 0's
// system-scope release (one L2 write-back) then covers the whole block's stores, and its
// system-scope acquire (one cache invalidation) covers the whole block's later loads.
// XAR_FENCE_ALL=1: every thread fences at system scope on both sides instead (measured).
#ifndef XAR_FENCE_ALL
#define XAR_FENCE_ALL 0
#endif
__device__ __forceinline__ void ar_barrier(const ArArgs& a, int which, uint32_t e) {
  const int t = threadIdx.x, b = blockIdx.x;
  if (XAR_FENCE_ALL) __threadfence_system();
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (t < a.world) {
    __hip_atomic_store(ar_sig(a.sig[t], which, b, a.rank), e, XAR_WT ? __ATOMIC_RELAXED : __ATOMIC_RELEASE,
                       __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* f = ar_sig(a.sig[a.rank], which, b, t);
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
      if (wall_clock64() - t0 > a.timeout) {
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    if (!XAR_WT) __atomic_thread_fence(__ATOMIC_ACQUIRE);  // system scope: the peers' data after their flags
  }
  __syncthreads();
  if (XAR_FENCE_ALL) __threadfence_system();
}

template <typename T>
struct ArVec;
template <>
struct ArVec<float> {
  static constexpr int V = 4;
  __device__ static void add(float* acc, uint4_t v) {
#pragma unroll
    for (int i = 0; i < 4; ++i) acc[i] += __uint_as_float(v[i]);
  }
  __device__ static uint4_t pack(const float* acc) {
    uint4_t r;
#pragma unroll
    for (int i = 0; i < 4; ++i) r[i] = __float_as_uint(acc[i]);
    return r;
  }
};
template <>
struct ArVec<bf16_t> {
  static constexpr int V = 8;
  __device__ static void add(float* acc, uint4_t v) { acc_bf16x8(acc, v); }
  __device__ static uint4_t pack(const float* acc) { return pack_bf16x8(acc); }
};

template <typename T>
__global__ __launch_bounds__(kArThreads) void xgmi_allreduce_kernel(ArArgs a) {
  constexpr int V = ArVec<T>::V;
  const int b = blockIdx.x, G = gridDim.x, t = threadIdx.x;
  __shared__ uint32_t e_s;
  if (t == 0) e_s = a.epoch[b] + 1;
  __syncthreads();
  const uint32_t e = e_s;
  // block b owns vectors [b * kArThreads + t] + k * G * kArThreads of every shard
  const int64_t step = static_cast<int64_t>(G) * kArThreads * V;  // elements per grid sweep of a shard
  const int64_t first = (static_cast<int64_t>(b) * kArThreads + t) * V;
  auto shard_len = [&](int s) {
    const int64_t lo = s * a.shard;
    const int64_t hi = lo + a.shard < a.n ? lo + a.shard : a.n;
    return hi > lo ? hi - lo : int64_t{0};
  };
  uint4_t* __restrict__ data = reinterpret_cast<uint4_t*>(a.data);
  const int64_t in_off = a.in_off > 0 ? a.in_off : 0;
  auto in_of = [&](int r) { return reinterpret_cast<uint4_t*>(a.buf[r] + in_off); };
  auto out_of = [&](int r) { return reinterpret_cast<uint4_t*>(a.buf[r] + a.cap + in_off); };

  // A: stage this rank's input (the chunks block b owns in every shard); every load of a
  // sweep is issued before its stores.  In place (in_off >= 0) the producer kernel already
  // wrote it into the IPC region, and the kernel boundary wrote it back to memory.
  uint4_t* __restrict__ my_in = in_of(a.rank);
  for (int s = 0; s < (a.in_off >= 0 ? 0 : a.world); ++s) {
    const int64_t len = shard_len(s), base = s * a.shard;
    for (int64_t o0 = first; o0 < len; o0 += kArVecPerThread * step) {
      uint4_t v[kArVecPerThread];
#pragma unroll
      for (int k = 0; k < kArVecPerThread; ++k)
        if (o0 + k * step < len) v[k] = data[(base + o0 + k * step) / V];
#pragma unroll
      for (int k = 0; k < kArVecPerThread; ++k)
        if (o0 + k * step < len) st_x(&my_in[(base + o0 + k * step) / V], v[k]);
    }
  }
  ar_barrier(a, 0, e);

  // B: reduce this rank's shard over every peer's staged input
  {
    const int64_t len = shard_len(a.rank), base = a.rank * a.shard;
    uint4_t* my_out = out_of(a.rank);
    for (int64_t o = first; o < len; o += step) {
      const int64_t vi = (base + o) / V;
      uint4_t v[kArMaxRanks];
#pragma unroll
      for (int r = 0; r < kArMaxRanks; ++r)
        if (r < a.world) v[r] = ld_x(&in_of(r)[vi]);  // one load per link in flight
      float acc[V];
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
      for (int r = 0; r < kArMaxRanks; ++r)
        if (r < a.world) ArVec<T>::add(acc, v[r]);
      const uint4_t res = ArVec<T>::pack(acc);
      st_x(&my_out[vi], res);
      data[vi] = res;
    }
  }
  ar_barrier(a, 1, e);

  // D: gather every other rank's reduced shard (all loads of a sweep in flight)
  for (int64_t o0 = first; o0 < a.shard; o0 += kArVecPerThread * step) {
    uint4_t v[kArVecPerThread][kArMaxRanks];
#pragma unroll
    for (int k = 0; k < kArVecPerThread; ++k)
#pragma unroll
      for (int s = 0; s < kArMaxRanks; ++s)
        if (s < a.world && s != a.rank && o0 + k * step < shard_len(s))
          v[k][s] = ld_x(&out_of(s)[(s * a.shard + o0 + k * step) / V]);
#pragma unroll
    for (int k = 0; k < kArVecPerThread; ++k)
#pragma unroll
      for (int s = 0; s < kArMaxRanks; ++s)
        if (s < a.world && s != a.rank && o0 + k * step < shard_len(s))
          data[(s * a.shard + o0 + k * step) / V] = v[k][s];
  }
  if (t == 0) a.epoch[b] = e;
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

int eh_xar_max_ranks() { return kArMaxRanks; }
int eh_xar_max_blocks() { return kArMaxBlocks; }
int eh_xar_vec_per_thread() { return kArVecPerThread; }

// one rank's flag area (uncached: polled across the xGMI peers) and data area (in + out,
// ordinary HBM unless XAR_UNCACHED_DATA), both zeroed
hipError_t eh_xar_alloc(int64_t cap, void** sig, void** data) {
  hipError_t e = hipExtMallocWithFlags(sig, static_cast<size_t>(kArSigBytes), hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  if ((e = hipMemset(*sig, 0, static_cast<size_t>(kArSigBytes))) != hipSuccess) return e;
  const size_t bytes = static_cast<size_t>(2 * cap);
  e = XAR_UNCACHED_DATA ? hipExtMallocWithFlags(data, bytes, hipDeviceMallocUncached) : hipMalloc(data, bytes);
  if (e != hipSuccess) return e;
  if ((e = hipMemset(*data, 0, bytes)) != hipSuccess) return e;
  return hipDeviceSynchronize();
}

// sigs / bufs: world pointers (this rank's own and the mapped peers'); blocks <= kArMaxBlocks
// data inside this rank's `in` region (bufs[rank] .. + cap): the all-reduce runs in place
// there, and every rank must pass the same offset (same tensor slicing on every rank)
hipError_t eh_xar_run(void* const* sigs, void* const* bufs, int world, int rank, void* data, int is_bf16, int64_t n,
                      int64_t cap, int blocks, uint32_t* epoch, int* err, long long timeout, hipStream_t s) {
  if (world < 1 || world > kArMaxRanks || rank < 0 || rank >= world || blocks < 1 || blocks > kArMaxBlocks ||
      !data || !epoch || !err || n < 0)
    return hipErrorInvalidValue;
  const int V = is_bf16 ? 8 : 4;
  const int64_t esz = is_bf16 ? 2 : 4;
  if (n % V != 0 || n * esz > cap) return hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(data) % 16 != 0) return hipErrorInvalidValue;
  ArArgs a{};
  for (int r = 0; r < world; ++r) {
    if (!bufs[r] || !sigs[r]) return hipErrorInvalidValue;
    a.buf[r] = static_cast<char*>(bufs[r]);
    a.sig[r] = static_cast<char*>(sigs[r]);
  }
  a.data = data;
  const char* own = static_cast<const char*>(bufs[rank]);
  const char* d = static_cast<const char*>(data);
  a.in_off = (d >= own && d + n * esz <= own + cap) ? static_cast<int64_t>(d - own) : -1;
  a.n = n;
  a.shard = ((n / V + world - 1) / world) * V;
  a.cap = cap;
  a.rank = rank;
  a.world = world;
  a.epoch = epoch;
  a.err = err;
  a.timeout = timeout;
  if (n == 0) return hipSuccess;
  if (is_bf16)
    hipLaunchKernelGGL(xgmi_allreduce_kernel<bf16_t>, dim3(blocks), dim3(kArThreads), 0, s, a);
  else
    hipLaunchKernelGGL(xgmi_allreduce_kernel<float>, dim3(blocks), dim3(kArThreads), 0, s, a);
  return hipGetLastError();
}

}  // extern "C"
