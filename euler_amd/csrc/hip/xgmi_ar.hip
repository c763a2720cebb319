// Two-shot all-reduce over xGMI peer memory for the data-parallel gradient sync.
//
// The headline step's gradient is small (278 K parameters: 1.12 MB fp32 / 0.56 MB bf16), so a
// ring all-reduce is latency-bound: 2 (W - 1) dependent hops, each a flag round trip on one
// xGMI link.  MI355X's xGMI is point-to-point (every GPU has a direct link to each of its 7
// peers), so a rank can read every peer's memory directly and the whole reduction takes two
// phases with one cross-GPU barrier each:
//
//   A  stage: copy the local gradient into this rank's IPC buffer `in` (uncached HBM);
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
// Memory model: `in`, `out` and the flags live in one hipDeviceMallocUncached allocation per
// rank, exported with hipIpcGetMemHandle and mapped by the peers; data stores are followed by
// a system-scope fence in every thread before the block barrier, flags are written with
// system-scope release stores and polled with system-scope acquire loads.  Every wait is
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
constexpr int64_t kArHeader = 4096;  // flags, padded so `in` starts 4 KiB aligned
static_assert(kArSigBytes <= kArHeader, "flag area exceeds the header");

struct ArArgs {
  char* buf[kArMaxRanks];  // every rank's buffer (own included), identical layout
  void* data;              // local tensor: input and output, n elements
  int64_t n;               // elements; a multiple of the 16-byte vector width
  int64_t shard;           // elements per rank's shard (multiple of the vector width)
  int64_t cap;             // bytes of each of `in` and `out`
  int rank, world;
  uint32_t* epoch;         // [gridDim.x] call counters (this rank, ordinary memory)
  int* err;                // set to 1 by a wait that timed out
  long long timeout;       // wall_clock64 ticks per wait
};

__device__ __forceinline__ uint32_t* ar_sig(char* buf, int which, int b, int r) {
  return reinterpret_cast<uint32_t*>(buf) + (which * kArMaxBlocks + b) * kArMaxRanks + r;
}

// thread t < world signals peer t; then thread t < world waits for peer t's signal
__device__ __forceinline__ void ar_barrier(const ArArgs& a, int which, uint32_t e) {
  const int t = threadIdx.x, b = blockIdx.x;
  // every thread's stores of this phase are visible at system scope before any signal leaves
  __threadfence_system();
  __syncthreads();
  if (t < a.world) {
    __hip_atomic_store(ar_sig(a.buf[t], which, b, a.rank), e, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_SYSTEM);
    const uint32_t* f = ar_sig(a.buf[a.rank], which, b, t);
    const long long t0 = wall_clock64();
    while (__hip_atomic_load(f, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_SYSTEM) < e) {
      if (__hip_atomic_load(a.err, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) != 0) break;
      if (wall_clock64() - t0 > a.timeout) {
        __hip_atomic_store(a.err, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        break;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    __atomic_thread_fence(__ATOMIC_ACQUIRE);  // system scope: the peers' data after their flags
  }
  __syncthreads();
  __threadfence_system();
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
  const int64_t step = static_cast<int64_t>(G) * kArThreads * V;  // elements per grid sweep of a shard
  const int64_t first = (static_cast<int64_t>(b) * kArThreads + t) * V;
  auto shard_len = [&](int s) {
    const int64_t lo = s * a.shard;
    const int64_t hi = lo + a.shard < a.n ? lo + a.shard : a.n;
    return hi > lo ? hi - lo : int64_t{0};
  };
  uint4_t* data = reinterpret_cast<uint4_t*>(a.data);
  auto in_of = [&](int r) { return reinterpret_cast<uint4_t*>(a.buf[r] + kArHeader); };
  auto out_of = [&](int r) { return reinterpret_cast<uint4_t*>(a.buf[r] + kArHeader + a.cap); };

  // A: stage this rank's input (the chunks block b owns in every shard)
  uint4_t* my_in = in_of(a.rank);
  for (int s = 0; s < a.world; ++s) {
    const int64_t len = shard_len(s), base = s * a.shard;
    for (int64_t o = first; o < len; o += step) my_in[(base + o) / V] = data[(base + o) / V];
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
        if (r < a.world) v[r] = in_of(r)[vi];  // one load per link in flight
      float acc[V];
#pragma unroll
      for (int i = 0; i < V; ++i) acc[i] = 0.f;
#pragma unroll
      for (int r = 0; r < kArMaxRanks; ++r)
        if (r < a.world) ArVec<T>::add(acc, v[r]);
      const uint4_t res = ArVec<T>::pack(acc);
      my_out[vi] = res;
      data[vi] = res;
    }
  }
  ar_barrier(a, 1, e);

  // D: gather every other rank's reduced shard
  for (int s = 0; s < a.world; ++s) {
    if (s == a.rank) continue;
    const int64_t len = shard_len(s), base = s * a.shard;
    const uint4_t* src = out_of(s);
    for (int64_t o = first; o < len; o += step) data[(base + o) / V] = src[(base + o) / V];
  }
  if (t == 0) a.epoch[b] = e;
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

int64_t eh_xar_header_bytes() { return kArHeader; }
int eh_xar_max_ranks() { return kArMaxRanks; }
int eh_xar_max_blocks() { return kArMaxBlocks; }

// one rank's buffer: flags + in + out, uncached (coherent across the xGMI peers), zeroed
hipError_t eh_xar_alloc(int64_t cap, void** out) {
  const size_t bytes = static_cast<size_t>(kArHeader + 2 * cap);
  hipError_t e = hipExtMallocWithFlags(out, bytes, hipDeviceMallocUncached);
  if (e != hipSuccess) return e;
  e = hipMemset(*out, 0, bytes);
  if (e != hipSuccess) return e;
  return hipDeviceSynchronize();
}

// bufs: world pointers (this rank's own and the mapped peers'); blocks <= kArMaxBlocks
hipError_t eh_xar_run(void* const* bufs, int world, int rank, void* data, int is_bf16, int64_t n, int64_t cap,
                      int blocks, uint32_t* epoch, int* err, long long timeout, hipStream_t s) {
  if (world < 1 || world > kArMaxRanks || rank < 0 || rank >= world || blocks < 1 || blocks > kArMaxBlocks ||
      !data || !epoch || !err || n < 0)
    return hipErrorInvalidValue;
  const int V = is_bf16 ? 8 : 4;
  const int64_t esz = is_bf16 ? 2 : 4;
  if (n % V != 0 || n * esz > cap) return hipErrorInvalidValue;
  if (reinterpret_cast<uintptr_t>(data) % 16 != 0) return hipErrorInvalidValue;
  ArArgs a{};
  for (int r = 0; r < world; ++r) {
    if (!bufs[r]) return hipErrorInvalidValue;
    a.buf[r] = static_cast<char*>(bufs[r]);
  }
  a.data = data;
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
