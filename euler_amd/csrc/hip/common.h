// Shared device helpers for the euler_amd CDNA4 (gfx950) kernels.
//
// Conventions used by every kernel in this directory:
//   * wave64 everywhere: lane = threadIdx.x & 63, block sizes are multiples of 64;
//   * bf16 storage / fp32 accumulation; bf16 moved as 16-byte vectors (8 elems);
//   * launchers are plain C++ functions taking raw device pointers + hipStream_t,
//     so they can be captured into hipGraphs by the caller (no allocation, no sync).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace euler_hip {

using bf16_t = uint16_t;  // raw bf16 bits
typedef float float4_t __attribute__((ext_vector_type(4)));
typedef float float16_t __attribute__((ext_vector_type(16)));
typedef short short8_t __attribute__((ext_vector_type(8)));
typedef uint32_t uint4_t __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf2f(bf16_t v) {
  return __uint_as_float(static_cast<uint32_t>(v) << 16);
}

typedef float cm_float2_t __attribute__((ext_vector_type(2)));
typedef __bf16 cm_bf16x2_t __attribute__((ext_vector_type(2)));

// round-to-nearest-even fp32 pair -> packed bf16 (one v_cvt_pk_bf16_f32 on gfx950)
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(uint32_t, __builtin_convertvector(cm_float2_t{a, b}, cm_bf16x2_t));
}

__device__ __forceinline__ bf16_t f2bf(float f) { return static_cast<bf16_t>(pack_bf16x2(f, 0.f)); }

// unpack 8 bf16 held in a 16-byte vector into fp32 and add to acc[8]
__device__ __forceinline__ void acc_bf16x8(float* acc, uint4_t v, float scale = 1.f) {
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    acc[2 * i] += scale * __uint_as_float(v[i] << 16);
    acc[2 * i + 1] += scale * __uint_as_float(v[i] & 0xffff0000u);
  }
}

__device__ __forceinline__ uint4_t pack_bf16x8(const float* a) {
  uint4_t r;
#pragma unroll
  for (int i = 0; i < 4; ++i) r[i] = pack_bf16x2(a[2 * i], a[2 * i + 1]);
  return r;
}

// ---------------------------------------------------------------------------
// Philox4x32-10 counter-based RNG.  Every random draw is a pure function of
// (seed, counter, subsequence) so sampling is reproducible per
// (global seed, step, rank, element) — fixes the reference's time(0)-seeded
// thread-local engines (reference: euler/common/random.cc:21-28).
// ---------------------------------------------------------------------------
struct Philox {
  __device__ __forceinline__ static void round(uint32_t& c0, uint32_t& c1, uint32_t& c2, uint32_t& c3,
                                               uint32_t k0, uint32_t k1) {
    const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
    uint32_t hi0 = __umulhi(M0, c0), lo0 = M0 * c0;
    uint32_t hi1 = __umulhi(M1, c2), lo1 = M1 * c2;
    uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
  }
  // returns 4 uniform 32-bit words for (seed, ctr_hi, ctr_lo)
  __device__ __forceinline__ static uint4_t gen(uint64_t seed, uint64_t hi, uint64_t lo) {
    uint32_t c0 = static_cast<uint32_t>(lo), c1 = static_cast<uint32_t>(lo >> 32);
    uint32_t c2 = static_cast<uint32_t>(hi), c3 = static_cast<uint32_t>(hi >> 32);
    uint32_t k0 = static_cast<uint32_t>(seed), k1 = static_cast<uint32_t>(seed >> 32);
#pragma unroll
    for (int r = 0; r < 10; ++r) {
      round(c0, c1, c2, c3, k0, k1);
      k0 += 0x9E3779B9u;
      k1 += 0xBB67AE85u;
    }
    uint4_t out;
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
    return out;
  }
};

// uniform float in [0, 1) from 32 random bits (24-bit mantissa)
__device__ __forceinline__ float u01(uint32_t x) { return (x >> 8) * (1.0f / 16777216.0f); }

__host__ __device__ __forceinline__ int64_t ceil_div(int64_t a, int64_t b) { return (a + b - 1) / b; }

// One-thread-per-item kernels over possibly more than 2^32 items (an [E, 128] message
// tensor of a 50M-edge graph has 6.4e9 elements): a dispatch counts its work-items in 32
// bits, so a grid of ceil(n / 256) blocks would wrap and silently drop most of the items.
// Launch grid_for(n) (capped) and loop with grid_stride inside the kernel.
constexpr int64_t kMaxGridBlocks = int64_t{1} << 22;  // 2^30 work-items per dispatch
inline dim3 grid_for(int64_t n, int threads = 256) {
  const int64_t b = ceil_div(n, threads);
  return dim3(static_cast<uint32_t>(b < kMaxGridBlocks ? (b > 0 ? b : 1) : kMaxGridBlocks));
}
template <typename F>
__device__ __forceinline__ void grid_stride(int64_t n, F&& f) {
  const int64_t step = static_cast<int64_t>(gridDim.x) * blockDim.x;
  for (int64_t t = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x; t < n; t += step) f(t);
}

// XCD-aware bijective block remap (cdna_hip_programming.md §5 "XCD swizzle must
// be bijective"): consecutive logical tiles land on the same XCD / L2.
__device__ __forceinline__ int xcd_remap(int orig, int nwg) {
  const int q = nwg / 8, r = nwg % 8;
  const int xcd = orig % 8;
  return (xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q) + orig / 8;
}

}  // namespace euler_hip

#define EULER_HIP_CHECK(expr)                                                            \
  do {                                                                                   \
    hipError_t _e = (expr);                                                              \
    if (_e != hipSuccess) return _e;                                                     \
  } while (0)
