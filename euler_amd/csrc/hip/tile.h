// MFMA tile helpers shared by the fused GraphSAGE kernels (sage_tree.hip).
//
// Two operand layouts make every MFMA operand load a single 16-byte vector:
//   * "kt" (k-tiled) X_kt[M/32][N][32]: the reduction index m of a weight-gradient
//     GEMM dW = G^T X is contiguous, so lane l's fragment (8 consecutive m at column
//     l & 15) is one load and no LDS transpose is needed;
//   * "fm" (fragment-major) Wf[N/16][K/32][64 lanes][8] for bf16 weight shadows used as
//     B operands: the fragment of (16-column slab, 32-deep k step) is one contiguous
//     1 KB, fully coalesced across the wave.
// gfx950 mfma_f32_16x16x32_bf16 lane maps: A[row l&15][k 8(l>>4)+j], B[k 8(l>>4)+j][col
// l&15], C/D col = l&15, row = (l>>4)*4 + reg.
#pragma once
#include "hip/common.h"

namespace euler_hip {

typedef __bf16 tl_bf16x8 __attribute__((ext_vector_type(8)));
typedef uint32_t tl_uint2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float4_t mfma16(uint4_t a, uint4_t b, float4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(__builtin_bit_cast(tl_bf16x8, a), __builtin_bit_cast(tl_bf16x8, b),
                                                 c, 0, 0, 0);
}

// element (m, n) of an [M][N] matrix stored k-tiled
__device__ __forceinline__ int64_t kt_off(int64_t m, int64_t n, int64_t N) {
  return ((m >> 5) * N + n) * 32 + (m & 31);
}

// element (n, k) of a weight W[N][K] stored fragment-major
__device__ __forceinline__ int64_t fm_off(int64_t n, int64_t k, int64_t K) {
  return (((n >> 4) * (K >> 5) + (k >> 5)) * 64 + ((k & 31) >> 3) * 16 + (n & 15)) * 8 + (k & 7);
}

// the B fragment of slab n0 (multiple of 16), k step k0 (multiple of 32) for this lane
__device__ __forceinline__ uint4_t fm_frag(const bf16_t* __restrict__ Wf, int n0, int k0, int K, int lane) {
  return *reinterpret_cast<const uint4_t*>(Wf +
                                           ((static_cast<int64_t>(n0 >> 4) * (K >> 5) + (k0 >> 5)) * 64 + lane) * 8);
}

// MFMA fragment of 16 columns c0.. of a row-major bf16 LDS image [rows][LD] whose rows are
// the reduction index (k-major operands: dW = G^T X, C = A^T B), via the gfx950 transposing
// read ds_read_b64_tr_b16: a 16-lane group reads a 4-row x 16-column block and lane i gets
// column i.  Lane group g holds rows e0 + 4g .. +3 and e0 + 16 + 4g .. +3 (the same row map
// for both operands, which is all the MFMA needs).  LD = 80 or 144 halfwords keeps the 8
// rows a 32-lane half reads on disjoint bank sets.
typedef short tl_v4i16 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) tl_v4i16 tl_lds_v4i16;

template <int LD>
__device__ __forceinline__ uint4_t tl_tr_frag(const bf16_t* img, int e0, int c0, int lane) {
  const int g = lane >> 4, i = lane & 15;
  const bf16_t* a = img + (e0 + 4 * g + (i >> 2)) * LD + c0 + 4 * (i & 3);
  const tl_v4i16 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tl_lds_v4i16*)(a));
  const tl_v4i16 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((tl_lds_v4i16*)(a + 16 * LD));
  const tl_uint2 l2 = __builtin_bit_cast(tl_uint2, lo), h2 = __builtin_bit_cast(tl_uint2, hi);
  return uint4_t{l2[0], l2[1], h2[0], h2[1]};
}

__device__ __forceinline__ bool bf_pos(bf16_t v) { return (v & 0x8000u) == 0 && (v & 0x7fffu) != 0; }

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

__device__ __forceinline__ int wave_sum_i(int v) {
#pragma unroll
  for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

template <int FM, int FN>
__device__ __forceinline__ void tl_zero(float4_t (&acc)[FM][FN]) {
#pragma unroll
  for (int m = 0; m < FM; ++m)
#pragma unroll
    for (int n = 0; n < FN; ++n) acc[m][n] = float4_t{0.f, 0.f, 0.f, 0.f};
}

// 4 consecutive rows (j = 0..3) of one column into a kt matrix: one 8-byte store
__device__ __forceinline__ void kt_store4(bf16_t* kt, int64_t row, int col, int N, float a, float b, float c,
                                          float d) {
  tl_uint2 v;
  v[0] = pack_bf16x2(a, b);
  v[1] = pack_bf16x2(c, d);
  *reinterpret_cast<tl_uint2*>(kt + kt_off(row, col, N)) = v;
}

}  // namespace euler_hip
