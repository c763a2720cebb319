// Optimizer kernels.
//   flat_adam   : one launch updates every dense parameter of a model whose params
//                 live in one flat fp32 buffer (FlatParams); the step count is a
//                 device scalar so the update is hipGraph-replay safe.
//   sparse_adam : row-sparse Adam/Adagrad on the rows of an embedding shard that
//                 received gradients (ids already de-duplicated by the caller).
// Reference optimizers: tf_euler/python/utils/optimizers.py:22-31 (sgd, momentum,
// adagrad, adam); embedding stores: utils/embedding.py:24-68.
#include "hip/common.h"
#include "hip/launchers.h"
#include "hip/optim_math.h"

namespace euler_hip {

// One optimizer launch over a flat fp32 buffer (p, g, m, v), hipGraph-replay safe.
//   * The Adam step count lives on the device: every block uses t = step + bias (bias 1:
//     this launch advances it), and with a ticket the LAST block to finish stores step + 1
//     and re-arms the ticket — no separate increment launch.  Every block has read the
//     step before it takes its ticket, so none can see the new value.
//   * Weight decay wd, or wd2 on the elements [w0, w1) (a per-parameter-group decay, e.g.
//     only on a model's relation matrices).
struct FlatOptArgs {
  float *p, *m, *v;
  const float* g;
  int64_t n;     // elements
  int64_t base;  // index of element 0 in the whole buffer (decay range)
  int64_t* step;
  int32_t* ticket;  // null: the step is advanced by step_inc_kernel before the launch
  int32_t step_bias, advance;
  float lr, b1, b2, eps, wd, wd2, grad_scale;
  int64_t w0, w1;
  int32_t kind;  // 0 adam, 1 adagrad, 2 sgd, 3 momentum
};

__device__ __forceinline__ float flat_wd(const FlatOptArgs& a, int64_t e) {
  return (e >= a.w0 && e < a.w1) ? a.wd2 : a.wd;
}

// the last block to finish advances the step (see FlatOptArgs)
__device__ __forceinline__ void flat_step_ticket(const FlatOptArgs& a) {
  if (!a.ticket || !a.advance) return;
  __syncthreads();
  if (threadIdx.x == 0) {
    const int prev = atomicAdd(a.ticket, 1);
    if (prev == static_cast<int>(gridDim.x) - 1) {
      a.step[0] += 1;
      *a.ticket = 0;
    }
  }
}

__global__ __launch_bounds__(256) void flat_optim_kernel(FlatOptArgs a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const float t = static_cast<float>(a.step[0] + a.step_bias);
  if (i < a.n) {
    float p = a.p[i], m = a.m[i], v = a.v[i];
    optim_one(p, a.g[i], m, v, t, a.lr, a.b1, a.b2, a.eps, flat_wd(a, a.base + i), a.grad_scale, a.kind);
    a.p[i] = p;
    if (a.kind == 0 || a.kind == 3) a.m[i] = m;
    if (a.kind == 0 || a.kind == 1) a.v[i] = v;
  }
  flat_step_ticket(a);
}

// float4 form: 16-byte loads / stores of p, g, m, v, all four loads issued before the math
// (the update is bandwidth-bound: 28 B per parameter).  a.n counts ELEMENTS; thread i owns
// elements [4i, 4i + 4) and the last thread takes a ragged tail element-wise, so one launch
// covers any length
__global__ __launch_bounds__(256) void flat_optim4_kernel(FlatOptArgs a) {
  const int64_t i = static_cast<int64_t>(blockIdx.x) * blockDim.x + threadIdx.x;
  const float t = static_cast<float>(a.step[0] + a.step_bias);
  if (4 * i + 4 <= a.n) {
    float4_t pv = reinterpret_cast<float4_t*>(a.p)[i];
    const float4_t gv = reinterpret_cast<const float4_t*>(a.g)[i];
    float4_t mv = a.kind == 0 || a.kind == 3 ? reinterpret_cast<float4_t*>(a.m)[i] : float4_t{0.f, 0.f, 0.f, 0.f};
    float4_t vv = a.kind == 0 || a.kind == 1 ? reinterpret_cast<float4_t*>(a.v)[i] : float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int c = 0; c < 4; ++c) {
      float pc = pv[c], mc = mv[c], vc = vv[c];
      optim_one(pc, gv[c], mc, vc, t, a.lr, a.b1, a.b2, a.eps, flat_wd(a, a.base + 4 * i + c), a.grad_scale, a.kind);
      pv[c] = pc;
      mv[c] = mc;
      vv[c] = vc;
    }
    reinterpret_cast<float4_t*>(a.p)[i] = pv;
    if (a.kind == 0 || a.kind == 3) reinterpret_cast<float4_t*>(a.m)[i] = mv;
    if (a.kind == 0 || a.kind == 1) reinterpret_cast<float4_t*>(a.v)[i] = vv;
  } else {
    for (int64_t e = 4 * i; e < a.n; ++e) {
      float pc = a.p[e], mc = a.m[e], vc = a.v[e];
      optim_one(pc, a.g[e], mc, vc, t, a.lr, a.b1, a.b2, a.eps, flat_wd(a, a.base + e), a.grad_scale, a.kind);
      a.p[e] = pc;
      if (a.kind == 0 || a.kind == 3) a.m[e] = mc;
      if (a.kind == 0 || a.kind == 1) a.v[e] = vc;
    }
  }
  flat_step_ticket(a);
}

__global__ void step_inc_kernel(int64_t* step) { step[0] += 1; }

__device__ __forceinline__ float4_t load_grad4(const float* g) { return *reinterpret_cast<const float4_t*>(g); }
__device__ __forceinline__ float4_t load_grad4(const bf16_t* g) {
  const uint32_t* u = reinterpret_cast<const uint32_t*>(g);
  const uint32_t a = u[0], b = u[1];
  return float4_t{bf2f(static_cast<bf16_t>(a & 0xffffu)), bf2f(static_cast<bf16_t>(a >> 16)),
                  bf2f(static_cast<bf16_t>(b & 0xffffu)), bf2f(static_cast<bf16_t>(b >> 16))};
}

// float4 form of sparse_optim_kernel for D % 4 == 0: 16-byte loads/stores of the table,
// slots and grads (a quarter of the threads, 4x the bytes in flight per thread); GT =
// bf16 takes the gradients straight from a bf16 exchange buffer
template <typename GT>
__global__ __launch_bounds__(256) void sparse_optim4_kernel(float* __restrict__ table, float* __restrict__ m,
                                                            float* __restrict__ v, const int64_t* __restrict__ rows,
                                                            const GT* __restrict__ grads, int64_t n, int D,
                                                            int64_t n_rows, const int64_t* __restrict__ step, float lr,
                                                            float b1, float b2, float eps, int kind) {
  const int D4 = D >> 2;
  grid_stride(n * D4, [&](int64_t t) {
    const int64_t e = t / D4;
    const int d = static_cast<int>(t - e * D4) * 4;
    const int64_t r = rows[e];
    if (r < 0 || r >= n_rows) return;
    const int64_t o = r * D + d;
    const float4_t gi = load_grad4(grads + e * D + d);
    float4_t p = *reinterpret_cast<float4_t*>(table + o);
    if (kind == 0) {
      const float st = static_cast<float>(step[0]);
      const float bc1 = 1.f - __powf(b1, st), bc2 = 1.f - __powf(b2, st);
      float4_t mi = *reinterpret_cast<float4_t*>(m + o), vi = *reinterpret_cast<float4_t*>(v + o);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        mi[k] = b1 * mi[k] + (1.f - b1) * gi[k];
        vi[k] = b2 * vi[k] + (1.f - b2) * gi[k] * gi[k];
        p[k] -= lr * (mi[k] / bc1) / (sqrtf(vi[k] / bc2) + eps);
      }
      *reinterpret_cast<float4_t*>(m + o) = mi;
      *reinterpret_cast<float4_t*>(v + o) = vi;
    } else if (kind == 1) {
      float4_t acc = *reinterpret_cast<float4_t*>(v + o);
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        acc[k] += gi[k] * gi[k];
        p[k] -= lr * gi[k] / (sqrtf(acc[k]) + eps);
      }
      *reinterpret_cast<float4_t*>(v + o) = acc;
    } else {
#pragma unroll
      for (int k = 0; k < 4; ++k) p[k] -= lr * gi[k];
    }
    *reinterpret_cast<float4_t*>(table + o) = p;
  });
}

// rows: unique row ids (int64) into the table, grads [n, D] fp32
__global__ __launch_bounds__(256) void sparse_optim_kernel(float* __restrict__ table, float* __restrict__ m,
                                                           float* __restrict__ v, const int64_t* __restrict__ rows,
                                                           const float* __restrict__ grads, int64_t n, int D,
                                                           int64_t n_rows, const int64_t* __restrict__ step, float lr,
                                                           float b1, float b2, float eps, int kind) {

  grid_stride(n * D, [&](int64_t t) {
    const int64_t e = t / D;
    const int d = static_cast<int>(t - e * D);
    const int64_t r = rows[e];
    if (r < 0 || r >= n_rows) return;
    const int64_t o = r * D + d;
    const float gi = grads[t];
    if (kind == 0) {
      const float st = static_cast<float>(step[0]);
      const float mi = b1 * m[o] + (1.f - b1) * gi;
      const float vi = b2 * v[o] + (1.f - b2) * gi * gi;
      m[o] = mi;
      v[o] = vi;
      const float bc1 = 1.f - __powf(b1, st), bc2 = 1.f - __powf(b2, st);
      table[o] -= lr * (mi / bc1) / (sqrtf(vi / bc2) + eps);
    } else if (kind == 1) {
      const float acc = v[o] + gi * gi;
      v[o] = acc;
      table[o] -= lr * gi / (sqrtf(acc) + eps);
    } else {
      table[o] -= lr * gi;
    }
  });
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

hipError_t eh_flat_optim(float* p, const float* g, float* m, float* v, int64_t n, int64_t* step, float lr, float b1,
                         float b2, float eps, float wd, float grad_scale, int kind, hipStream_t s) {
  return eh_flat_optim2(p, g, m, v, n, step, nullptr, lr, b1, b2, eps, wd, 0.f, 0, 0, grad_scale, kind, s);
}

hipError_t eh_flat_optim2(float* p, const float* g, float* m, float* v, int64_t n, int64_t* step, int32_t* ticket,
                          float lr, float b1, float b2, float eps, float wd, float wd2, int64_t w0, int64_t w1,
                          float grad_scale, int kind, hipStream_t s) {
  // the ticket is one contended atomic per block: ~1.4 ns each on one L2 channel, 70 us
  // on a 38M-parameter buffer (49K blocks) against the ~4 us step_inc launch it saves
  if (ceil_div(n, 1024) > 2048) ticket = nullptr;
  if (!ticket) hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, s, step);
  if (n == 0) {
    if (ticket) hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, s, step);
    return hipGetLastError();
  }
  FlatOptArgs a{p, m, v, g, 0, 0, step, ticket, ticket ? 1 : 0, 1, lr, b1, b2, eps, wd, wd2, grad_scale, w0, w1, kind};
  // 16-byte aligned buffers (torch allocations; offset 0): one float4 launch (ragged tail
  // included); otherwise the scalar kernel
  const bool al = (reinterpret_cast<uintptr_t>(p) | reinterpret_cast<uintptr_t>(g) | reinterpret_cast<uintptr_t>(m) |
                   reinterpret_cast<uintptr_t>(v)) % 16 == 0;
  FlatOptArgs b = a;
  b.n = n;
  if (al)
    hipLaunchKernelGGL(flat_optim4_kernel, dim3(static_cast<uint32_t>(ceil_div(ceil_div(n, 4), 256))), dim3(256), 0, s, b);
  else
    hipLaunchKernelGGL(flat_optim_kernel, dim3(static_cast<uint32_t>(ceil_div(n, 256))), dim3(256), 0, s, b);
  return hipGetLastError();
}

hipError_t eh_sparse_optim(float* table, float* m, float* v, const int64_t* rows, const void* grads, int grads_bf16,
                           int64_t n, int D, int64_t n_rows, int64_t* step, float lr, float b1, float b2, float eps,
                           int kind, hipStream_t s) {
  hipLaunchKernelGGL(step_inc_kernel, dim3(1), dim3(1), 0, s, step);
  if (n == 0 || D == 0) return hipGetLastError();
  if (grads_bf16 && D % 4 != 0) return hipErrorInvalidValue;
  if (D % 4 == 0) {
    const dim3 grid = grid_for(n * (D / 4));
    if (grads_bf16)
      hipLaunchKernelGGL(sparse_optim4_kernel<bf16_t>, grid, dim3(256), 0, s, table, m, v, rows,
                         static_cast<const bf16_t*>(grads), n, D, n_rows, step, lr, b1, b2, eps, kind);
    else
      hipLaunchKernelGGL(sparse_optim4_kernel<float>, grid, dim3(256), 0, s, table, m, v, rows,
                         static_cast<const float*>(grads), n, D, n_rows, step, lr, b1, b2, eps, kind);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(sparse_optim_kernel, grid_for(n * D), dim3(256), 0, s, table,
                     m, v, rows, static_cast<const float*>(grads), n, D, n_rows, step, lr, b1, b2, eps, kind);
  return hipGetLastError();
}

}  // extern "C"
