// One element of the flat optimizers (Adam / Adagrad / SGD / momentum), shared by the flat
// optimizer launch (optim.hip) and the launches that fold the update into their own tail
// (gcn.hip gcn_reduce_kernel).  t: the 1-based step of the update.
#pragma once
#include <hip/hip_runtime.h>

namespace euler_hip {

__device__ __forceinline__ float optim_one(float& p, float g, float& m, float& v, float t, float lr, float b1,
                                           float b2, float eps, float wd, float grad_scale, int kind) {
  const float gi = g * grad_scale + wd * p;
  if (kind == 0) {
    m = b1 * m + (1.f - b1) * gi;
    v = b2 * v + (1.f - b2) * gi * gi;
    const float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
    p -= lr * (m / bc1) / (sqrtf(v / bc2) + eps);
  } else if (kind == 1) {
    v += gi * gi;
    p -= lr * gi / (sqrtf(v) + eps);
  } else if (kind == 2) {
    p -= lr * gi;
  } else {
    m = b1 * m + gi;
    p -= lr * m;
  }
  return p;
}

}  // namespace euler_hip
