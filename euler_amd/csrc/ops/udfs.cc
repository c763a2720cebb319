// Built-in values() UDFs (reference euler/core/kernels/{mean,min,max}_udf.cc), registered
// through the UDF registry like a user's own (framework/udf.h).
//   udf_mean  dense: mean of a node's values (one value; none for an empty row)
//   udf_min / udf_max  dense and sparse: the extreme value (one value; none when empty)
//   udf_sum   dense: sum of the values (one value, 0 for an empty row)
//   udf_topk  dense and sparse, parameter [k] (default 1): the k largest values in
//             descending order (fewer when the row is shorter)
#include <algorithm>
#include <cmath>
#include <functional>
#include <limits>

#include "framework/udf.h"

namespace euler {
namespace {

class MeanUdf : public PerNodeUdf {
 protected:
  void Dense(const float* v, int64_t n, const std::vector<float>&, std::vector<float>* out) const override {
    if (n == 0) return;
    double s = 0;
    for (int64_t i = 0; i < n; ++i) s += v[i];
    out->push_back(static_cast<float>(s / n));
  }
};

template <bool kMax>
class ExtremeUdf : public PerNodeUdf {
 protected:
  void Dense(const float* v, int64_t n, const std::vector<float>&, std::vector<float>* out) const override {
    if (n == 0) return;
    out->push_back(kMax ? *std::max_element(v, v + n) : *std::min_element(v, v + n));
  }
  void Sparse(const uint64_t* v, int64_t n, const std::vector<float>&, std::vector<uint64_t>* out) const override {
    if (n == 0) return;
    out->push_back(kMax ? *std::max_element(v, v + n) : *std::min_element(v, v + n));
  }
};

class SumUdf : public PerNodeUdf {
 protected:
  void Dense(const float* v, int64_t n, const std::vector<float>&, std::vector<float>* out) const override {
    double s = 0;
    for (int64_t i = 0; i < n; ++i) s += v[i];
    out->push_back(static_cast<float>(s));
  }
};

class TopKUdf : public PerNodeUdf {
  static int64_t K(const std::vector<float>& params) {
    const float k = params.empty() ? 1.f : params[0];
    return k >= 1.f ? static_cast<int64_t>(std::floor(k)) : 1;
  }

  template <typename T>
  static void Top(const T* v, int64_t n, int64_t k, std::vector<T>* out) {
    std::vector<T> tmp(v, v + n);
    const int64_t m = std::min(k, n);
    std::partial_sort(tmp.begin(), tmp.begin() + m, tmp.end(), std::greater<T>());
    out->insert(out->end(), tmp.begin(), tmp.begin() + m);
  }

 protected:
  void Dense(const float* v, int64_t n, const std::vector<float>& p, std::vector<float>* out) const override {
    Top(v, n, K(p), out);
  }
  void Sparse(const uint64_t* v, int64_t n, const std::vector<float>& p, std::vector<uint64_t>* out) const override {
    Top(v, n, K(p), out);
  }
};

REGISTER_UDF("udf_mean", MeanUdf);
REGISTER_UDF("udf_min", ExtremeUdf<false>);
REGISTER_UDF("udf_max", ExtremeUdf<true>);
REGISTER_UDF("udf_sum", SumUdf);
REGISTER_UDF("udf_topk", TopKUdf);

}  // namespace
}  // namespace euler
