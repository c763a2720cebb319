// euler_amd engine — user-defined functions over values() columns (SURVEY §2.1 N13;
// reference euler/core/framework/udf.h:95-144, udf.cc:61-128, kernels/{mean,min,max}_udf.cc).
//
// GQL  `v(ids).values(f1, f2).udf_topk(f2)[3].as(x)`  applies the UDF registered as
// "udf_topk" to feature f2 of every node (f1 is returned as is), with the numeric
// parameter list [3].  The UDF runs where the feature lives: on the shard server in
// distribute mode (the name and parameters travel inside the REMOTE sub-DAG), in-process
// in local mode.  mean / min / max / topk are registered with REGISTER_UDF like any other
// UDF (csrc/ops/udfs.cc): a new UDF is a ValuesUdf (or PerNodeUdf) subclass plus one
// REGISTER_UDF line in a source compiled into the engine, as in the reference.
#pragma once

#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace euler {

// one feature of a batch of nodes / edges in the engine's ragged layout
struct UdfColumn {
  enum Kind { kDense = 0, kSparse = 1 };
  int kind = kDense;
  std::vector<int64_t> counts;  // values per node (or edge)
  std::vector<float> f;         // kDense: flat values
  std::vector<uint64_t> u;      // kSparse: flat values
};

// Instances are shared by every query and executor thread: Compute must be thread-safe.
class ValuesUdf {
 public:
  virtual ~ValuesUdf() = default;
  // in -> out for every node; params = the query's numeric [..] list
  virtual void Compute(const UdfColumn& in, const std::vector<float>& params, UdfColumn* out) const = 0;
};

// per-node map: override Dense and/or Sparse (the default rejects the feature kind)
class PerNodeUdf : public ValuesUdf {
 public:
  void Compute(const UdfColumn& in, const std::vector<float>& params, UdfColumn* out) const override;

 protected:
  // append the outputs of one node's values v[0..n) to *out
  virtual void Dense(const float* v, int64_t n, const std::vector<float>& params, std::vector<float>* out) const;
  virtual void Sparse(const uint64_t* v, int64_t n, const std::vector<float>& params,
                      std::vector<uint64_t>* out) const;
};

typedef ValuesUdf* (*UdfFactory)();

// process-wide registry: a name registers once (a second registration throws)
void RegisterUdf(const char* name, UdfFactory factory);
std::shared_ptr<const ValuesUdf> FindUdf(const std::string& name);  // nullptr: unknown
std::vector<std::string> RegisteredUdfs();

struct UdfRegistrar {
  UdfRegistrar(const char* name, UdfFactory f) { RegisterUdf(name, f); }
};

#define EULER_UDF_CAT2(a, b) a##b
#define EULER_UDF_CAT(a, b) EULER_UDF_CAT2(a, b)
#define REGISTER_UDF(name, cls)                                                  \
  static ::euler::UdfRegistrar EULER_UDF_CAT(euler_udf_registrar_, __COUNTER__)( \
      name, []() -> ::euler::ValuesUdf* { return new cls(); })

}  // namespace euler
