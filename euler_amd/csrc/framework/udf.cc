// UDF registry (reference euler/core/framework/udf.cc:95-128: name -> factory map and a
// per-name instance cache).  Here the instance is created at lookup time once and shared.
#include "framework/udf.h"

#include <map>
#include <mutex>

#include "common/common.h"

namespace euler {

namespace {

struct Registry {
  std::mutex mu;
  std::map<std::string, UdfFactory> factories;
  std::map<std::string, std::shared_ptr<const ValuesUdf>> instances;
};

Registry& Reg() {
  static Registry* r = new Registry;  // never destroyed: registrars run during static init
  return *r;
}

}  // namespace

void RegisterUdf(const char* name, UdfFactory factory) {
  Registry& r = Reg();
  std::lock_guard<std::mutex> l(r.mu);
  if (!factory || !r.factories.emplace(name, factory).second) EULER_THROW("UDF '" << name << "' registered twice");
}

std::shared_ptr<const ValuesUdf> FindUdf(const std::string& name) {
  Registry& r = Reg();
  std::lock_guard<std::mutex> l(r.mu);
  auto it = r.instances.find(name);
  if (it != r.instances.end()) return it->second;
  auto f = r.factories.find(name);
  if (f == r.factories.end()) return nullptr;
  std::shared_ptr<const ValuesUdf> inst(f->second());
  r.instances[name] = inst;
  return inst;
}

std::vector<std::string> RegisteredUdfs() {
  Registry& r = Reg();
  std::lock_guard<std::mutex> l(r.mu);
  std::vector<std::string> out;
  for (auto& kv : r.factories) out.push_back(kv.first);
  return out;
}

void PerNodeUdf::Compute(const UdfColumn& in, const std::vector<float>& params, UdfColumn* out) const {
  out->kind = in.kind;
  out->counts.assign(in.counts.size(), 0);
  int64_t off = 0;
  for (size_t i = 0; i < in.counts.size(); ++i) {
    const int64_t k = in.counts[i];
    if (in.kind == UdfColumn::kDense) {
      const size_t before = out->f.size();
      Dense(in.f.data() + off, k, params, &out->f);
      out->counts[i] = static_cast<int64_t>(out->f.size() - before);
    } else {
      const size_t before = out->u.size();
      Sparse(in.u.data() + off, k, params, &out->u);
      out->counts[i] = static_cast<int64_t>(out->u.size() - before);
    }
    off += k;
  }
}

void PerNodeUdf::Dense(const float*, int64_t, const std::vector<float>&, std::vector<float>*) const {
  EULER_THROW("this UDF does not take dense features");
}

void PerNodeUdf::Sparse(const uint64_t*, int64_t, const std::vector<float>&, std::vector<uint64_t>*) const {
  EULER_THROW("this UDF does not take sparse features");
}

}  // namespace euler
