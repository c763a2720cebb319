#include "framework/framework.h"

#include <algorithm>
#include <cstdlib>
#include <cstring>

namespace euler {

// ============================================================================ buffer cache
namespace {
constexpr size_t kBlockMin = size_t(1) << 20;
struct BlockCache {
  std::mutex mu;
  std::vector<std::vector<void*>> free;  // by log2 size class
  size_t cached = 0, cap = 0;
  BlockCache() : free(64) {
    const char* e = getenv("EULER_TENSOR_CACHE_MB");
    cap = static_cast<size_t>(e ? std::max(0L, atol(e)) : 512) << 20;
  }
  ~BlockCache() = delete;  // process lifetime (buffers may be freed during static teardown)
};
BlockCache& Cache() {
  static BlockCache* c = new BlockCache();
  return *c;
}
int SizeClass(size_t n) {
  int k = 20;
  while ((size_t(1) << k) < n) ++k;
  return k;
}
}  // namespace

void* TensorBlockAlloc(size_t n) {
  if (n < kBlockMin) {
    void* p = std::malloc(n ? n : 1);
    if (!p) throw std::bad_alloc();
    return p;
  }
  const int k = SizeClass(n);
  BlockCache& c = Cache();
  {
    std::lock_guard<std::mutex> l(c.mu);
    if (!c.free[k].empty()) {
      void* p = c.free[k].back();
      c.free[k].pop_back();
      c.cached -= size_t(1) << k;
      return p;
    }
  }
  void* p = std::malloc(size_t(1) << k);
  if (!p) throw std::bad_alloc();
  return p;
}

void TensorBlockFree(void* p, size_t n) {
  if (!p) return;
  if (n < kBlockMin) {
    std::free(p);
    return;
  }
  const int k = SizeClass(n);
  BlockCache& c = Cache();
  {
    std::lock_guard<std::mutex> l(c.mu);
    if (c.cached + (size_t(1) << k) <= c.cap) {
      c.free[k].push_back(p);
      c.cached += size_t(1) << k;
      return;
    }
  }
  std::free(p);
}

size_t TensorBlockCached() {
  std::lock_guard<std::mutex> l(Cache().mu);
  return Cache().cached;
}

// ============================================================================ Tensor
size_t DTypeSize(DType t) {
  switch (t) {
    case DType::kInt8: case DType::kUInt8: case DType::kBool: return 1;
    case DType::kInt16: case DType::kUInt16: return 2;
    case DType::kInt32: case DType::kUInt32: case DType::kFloat: return 4;
    case DType::kInt64: case DType::kUInt64: case DType::kDouble: return 8;
    case DType::kString: return 0;
  }
  return 0;
}

const char* DTypeName(DType t) {
  static const char* n[] = {"int8", "int16", "int32", "int64", "uint8", "uint16",
                            "uint32", "uint64", "float", "double", "bool", "string"};
  return n[static_cast<int>(t)];
}

Tensor::Tensor(DType t, std::vector<int64_t> shape) : dtype_(t), shape_(std::move(shape)) {
  const int64_t n = numel();
  if (t == DType::kString) strs_ = std::make_shared<std::vector<std::string>>(n);
  else {
    bytes_ = std::make_shared<ByteBuf>(static_cast<size_t>(n) * DTypeSize(t));
    if (!bytes_->empty()) memset(bytes_->data(), 0, bytes_->size());
  }
}

Tensor Tensor::Uninit(DType t, std::vector<int64_t> shape) {
  if (t == DType::kString) return Tensor(t, std::move(shape));
  Tensor r;
  r.dtype_ = t;
  r.shape_ = std::move(shape);
  r.bytes_ = std::make_shared<ByteBuf>(static_cast<size_t>(r.numel()) * DTypeSize(t));
  return r;
}

Tensor Tensor::Strings(const std::vector<std::string>& v, std::vector<int64_t> shape) {
  Tensor t(DType::kString, shape.empty() ? std::vector<int64_t>{static_cast<int64_t>(v.size())} : shape);
  *t.strs_ = v;
  return t;
}

int64_t Tensor::numel() const {
  int64_t n = 1;
  for (int64_t d : shape_) n *= d;
  return n;
}

int64_t Tensor::AsInt(int64_t i) const {
  switch (dtype_) {
    case DType::kInt8: return data<int8_t>()[i];
    case DType::kInt16: return data<int16_t>()[i];
    case DType::kInt32: return data<int32_t>()[i];
    case DType::kInt64: return data<int64_t>()[i];
    case DType::kUInt8: case DType::kBool: return data<uint8_t>()[i];
    case DType::kUInt16: return data<uint16_t>()[i];
    case DType::kUInt32: return data<uint32_t>()[i];
    case DType::kUInt64: return static_cast<int64_t>(data<uint64_t>()[i]);
    case DType::kFloat: return static_cast<int64_t>(data<float>()[i]);
    case DType::kDouble: return static_cast<int64_t>(data<double>()[i]);
    case DType::kString: {
      int64_t v = 0;
      ParseInt64((*strs_)[i], &v);
      return v;
    }
  }
  return 0;
}

double Tensor::AsDouble(int64_t i) const {
  switch (dtype_) {
    case DType::kFloat: return data<float>()[i];
    case DType::kDouble: return data<double>()[i];
    case DType::kUInt64: return static_cast<double>(data<uint64_t>()[i]);
    case DType::kString: {
      double v = 0;
      ParseDouble((*strs_)[i], &v);
      return v;
    }
    default: return static_cast<double>(AsInt(i));
  }
}

std::vector<int64_t> Tensor::ToInt64() const {
  std::vector<int64_t> v(numel());
  for (int64_t i = 0; i < numel(); ++i) v[i] = AsInt(i);
  return v;
}

std::vector<uint64_t> Tensor::ToUInt64() const {
  std::vector<uint64_t> v(numel());
  if (dtype_ == DType::kUInt64 || dtype_ == DType::kInt64) {
    if (numel()) memcpy(v.data(), raw(), numel() * 8);
  } else {
    for (int64_t i = 0; i < numel(); ++i) v[i] = static_cast<uint64_t>(AsInt(i));
  }
  return v;
}

std::vector<int32_t> Tensor::ToInt32() const {
  std::vector<int32_t> v(numel());
  for (int64_t i = 0; i < numel(); ++i) v[i] = static_cast<int32_t>(AsInt(i));
  return v;
}

std::vector<std::string> Tensor::ToStrings() const {
  if (dtype_ == DType::kString) return *strs_;
  std::vector<std::string> v(numel());
  for (int64_t i = 0; i < numel(); ++i) {
    if (dtype_ == DType::kFloat || dtype_ == DType::kDouble) {
      std::ostringstream os;
      os << AsDouble(i);
      v[i] = os.str();
    } else {
      v[i] = std::to_string(AsInt(i));
    }
  }
  return v;
}

void Tensor::Encode(BytesWriter* w) const {
  w->Write<int32_t>(static_cast<int32_t>(dtype_));
  w->Write<uint32_t>(static_cast<uint32_t>(shape_.size()));
  for (int64_t d : shape_) w->Write(d);
  if (dtype_ == DType::kString) {
    for (const auto& s : *strs_) w->Write(s);
  } else {
    w->Write<uint64_t>(nbytes());
    if (nbytes()) w->WriteRaw(raw(), nbytes());
  }
}

size_t Tensor::EncodedSize() const {
  size_t n = 4 + 4 + 8 * shape_.size();
  if (dtype_ == DType::kString) {
    for (const auto& x : *strs_) n += 4 + x.size();
  } else {
    n += 8 + nbytes();
  }
  return n;
}

bool Tensor::Decode(BytesReader* r, Tensor* t) {
  int32_t dt;
  uint32_t rank;
  if (!r->Read(&dt) || !r->Read(&rank) || dt < 0 || dt > 11 || rank > 16) return false;
  std::vector<int64_t> shape(rank);
  for (auto& d : shape)
    if (!r->Read(&d)) return false;
  *t = Tensor::Uninit(static_cast<DType>(dt), shape);
  if (t->dtype() == DType::kString) {
    for (auto& s : t->strings())
      if (!r->Read(&s)) return false;
  } else {
    uint64_t nb;
    if (!r->Read(&nb) || nb != t->nbytes() || r->remaining() < nb) return false;
    if (nb) memcpy(t->raw(), r->cur(), nb);
    r->skip(nb);
  }
  return true;
}

// ============================================================================ DAG
void NodeDef::Encode(BytesWriter* w) const {
  w->Write(op);
  w->Write<int32_t>(id);
  auto ws = [&](const std::vector<std::string>& v) {
    w->Write<uint32_t>(static_cast<uint32_t>(v.size()));
    for (auto& s : v) w->Write(s);
  };
  ws(inputs);
  ws(attrs);
  ws(dnf);
  ws(post_process);
  w->Write(udf_name);
  ws(udf_str_params);
  w->Write(udf_num_params);
  w->Write<int32_t>(output_num);
  w->Write<int32_t>(shard_idx);
  w->Write<uint32_t>(static_cast<uint32_t>(inner.size()));
  for (auto& n : inner) n.Encode(w);
  ws(output_list);
}

bool NodeDef::Decode(BytesReader* r, NodeDef* n) {
  auto rs = [&](std::vector<std::string>* v) {
    uint32_t k;
    if (!r->Read(&k) || k > (1u << 24)) return false;
    v->resize(k);
    for (auto& s : *v)
      if (!r->Read(&s)) return false;
    return true;
  };
  int32_t id, on, si;
  uint32_t ni;
  if (!r->Read(&n->op) || !r->Read(&id) || !rs(&n->inputs) || !rs(&n->attrs) || !rs(&n->dnf) ||
      !rs(&n->post_process) || !r->Read(&n->udf_name) || !rs(&n->udf_str_params) || !r->Read(&n->udf_num_params) ||
      !r->Read(&on) || !r->Read(&si) || !r->Read(&ni) || ni > (1u << 20))
    return false;
  n->id = id;
  n->output_num = on;
  n->shard_idx = si;
  n->inner.resize(ni);
  for (auto& c : n->inner)
    if (!Decode(r, &c)) return false;
  return rs(&n->output_list);
}

std::string NodeDef::DebugString(int indent) const {
  std::ostringstream os;
  std::string pad(indent, ' ');
  os << pad << name() << " in=[" << Join(inputs, " ") << "]";
  if (!attrs.empty()) os << " attrs=[" << Join(attrs, " ") << "]";
  if (!dnf.empty()) os << " dnf=[" << Join(dnf, " | ") << "]";
  if (!post_process.empty()) os << " pp=[" << Join(post_process, "; ") << "]";
  if (!udf_name.empty()) os << " udf=" << udf_name;
  if (shard_idx >= 0) os << " shard=" << shard_idx << " fetch=[" << Join(output_list, " ") << "]";
  os << " outs=" << output_num << "\n";
  for (auto& c : inner) os << c.DebugString(indent + 4);
  return os.str();
}

std::string DAGDef::Serialize() const {
  BytesWriter w;
  w.Write<uint32_t>(static_cast<uint32_t>(nodes.size()));
  for (auto& n : nodes) n.Encode(&w);
  return w.str();
}

bool DAGDef::Parse(const char* p, size_t n, DAGDef* d) {
  BytesReader r(p, n);
  uint32_t k;
  if (!r.Read(&k) || k > (1u << 20)) return false;
  d->nodes.resize(k);
  for (auto& nd : d->nodes)
    if (!NodeDef::Decode(&r, &nd)) return false;
  return true;
}

std::string DAGDef::DebugString() const {
  std::string s;
  for (auto& n : nodes) s += n.DebugString();
  return s;
}

const NodeDef* DAGDef::Find(const std::string& name) const {
  for (auto& n : nodes)
    if (n.name() == name) return &n;
  return nullptr;
}

std::string InputNode(const std::string& input) {
  const size_t c = input.rfind(':');
  return c == std::string::npos ? input : input.substr(0, c);
}

// ============================================================================ OpContext
bool OpContext::Has(const std::string& name) const {
  std::lock_guard<std::mutex> l(mu_);
  return tensors_.count(name) > 0;
}

const Tensor& OpContext::Get(const std::string& name) const {
  std::lock_guard<std::mutex> l(mu_);
  auto it = tensors_.find(name);
  if (it == tensors_.end()) EULER_THROW("tensor '" << name << "' not found in query context");
  return it->second;
}

bool OpContext::TryGet(const std::string& name, Tensor* t) const {
  std::lock_guard<std::mutex> l(mu_);
  auto it = tensors_.find(name);
  if (it == tensors_.end()) return false;
  *t = it->second;
  return true;
}

void OpContext::Set(const std::string& name, Tensor t) {
  std::lock_guard<std::mutex> l(mu_);
  tensors_[name] = std::move(t);
}

std::map<std::string, Tensor> OpContext::Snapshot() const {
  std::lock_guard<std::mutex> l(mu_);
  return std::map<std::string, Tensor>(tensors_.begin(), tensors_.end());
}

// An attribute is a literal ("0,1", "5", "-1") or the name of an input tensor.
std::vector<int32_t> OpContext::AttrInts(const std::string& a) const {
  Tensor t;
  if (TryGet(a, &t)) return t.ToInt32();
  std::vector<int32_t> v;
  for (auto& s : Split(a, ",")) {
    int64_t x;
    if (ParseInt64(Trim(s), &x)) v.push_back(static_cast<int32_t>(x));
    else EULER_THROW("attribute '" << a << "' is neither a tensor nor an integer list");
  }
  return v;
}

int64_t OpContext::AttrInt(const std::string& a) const {
  Tensor t;
  if (TryGet(a, &t)) {
    if (t.numel() < 1) EULER_THROW("empty tensor attribute " << a);
    return t.AsInt(0);
  }
  int64_t x;
  if (!ParseInt64(Trim(a), &x)) EULER_THROW("attribute '" << a << "' is not an integer");
  return x;
}

std::string OpContext::AttrStr(const std::string& a) const {
  Tensor t;
  if (TryGet(a, &t) && t.numel() > 0) return t.ToStrings()[0];
  return a;
}

std::vector<std::string> OpContext::AttrStrs(const std::string& a) const {
  Tensor t;
  if (TryGet(a, &t)) return t.ToStrings();
  return Split(a, ",");
}

// ============================================================================ registry
KernelRegistry& KernelRegistry::Get() {
  static KernelRegistry r;
  return r;
}

void KernelRegistry::Register(const std::string& op, std::function<OpKernel*()> f) {
  std::lock_guard<std::mutex> l(mu_);
  factories_[op] = std::move(f);
}

OpKernel* KernelRegistry::Lookup(const std::string& op) {
  std::lock_guard<std::mutex> l(mu_);
  auto c = cache_.find(op);
  if (c != cache_.end()) return c->second.get();
  auto f = factories_.find(op);
  if (f == factories_.end()) return nullptr;
  OpKernel* k = f->second();
  cache_[op].reset(k);
  return k;
}

std::vector<std::string> KernelRegistry::Ops() const {
  std::lock_guard<std::mutex> l(mu_);
  std::vector<std::string> v;
  for (auto& kv : factories_) v.push_back(kv.first);
  return v;
}

// ============================================================================ Executor
Executor::Executor(const DAGDef& dag, OpContext* ctx, ThreadPool* pool)
    : dag_(dag), ctx_(ctx), pool_(pool), succ_(dag.nodes.size()), pending_(dag.nodes.size()) {
  std::unordered_map<std::string, size_t> by_name;
  for (size_t i = 0; i < dag.nodes.size(); ++i) by_name[dag.nodes[i].name()] = i;
  for (size_t i = 0; i < dag.nodes.size(); ++i) {
    std::vector<size_t> deps;
    for (const auto& in : dag.nodes[i].inputs) {
      auto it = by_name.find(InputNode(in));
      if (it != by_name.end() && it->second != i) deps.push_back(it->second);
    }
    // attributes may also reference node outputs
    for (const auto& a : dag.nodes[i].attrs) {
      auto it = by_name.find(InputNode(a));
      if (it != by_name.end() && it->second != i) deps.push_back(it->second);
    }
    std::sort(deps.begin(), deps.end());
    deps.erase(std::unique(deps.begin(), deps.end()), deps.end());
    pending_[i].store(static_cast<int>(deps.size()));
    for (size_t d : deps) succ_[d].push_back(i);
  }
}

void Executor::Schedule(size_t i) {
  const NodeDef& nd = dag_.nodes[i];
  OpKernel* k = KernelRegistry::Get().Lookup(nd.op);
  if (!k) {
    NodeDone(i, Status::NotFound("no kernel registered for op " + nd.op));
    return;
  }
  EngineCounters::Get().dag_nodes.fetch_add(1, std::memory_order_relaxed);
  auto run = [this, i, k, &nd] {
    const bool prof = OpProfileEnabled();
    const uint64_t t0 = prof ? NowMicros() : 0;
    if (k->is_async()) {
      k->ComputeAsync(nd, ctx_, [this, i, prof, t0, &nd](Status st) {
        if (prof) OpProfileAdd(nd.op, static_cast<int64_t>(NowMicros() - t0));
        NodeDone(i, st);
      });
      return;
    }
    Status st;
    try {
      k->Compute(nd, ctx_);
    } catch (const std::exception& e) {
      st = Status::Internal(nd.name() + ": " + e.what());
    }
    if (prof) OpProfileAdd(nd.op, static_cast<int64_t>(NowMicros() - t0));
    NodeDone(i, st);
  };
  run();
}

void Executor::NodeDone(size_t i, Status st) {
  if (!st.ok()) {
    std::lock_guard<std::mutex> l(mu_);
    if (status_.ok()) status_ = st;
  }
  std::vector<size_t> ready;
  for (size_t s : succ_[i])
    if (pending_[s].fetch_sub(1) == 1) ready.push_back(s);
  // run one successor inline, hand the rest to the pool
  for (size_t r = 1; r < ready.size(); ++r) {
    const size_t s = ready[r];
    pool_->Schedule([this, s] { Schedule(s); });
  }
  const bool last = remaining_.fetch_sub(1) == 1;
  if (!ready.empty()) Schedule(ready[0]);
  if (last) {
    std::function<void(Status)> done;
    Status final_st;
    {
      std::lock_guard<std::mutex> l(mu_);
      done.swap(done_);
      final_st = status_;
    }
    if (done) done(final_st);
  }
}

void Executor::RunAsync(std::function<void(Status)> done) {
  const size_t n = dag_.nodes.size();
  if (n == 0) {
    done(Status::OK());
    return;
  }
  done_ = std::move(done);
  remaining_.store(static_cast<int64_t>(n));
  std::vector<size_t> roots;
  for (size_t i = 0; i < n; ++i)
    if (pending_[i].load() == 0) roots.push_back(i);
  for (size_t r = 1; r < roots.size(); ++r) {
    const size_t s = roots[r];
    pool_->Schedule([this, s] { Schedule(s); });
  }
  if (!roots.empty()) Schedule(roots[0]);
}

Status Executor::Run() {
  Latch latch(1);
  Status result;
  RunAsync([&](Status st) {
    result = st;
    latch.CountDown();
  });
  latch.Wait();
  return result;
}

}  // namespace euler
