// euler_amd engine — tensors, DAG IR, op-kernel registry and the dependency-counting
// executor.
//
// Conventions kept from the reference so compiled DAGs read the same
// (dag_node_def.cc:20-91): a node is named "<OP>,<id>", its outputs are
// "<OP>,<id>:<slot>", an external input is a bare tensor name; REMOTE nodes carry
// a shard index, an inner sub-DAG and the inner output names to fetch.  Results
// of every graph op use the ragged "idx [N,2] (begin,end) + flat data" layout
// (SURVEY §2.4).
//
// The wire format is our own (length-prefixed binary, no protobuf): tensors as
// dtype + shape + raw bytes, DAGs as a flat list of NodeDefs.
#pragma once

#include <stdint.h>

#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "common/common.h"
#include "common/runtime.h"

namespace euler {

// ============================================================================ Tensor
enum class DType : int32_t {
  kInt8 = 0, kInt16, kInt32, kInt64, kUInt8, kUInt16, kUInt32, kUInt64, kFloat, kDouble, kBool, kString
};
size_t DTypeSize(DType t);
const char* DTypeName(DType t);

template <typename T>
struct DTypeOf;
template <> struct DTypeOf<int8_t> { static constexpr DType v = DType::kInt8; };
template <> struct DTypeOf<int16_t> { static constexpr DType v = DType::kInt16; };
template <> struct DTypeOf<int32_t> { static constexpr DType v = DType::kInt32; };
template <> struct DTypeOf<int64_t> { static constexpr DType v = DType::kInt64; };
template <> struct DTypeOf<uint8_t> { static constexpr DType v = DType::kUInt8; };
template <> struct DTypeOf<uint16_t> { static constexpr DType v = DType::kUInt16; };
template <> struct DTypeOf<uint32_t> { static constexpr DType v = DType::kUInt32; };
template <> struct DTypeOf<uint64_t> { static constexpr DType v = DType::kUInt64; };
template <> struct DTypeOf<float> { static constexpr DType v = DType::kFloat; };
template <> struct DTypeOf<double> { static constexpr DType v = DType::kDouble; };

// Large tensor buffers (>= 1 MiB) are recycled through a process-wide cache of
// power-of-two blocks instead of going back to the OS: a fresh multi-MB malloc is an
// mmap whose first touch page-faults every 4 KiB, which dominated the remote feature
// path (13 MB replies).  Capped by EULER_TENSOR_CACHE_MB (default 512; 0 disables).
void* TensorBlockAlloc(size_t n);
void TensorBlockFree(void* p, size_t n);
size_t TensorBlockCached();

// byte storage whose resize leaves the bytes uninitialised: Tensor's constructor zeroes
// them explicitly, Tensor::Uninit skips that for buffers the caller overwrites whole
template <typename T>
struct NoInitAlloc : std::allocator<T> {
  using value_type = T;
  T* allocate(size_t n) { return static_cast<T*>(TensorBlockAlloc(n * sizeof(T))); }
  void deallocate(T* p, size_t n) { TensorBlockFree(p, n * sizeof(T)); }
  template <typename U>
  struct rebind {
    using other = NoInitAlloc<U>;
  };
  NoInitAlloc() = default;
  template <typename U>
  NoInitAlloc(const NoInitAlloc<U>&) {}
  template <typename U>
  void construct(U* p) {
    ::new (static_cast<void*>(p)) U;
  }
  template <typename U, typename... A>
  void construct(U* p, A&&... a) {
    ::new (static_cast<void*>(p)) U(std::forward<A>(a)...);
  }
};
using ByteBuf = std::vector<char, NoInitAlloc<char>>;

class Tensor {
 public:
  Tensor() = default;
  Tensor(DType t, std::vector<int64_t> shape);  // zero-filled
  static Tensor Uninit(DType t, std::vector<int64_t> shape);  // numeric only, bytes undefined
  template <typename T>
  static Tensor FromVector(const std::vector<T>& v, std::vector<int64_t> shape = {}) {
    Tensor t = Uninit(DTypeOf<T>::v, shape.empty() ? std::vector<int64_t>{static_cast<int64_t>(v.size())} : shape);
    if (t.nbytes() > v.size() * sizeof(T)) memset(t.raw(), 0, t.nbytes());
    if (!v.empty()) memcpy(t.raw(), v.data(), v.size() * sizeof(T));
    return t;
  }
  static Tensor Strings(const std::vector<std::string>& v, std::vector<int64_t> shape = {});
  template <typename T>
  static Tensor Scalar(T x) {
    Tensor t(DTypeOf<T>::v, {1});
    *t.data<T>() = x;
    return t;
  }

  DType dtype() const { return dtype_; }
  const std::vector<int64_t>& shape() const { return shape_; }
  int64_t numel() const;
  int64_t dim(int i) const { return shape_[i]; }
  bool defined() const { return bytes_ != nullptr || strs_ != nullptr; }
  template <typename T>
  T* data() {
    return reinterpret_cast<T*>(bytes_->data());
  }
  template <typename T>
  const T* data() const {
    return reinterpret_cast<const T*>(bytes_->data());
  }
  void* raw() { return bytes_ ? bytes_->data() : nullptr; }
  const void* raw() const { return bytes_ ? bytes_->data() : nullptr; }
  size_t nbytes() const { return bytes_ ? bytes_->size() : 0; }
  std::vector<std::string>& strings() { return *strs_; }
  const std::vector<std::string>& strings() const { return *strs_; }
  // element i as int64 / double regardless of numeric dtype
  int64_t AsInt(int64_t i) const;
  double AsDouble(int64_t i) const;
  std::vector<int64_t> ToInt64() const;
  std::vector<uint64_t> ToUInt64() const;
  std::vector<int32_t> ToInt32() const;
  std::vector<std::string> ToStrings() const;  // numeric -> decimal text
  void Reshape(std::vector<int64_t> s) { shape_ = std::move(s); }

  void Encode(BytesWriter* w) const;
  size_t EncodedSize() const;  // bytes Encode writes
  static bool Decode(BytesReader* r, Tensor* t);

 private:
  DType dtype_ = DType::kInt64;
  std::vector<int64_t> shape_;
  std::shared_ptr<ByteBuf> bytes_;
  std::shared_ptr<std::vector<std::string>> strs_;
};

// ============================================================================ DAG IR
struct NodeDef {
  std::string op;
  int id = 0;
  std::vector<std::string> inputs;        // "<node>:<slot>" or external tensor names
  std::vector<std::string> attrs;         // literal / tensor-name attributes (edge types, counts, ...)
  std::vector<std::string> dnf;           // one conjunction per entry: "f op v,f op v"
  std::vector<std::string> post_process;  // "order_by id asc", "limit 3"
  std::string udf_name;
  std::vector<std::string> udf_str_params;
  std::vector<float> udf_num_params;
  int output_num = 1;
  // REMOTE
  int shard_idx = -1;
  std::vector<NodeDef> inner;
  std::vector<std::string> output_list;  // inner outputs to fetch, in order

  std::string name() const { return op + "," + std::to_string(id); }
  std::string Output(int slot) const { return name() + ":" + std::to_string(slot); }
  void Encode(BytesWriter* w) const;
  size_t EncodedSize() const;  // bytes Encode writes
  static bool Decode(BytesReader* r, NodeDef* n);
  std::string DebugString(int indent = 0) const;
};

struct DAGDef {
  std::vector<NodeDef> nodes;
  std::string Serialize() const;
  static bool Parse(const char* p, size_t n, DAGDef* d);
  std::string DebugString() const;
  const NodeDef* Find(const std::string& name) const;
};

// ============================================================================ kernels
class Graph;
class IndexManager;
class RemoteClients;

// Per-process engine environment shared by kernels (graph shard, indexes, remote
// clients and the cluster-wide weight tables used by the sampling split ops).
struct EngineEnv {
  Graph* graph = nullptr;
  IndexManager* index = nullptr;
  RemoteClients* clients = nullptr;
  int shard_num = 1;
  uint32_t num_partitions = 1;
  // [type + 1][shard + 1] weight sums (last row / column = totals), reference query_proxy.cc:91-144
  std::vector<std::vector<double>> node_weight_sums, edge_weight_sums;
  std::vector<std::string> graph_labels;
  std::string index_info;
};

class OpContext {
 public:
  explicit OpContext(EngineEnv* env) : env_(env) {}
  EngineEnv* env() const { return env_; }
  bool Has(const std::string& name) const;
  const Tensor& Get(const std::string& name) const;  // throws when missing
  bool TryGet(const std::string& name, Tensor* t) const;
  void Set(const std::string& name, Tensor t);
  std::map<std::string, Tensor> Snapshot() const;
  // literal-or-tensor attribute helpers
  std::vector<int32_t> AttrInts(const std::string& a) const;
  int64_t AttrInt(const std::string& a) const;
  std::string AttrStr(const std::string& a) const;
  std::vector<std::string> AttrStrs(const std::string& a) const;

 private:
  EngineEnv* env_;
  mutable std::mutex mu_;
  std::unordered_map<std::string, Tensor> tensors_;
};

class OpKernel {
 public:
  virtual ~OpKernel() = default;
  virtual bool is_async() const { return false; }
  virtual void Compute(const NodeDef& node, OpContext* ctx) = 0;
  virtual void ComputeAsync(const NodeDef& node, OpContext* ctx, std::function<void(Status)> done) {
    try {
      Compute(node, ctx);
      done(Status::OK());
    } catch (const std::exception& e) {
      done(Status::Internal(e.what()));
    }
  }
};

class KernelRegistry {
 public:
  static KernelRegistry& Get();
  void Register(const std::string& op, std::function<OpKernel*()> factory);
  OpKernel* Lookup(const std::string& op);  // cached singleton per op; nullptr if unknown
  std::vector<std::string> Ops() const;

 private:
  mutable std::mutex mu_;
  std::map<std::string, std::function<OpKernel*()>> factories_;
  std::map<std::string, std::unique_ptr<OpKernel>> cache_;
};

#define EULER_CONCAT_(a, b) a##b
#define EULER_CONCAT(a, b) EULER_CONCAT_(a, b)
#define REGISTER_OP_KERNEL(NAME, CLASS)                                                         \
  static bool EULER_CONCAT(_euler_kreg_, __COUNTER__) = [] {                                  \
    ::euler::KernelRegistry::Get().Register(NAME, [] { return new CLASS(); });               \
    return true;                                                                             \
  }()

// force-link helper: every kernel TU defines one of these, module init calls them
void LinkGraphOps();
void LinkDistOps();
void LinkMiscOps();
void LinkRemoteOp();

// ============================================================================ executor
struct ExecStats {
  std::atomic<int64_t> nodes_run{0};
  std::atomic<int64_t> remote_calls{0};
  std::atomic<int64_t> micros{0};
};

// Runs a DAG with dependency counting on a thread pool; async kernels complete
// through callbacks.  Blocking Run() returns the first error.
class Executor {
 public:
  Executor(const DAGDef& dag, OpContext* ctx, ThreadPool* pool);
  Status Run();
  void RunAsync(std::function<void(Status)> done);

 private:
  void Schedule(size_t i);
  void NodeDone(size_t i, Status st);
  const DAGDef& dag_;
  OpContext* ctx_;
  ThreadPool* pool_;
  std::vector<std::vector<size_t>> succ_;
  std::vector<std::atomic<int>> pending_;
  std::atomic<int64_t> remaining_{0};
  std::mutex mu_;
  Status status_;
  std::function<void(Status)> done_;
};

// Dependencies: which node names does `input` refer to ("A,1:0" -> "A,1")
std::string InputNode(const std::string& input);

}  // namespace euler
