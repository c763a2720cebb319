// euler_amd engine — attribute indexes and DNF filtering.
//
// Index kinds (reference euler/core/index/*):
//   hash_index       value -> sorted (id, weight) list            (EQ / NE / IN / NOT_IN)
//   range_index      rows sorted by value, binary-searched        (LT LE GT GE EQ NE IN NOT_IN)
//   hash_range_index "neighbor index": root id -> range index over that root's
//                    neighbors' values (filters outV(...).has(...) on the shard)
// An IndexResult is a sorted (id, weight) list; AND = intersection, OR = union,
// and weighted sampling under a filter draws from it (reference
// common_index_result.cc:28-125).  Values are stored as double (numeric indexes)
// or std::string (string indexes).
//
// On-disk format (reference tools/json2partindex.py:199-294):
//   Index/<name>/meta            3 x int32: index type {0 hash, 1 range, 2 neighbor}, id type, value type
//   Index/<name>/<prefix>_<p>.dat partition data (shard filter p % shard_num == shard_idx)
#pragma once

#include <stdint.h>

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "common/common.h"
#include "common/runtime.h"

namespace euler {

struct IdWeight {
  uint64_t id;
  float weight;
};

class IndexResult {
 public:
  IndexResult() = default;
  explicit IndexResult(std::vector<IdWeight> v, bool sorted = false);
  const std::vector<IdWeight>& items() const { return items_; }
  std::vector<uint64_t> ids() const;
  std::vector<float> weights() const;
  IndexResult Intersection(const IndexResult& o) const;
  IndexResult Union(const IndexResult& o) const;
  bool Contains(uint64_t id) const;
  // weighted with-replacement sampling (alias table built lazily)
  void Sample(int64_t count, Rng& rng, std::vector<IdWeight>* out) const;
  size_t size() const { return items_.size(); }

 private:
  std::vector<IdWeight> items_;  // sorted by id, unique
  mutable std::shared_ptr<AliasTable> alias_;  // built lazily (atomic_load/store)
};

enum class IndexKind : int32_t { kHash = 0, kRange = 1, kHashRange = 2 };
enum class CmpOp { LT, LE, GT, GE, EQ, NE, IN, NOT_IN };
bool ParseCmpOp(const std::string& s, CmpOp* op);

struct IndexValue {
  bool is_str = false;
  double num = 0;
  std::string str;
  static IndexValue Parse(const std::string& s, bool as_string);
  bool operator<(const IndexValue& o) const { return is_str ? str < o.str : num < o.num; }
  bool operator==(const IndexValue& o) const { return is_str ? str == o.str : num == o.num; }
};

class SampleIndex {
 public:
  virtual ~SampleIndex() = default;
  virtual IndexKind kind() const = 0;
  virtual bool string_values() const = 0;
  // plain index search; values has 1 element except for IN / NOT_IN
  virtual IndexResult Search(CmpOp op, const std::vector<IndexValue>& values) const = 0;
  // neighbor index search restricted to the neighbors of `root`
  virtual IndexResult SearchNeighbors(uint64_t root, CmpOp op, const std::vector<IndexValue>& values) const {
    (void)root;
    return Search(op, values);
  }
  virtual void Add(const IndexValue& v, uint64_t id, float w, uint64_t root = 0) = 0;
  virtual void Finalize() = 0;
  virtual size_t size() const = 0;
};

std::unique_ptr<SampleIndex> NewIndex(IndexKind kind, bool string_values);

// one DNF term: "<index name> <op> <value>[::value...]"
struct Term {
  std::string field;
  CmpOp op = CmpOp::EQ;
  std::vector<std::string> values;
  static Status Parse(const std::string& s, Term* t);
};
using Conjunction = std::vector<Term>;
using Dnf = std::vector<Conjunction>;
Status ParseDnf(const std::vector<std::string>& conj_strings, Dnf* dnf);

class IndexManager {
 public:
  void Clear();
  Status Load(const std::string& index_dir, int shard_idx, int shard_num);
  void Put(const std::string& name, std::unique_ptr<SampleIndex> idx);
  const SampleIndex* Get(const std::string& name) const;
  bool Has(const std::string& name) const { return Get(name) != nullptr; }
  // "name:hash_index|range_index|hash_range_index,..." advertised to clients
  std::string IndexInfo() const;
  std::vector<std::string> Names() const;
  // evaluate a DNF over plain indexes: OR of ANDs
  Status Query(const Dnf& dnf, IndexResult* out) const;
  // evaluate a DNF over neighbor (hash-range) indexes for one root
  Status QueryNeighbors(uint64_t root, const Dnf& dnf, IndexResult* out) const;
  bool IsNeighborIndex(const std::string& name) const;

 private:
  std::map<std::string, std::unique_ptr<SampleIndex>> indexes_;
};

}  // namespace euler
