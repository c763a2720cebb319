#include "index/index.h"

#include <algorithm>

namespace euler {

// ============================================================================ IndexResult
IndexResult::IndexResult(std::vector<IdWeight> v, bool sorted) : items_(std::move(v)) {
  if (!sorted) {
    std::sort(items_.begin(), items_.end(), [](const IdWeight& a, const IdWeight& b) { return a.id < b.id; });
    // merge duplicates (sum weights)
    std::vector<IdWeight> u;
    u.reserve(items_.size());
    for (auto& x : items_) {
      if (!u.empty() && u.back().id == x.id) u.back().weight += x.weight;
      else u.push_back(x);
    }
    items_.swap(u);
  }
}

std::vector<uint64_t> IndexResult::ids() const {
  std::vector<uint64_t> v;
  v.reserve(items_.size());
  for (auto& x : items_) v.push_back(x.id);
  return v;
}

std::vector<float> IndexResult::weights() const {
  std::vector<float> v;
  v.reserve(items_.size());
  for (auto& x : items_) v.push_back(x.weight);
  return v;
}

IndexResult IndexResult::Intersection(const IndexResult& o) const {
  std::vector<IdWeight> r;
  size_t i = 0, j = 0;
  while (i < items_.size() && j < o.items_.size()) {
    if (items_[i].id < o.items_[j].id) ++i;
    else if (o.items_[j].id < items_[i].id) ++j;
    else {
      r.push_back(items_[i]);
      ++i;
      ++j;
    }
  }
  return IndexResult(std::move(r), true);
}

IndexResult IndexResult::Union(const IndexResult& o) const {
  std::vector<IdWeight> r;
  size_t i = 0, j = 0;
  while (i < items_.size() || j < o.items_.size()) {
    if (j >= o.items_.size() || (i < items_.size() && items_[i].id < o.items_[j].id)) r.push_back(items_[i++]);
    else if (i >= items_.size() || o.items_[j].id < items_[i].id) r.push_back(o.items_[j++]);
    else {
      r.push_back(items_[i]);
      ++i;
      ++j;
    }
  }
  return IndexResult(std::move(r), true);
}

bool IndexResult::Contains(uint64_t id) const {
  auto it = std::lower_bound(items_.begin(), items_.end(), id,
                             [](const IdWeight& a, uint64_t v) { return a.id < v; });
  return it != items_.end() && it->id == id;
}

void IndexResult::Sample(int64_t count, Rng& rng, std::vector<IdWeight>* out) const {
  out->clear();
  if (items_.empty()) return;
  std::shared_ptr<AliasTable> a = std::atomic_load(&alias_);
  if (!a) {
    a = std::make_shared<AliasTable>(weights());
    std::atomic_store(&alias_, a);
  }
  for (int64_t i = 0; i < count; ++i) out->push_back(items_[a->Sample(rng)]);
}

// ============================================================================ values / ops
bool ParseCmpOp(const std::string& s, CmpOp* op) {
  static const std::map<std::string, CmpOp> m = {{"lt", CmpOp::LT}, {"le", CmpOp::LE}, {"gt", CmpOp::GT},
                                                  {"ge", CmpOp::GE}, {"eq", CmpOp::EQ}, {"ne", CmpOp::NE},
                                                  {"in", CmpOp::IN}, {"not_in", CmpOp::NOT_IN}};
  auto it = m.find(s);
  if (it == m.end()) return false;
  *op = it->second;
  return true;
}

IndexValue IndexValue::Parse(const std::string& s, bool as_string) {
  IndexValue v;
  v.is_str = as_string;
  if (as_string) v.str = s;
  else if (!ParseDouble(s, &v.num)) v.num = 0;
  return v;
}

// ============================================================================ hash index
namespace {
class HashIndex : public SampleIndex {
 public:
  explicit HashIndex(bool str) : str_(str) {}
  IndexKind kind() const override { return IndexKind::kHash; }
  bool string_values() const override { return str_; }
  void Add(const IndexValue& v, uint64_t id, float w, uint64_t) override {
    (str_ ? sbuf_[v.str] : nbuf_[v.num]).push_back({id, w});
  }
  void Finalize() override {
    for (auto& kv : sbuf_) smap_[kv.first] = std::make_shared<IndexResult>(std::move(kv.second));
    for (auto& kv : nbuf_) nmap_[kv.first] = std::make_shared<IndexResult>(std::move(kv.second));
    sbuf_.clear();
    nbuf_.clear();
  }
  size_t size() const override { return str_ ? smap_.size() : nmap_.size(); }
  IndexResult Search(CmpOp op, const std::vector<IndexValue>& vals) const override {
    IndexResult r;
    auto lookup = [&](const IndexValue& v) -> const IndexResult* {
      if (str_) {
        auto it = smap_.find(v.str);
        return it == smap_.end() ? nullptr : it->second.get();
      }
      auto it = nmap_.find(v.num);
      return it == nmap_.end() ? nullptr : it->second.get();
    };
    if (op == CmpOp::EQ || op == CmpOp::IN) {
      for (auto& v : vals)
        if (auto* p = lookup(v)) r = r.Union(*p);
      return r;
    }
    if (op == CmpOp::NE || op == CmpOp::NOT_IN) {
      auto excluded = [&](bool s, double n, const std::string& st) {
        for (auto& v : vals)
          if ((s && v.str == st) || (!s && v.num == n)) return true;
        return false;
      };
      for (auto& kv : smap_)
        if (!excluded(true, 0, kv.first)) r = r.Union(*kv.second);
      for (auto& kv : nmap_)
        if (!excluded(false, kv.first, "")) r = r.Union(*kv.second);
      return r;
    }
    // ordered comparisons on a hash index: scan keys
    for (auto& kv : nmap_) {
      const double k = kv.first, x = vals.empty() ? 0 : vals[0].num;
      bool ok = (op == CmpOp::LT && k < x) || (op == CmpOp::LE && k <= x) || (op == CmpOp::GT && k > x) ||
                (op == CmpOp::GE && k >= x);
      if (ok) r = r.Union(*kv.second);
    }
    return r;
  }

 private:
  bool str_;
  std::map<std::string, std::vector<IdWeight>> sbuf_;
  std::map<double, std::vector<IdWeight>> nbuf_;
  std::unordered_map<std::string, std::shared_ptr<IndexResult>> smap_;
  std::map<double, std::shared_ptr<IndexResult>> nmap_;
};

// rows sorted by value; results re-sorted by id
class RangeIndex : public SampleIndex {
 public:
  explicit RangeIndex(bool str) : str_(str) {}
  IndexKind kind() const override { return IndexKind::kRange; }
  bool string_values() const override { return str_; }
  void Add(const IndexValue& v, uint64_t id, float w, uint64_t) override { rows_.push_back({v, {id, w}}); }
  void Finalize() override {
    std::stable_sort(rows_.begin(), rows_.end(),
                     [](const Row& a, const Row& b) { return a.first < b.first; });
  }
  size_t size() const override { return rows_.size(); }
  IndexResult Search(CmpOp op, const std::vector<IndexValue>& vals) const override {
    std::vector<IdWeight> out;
    if (vals.empty()) return IndexResult();
    auto lb = [&](const IndexValue& v) {
      return std::lower_bound(rows_.begin(), rows_.end(), v, [](const Row& r, const IndexValue& x) { return r.first < x; });
    };
    auto ub = [&](const IndexValue& v) {
      return std::upper_bound(rows_.begin(), rows_.end(), v, [](const IndexValue& x, const Row& r) { return x < r.first; });
    };
    auto take = [&](std::vector<Row>::const_iterator a, std::vector<Row>::const_iterator b) {
      for (; a != b; ++a) out.push_back(a->second);
    };
    switch (op) {
      case CmpOp::LT: take(rows_.begin(), lb(vals[0])); break;
      case CmpOp::LE: take(rows_.begin(), ub(vals[0])); break;
      case CmpOp::GT: take(ub(vals[0]), rows_.end()); break;
      case CmpOp::GE: take(lb(vals[0]), rows_.end()); break;
      case CmpOp::EQ: take(lb(vals[0]), ub(vals[0])); break;
      case CmpOp::IN:
        for (auto& v : vals) take(lb(v), ub(v));
        break;
      case CmpOp::NE:
      case CmpOp::NOT_IN: {
        for (auto& r : rows_) {
          bool ex = false;
          for (auto& v : vals) ex = ex || (r.first == v);
          if (!ex) out.push_back(r.second);
        }
        break;
      }
    }
    return IndexResult(std::move(out));
  }

 private:
  using Row = std::pair<IndexValue, IdWeight>;
  bool str_;
  std::vector<Row> rows_;
};

class HashRangeIndex : public SampleIndex {
 public:
  explicit HashRangeIndex(bool str) : str_(str) {}
  IndexKind kind() const override { return IndexKind::kHashRange; }
  bool string_values() const override { return str_; }
  void Add(const IndexValue& v, uint64_t id, float w, uint64_t root) override {
    auto& p = per_root_[root];
    if (!p) p.reset(new RangeIndex(str_));
    p->Add(v, id, w, 0);
  }
  void Finalize() override {
    for (auto& kv : per_root_) kv.second->Finalize();
  }
  size_t size() const override { return per_root_.size(); }
  IndexResult Search(CmpOp op, const std::vector<IndexValue>& vals) const override {
    IndexResult r;
    for (auto& kv : per_root_) r = r.Union(kv.second->Search(op, vals));
    return r;
  }
  IndexResult SearchNeighbors(uint64_t root, CmpOp op, const std::vector<IndexValue>& vals) const override {
    auto it = per_root_.find(root);
    if (it == per_root_.end()) return IndexResult();
    return it->second->Search(op, vals);
  }

 private:
  bool str_;
  std::unordered_map<uint64_t, std::unique_ptr<RangeIndex>> per_root_;
};
}  // namespace

std::unique_ptr<SampleIndex> NewIndex(IndexKind kind, bool string_values) {
  switch (kind) {
    case IndexKind::kHash: return std::unique_ptr<SampleIndex>(new HashIndex(string_values));
    case IndexKind::kRange: return std::unique_ptr<SampleIndex>(new RangeIndex(string_values));
    case IndexKind::kHashRange: return std::unique_ptr<SampleIndex>(new HashRangeIndex(string_values));
  }
  return nullptr;
}

// ============================================================================ DNF
Status Term::Parse(const std::string& s, Term* t) {
  auto parts = Split(Trim(s), " \t");
  if (parts.size() < 3) return Status::InvalidArgument("bad DNF term: '" + s + "'");
  t->field = parts[0];
  if (!ParseCmpOp(parts[1], &t->op)) return Status::InvalidArgument("bad comparison op in '" + s + "'");
  t->values.clear();
  std::string rest;
  for (size_t i = 2; i < parts.size(); ++i) rest += (i > 2 ? " " : "") + parts[i];
  // IN / NOT_IN lists: "a::b::c"
  if (rest.find("::") != std::string::npos) {
    size_t p = 0;
    for (;;) {
      size_t q = rest.find("::", p);
      t->values.push_back(rest.substr(p, q == std::string::npos ? std::string::npos : q - p));
      if (q == std::string::npos) break;
      p = q + 2;
    }
  } else {
    t->values.push_back(rest);
  }
  return Status::OK();
}

Status ParseDnf(const std::vector<std::string>& conj_strings, Dnf* dnf) {
  dnf->clear();
  for (const auto& c : conj_strings) {
    Conjunction conj;
    for (const auto& ts : Split(c, ",")) {
      Term t;
      EULER_RETURN_IF_ERROR(Term::Parse(ts, &t));
      conj.push_back(t);
    }
    if (!conj.empty()) dnf->push_back(conj);
  }
  return Status::OK();
}

// ============================================================================ IndexManager
void IndexManager::Clear() { indexes_.clear(); }

void IndexManager::Put(const std::string& name, std::unique_ptr<SampleIndex> idx) {
  idx->Finalize();
  indexes_[name] = std::move(idx);
}

const SampleIndex* IndexManager::Get(const std::string& name) const {
  auto it = indexes_.find(name);
  return it == indexes_.end() ? nullptr : it->second.get();
}

bool IndexManager::IsNeighborIndex(const std::string& name) const {
  const SampleIndex* s = Get(name);
  return s && s->kind() == IndexKind::kHashRange;
}

std::vector<std::string> IndexManager::Names() const {
  std::vector<std::string> v;
  for (auto& kv : indexes_) v.push_back(kv.first);
  return v;
}

std::string IndexManager::IndexInfo() const {
  std::vector<std::string> parts;
  for (auto& kv : indexes_) {
    const char* k = kv.second->kind() == IndexKind::kHash ? "hash_index"
                    : kv.second->kind() == IndexKind::kRange ? "range_index" : "hash_range_index";
    parts.push_back(kv.first + ":" + k);
  }
  return Join(parts, ",");
}

namespace {
// type codes of json2partindex.py: int8 int16 int32 int64 uint8 uint16 uint32 uint64 float double bool string
bool ReadTyped(BytesReader& r, int type, IndexValue* v, uint64_t* as_id) {
  v->is_str = false;
  switch (type) {
    case 0: { int8_t x; if (!r.Read(&x)) return false; v->num = x; break; }
    case 1: { int16_t x; if (!r.Read(&x)) return false; v->num = x; break; }
    case 2: { int32_t x; if (!r.Read(&x)) return false; v->num = x; break; }
    case 3: { int64_t x; if (!r.Read(&x)) return false; v->num = static_cast<double>(x); break; }
    case 4: { uint8_t x; if (!r.Read(&x)) return false; v->num = x; break; }
    case 5: { uint16_t x; if (!r.Read(&x)) return false; v->num = x; break; }
    case 6: { uint32_t x; if (!r.Read(&x)) return false; v->num = x; break; }
    case 7: { uint64_t x; if (!r.Read(&x)) return false; v->num = static_cast<double>(x); if (as_id) *as_id = x; break; }
    case 8: { float x; if (!r.Read(&x)) return false; v->num = x; break; }
    case 9: { double x; if (!r.Read(&x)) return false; v->num = x; break; }
    case 10: { uint8_t x; if (!r.Read(&x)) return false; v->num = x; break; }
    case 11: { v->is_str = true; if (!r.Read(&v->str)) return false; break; }
    default: return false;
  }
  return true;
}

bool ReadIdVec(BytesReader& r, int id_type, std::vector<uint64_t>* ids) {
  uint32_t k;
  if (!r.Read(&k)) return false;
  ids->resize(k);
  for (uint32_t i = 0; i < k; ++i) {
    IndexValue v;
    uint64_t id = 0;
    if (!ReadTyped(r, id_type, &v, &id)) return false;
    (*ids)[i] = id_type == 7 ? id : static_cast<uint64_t>(v.num);
  }
  return true;
}

Status ReadRangeBlock(BytesReader& r, int id_type, int value_type, SampleIndex* idx, uint64_t root) {
  std::vector<uint64_t> ids;
  if (!ReadIdVec(r, id_type, &ids)) return Status::DataLoss("range index ids");
  uint32_t nv;
  if (!r.Read(&nv)) return Status::DataLoss("range index values");
  std::vector<IndexValue> vals(nv);
  for (uint32_t i = 0; i < nv; ++i)
    if (!ReadTyped(r, value_type, &vals[i], nullptr)) return Status::DataLoss("range index value");
  std::vector<float> cum;
  if (!r.Read(&cum)) return Status::DataLoss("range index weights");
  for (size_t i = 0; i < ids.size() && i < vals.size() && i < cum.size(); ++i)
    idx->Add(vals[i], ids[i], i > 0 ? cum[i] - cum[i - 1] : cum[i], root);  // stored cumulative
  return Status::OK();
}
}  // namespace

Status IndexManager::Load(const std::string& index_dir, int shard_idx, int shard_num) {
  std::vector<std::string> names;
  if (!ListDir(index_dir, &names).ok()) return Status::OK();  // no indexes
  for (const auto& name : names) {
    const std::string dir = JoinPath(index_dir, name);
    std::unique_ptr<FileView> mf;
    if (!FileView::Open(JoinPath(dir, "meta"), &mf).ok()) continue;
    BytesReader mr(mf->data(), mf->size());
    int32_t kind, id_type, value_type;
    if (!mr.Read(&kind) || !mr.Read(&id_type) || !mr.Read(&value_type))
      return Status::DataLoss("index meta " + name);
    auto idx = NewIndex(static_cast<IndexKind>(kind), value_type == 11);
    if (!idx) return Status::DataLoss("unknown index kind in " + name);
    std::vector<std::string> files;
    ListDir(dir, &files);
    for (const auto& fn : files) {
      if (!EndsWith(fn, ".dat")) continue;
      const std::string stem = fn.substr(0, fn.size() - 4);
      const size_t us = stem.rfind('_');
      int64_t part = 0;
      if (us == std::string::npos || !ParseInt64(stem.substr(us + 1), &part)) continue;
      if (part % shard_num != shard_idx) continue;  // reference index_manager.cc:81-89
      std::unique_ptr<FileView> df;
      EULER_RETURN_IF_ERROR(FileView::Open(JoinPath(dir, fn), &df));
      BytesReader r(df->data(), df->size());
      if (kind == 0) {
        while (r.remaining() > 0) {
          IndexValue v;
          std::vector<uint64_t> ids;
          std::vector<float> ws;
          if (!ReadTyped(r, value_type, &v, nullptr) || !ReadIdVec(r, id_type, &ids) || !r.Read(&ws))
            return Status::DataLoss("hash index data " + fn);
          for (size_t i = 0; i < ids.size(); ++i) idx->Add(v, ids[i], i < ws.size() ? ws[i] : 1.f, 0);
        }
      } else if (kind == 1) {
        EULER_RETURN_IF_ERROR(ReadRangeBlock(r, id_type, value_type, idx.get(), 0));
      } else {
        while (r.remaining() > 0) {
          IndexValue rv;
          uint64_t root = 0;
          if (!ReadTyped(r, id_type, &rv, &root)) return Status::DataLoss("neighbor index root");
          if (id_type != 7) root = static_cast<uint64_t>(rv.num);
          EULER_RETURN_IF_ERROR(ReadRangeBlock(r, id_type, value_type, idx.get(), root));
        }
      }
    }
    Put(name, std::move(idx));
  }
  return Status::OK();
}

static IndexResult EvalConj(const IndexManager& m, const Conjunction& conj, const uint64_t* root, Status* st) {
  IndexResult acc;
  bool first = true;
  for (const auto& t : conj) {
    const SampleIndex* idx = m.Get(t.field);
    if (!idx) {
      *st = Status::NotFound("no index named '" + t.field + "'");
      return IndexResult();
    }
    std::vector<IndexValue> vals;
    for (auto& s : t.values) vals.push_back(IndexValue::Parse(s, idx->string_values()));
    IndexResult r = root ? idx->SearchNeighbors(*root, t.op, vals) : idx->Search(t.op, vals);
    acc = first ? r : acc.Intersection(r);
    first = false;
  }
  return acc;
}

Status IndexManager::Query(const Dnf& dnf, IndexResult* out) const {
  Status st;
  IndexResult acc;
  for (const auto& conj : dnf) {
    acc = acc.Union(EvalConj(*this, conj, nullptr, &st));
    if (!st.ok()) return st;
  }
  *out = acc;
  return Status::OK();
}

Status IndexManager::QueryNeighbors(uint64_t root, const Dnf& dnf, IndexResult* out) const {
  Status st;
  IndexResult acc;
  for (const auto& conj : dnf) {
    acc = acc.Union(EvalConj(*this, conj, &root, &st));
    if (!st.ok()) return st;
  }
  *out = acc;
  return Status::OK();
}

}  // namespace euler
