#include "graph/graph.h"

#include <cstdio>

#include <algorithm>
#include <cmath>
#include <mutex>
#include <numeric>
#include <thread>

#include <chrono>

namespace euler {

namespace {
// load-phase timing (EULER_LOG_LEVEL=info): where a large on-disk load spends its time
struct LoadTimer {
  std::chrono::steady_clock::time_point t = std::chrono::steady_clock::now();
  void Mark(const char* phase) {
    const auto now = std::chrono::steady_clock::now();
    EULER_LOG(Info) << "graph load: " << phase << " " << std::chrono::duration<double>(now - t).count() << " s";
    t = now;
  }
};
}  // namespace


// ============================================================================ GraphMeta
Status GraphMeta::Load(const std::string& path) {
  std::unique_ptr<FileView> f;
  EULER_RETURN_IF_ERROR(FileView::Open(path, &f));
  return Parse(f->data(), f->size());
}

Status GraphMeta::Parse(const char* data, size_t n) {
  BytesReader r(data, n);
  node_features.clear();
  edge_features.clear();
  node_types.clear();
  edge_types.clear();
  uint32_t parts = 0;
  if (!r.Read(&name) || !r.Read(&version) || !r.Read(&node_count) || !r.Read(&edge_count) || !r.Read(&parts))
    return Status::DataLoss("euler.meta header truncated");
  partitions_num = parts;
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t k = 0;
    if (!r.Read(&k)) return Status::DataLoss("euler.meta feature table truncated");
    for (uint32_t i = 0; i < k; ++i) {
      FeatureInfo fi;
      int32_t t = 0;
      if (!r.Read(&fi.name) || !r.Read(&t) || !r.Read(&fi.idx) || !r.Read(&fi.dim))
        return Status::DataLoss("euler.meta feature entry truncated");
      fi.type = static_cast<FeatureType>(t);
      (pass == 0 ? node_features : edge_features).push_back(fi);
    }
  }
  for (int pass = 0; pass < 2; ++pass) {
    uint32_t k = 0;
    if (!r.Read(&k)) return Status::OK();  // older metas may stop here
    for (uint32_t i = 0; i < k; ++i) {
      std::string tn;
      uint32_t id = 0;
      if (!r.Read(&tn) || !r.Read(&id)) return Status::DataLoss("euler.meta type map truncated");
      (pass == 0 ? node_types : edge_types).emplace_back(tn, id);
    }
  }
  return Status::OK();
}

std::string GraphMeta::Serialize() const {
  BytesWriter w;
  w.Write(name);
  w.Write(version);
  w.Write(node_count);
  w.Write(edge_count);
  w.Write(partitions_num);
  for (const auto* tab : {&node_features, &edge_features}) {
    w.Write<uint32_t>(static_cast<uint32_t>(tab->size()));
    for (const auto& fi : *tab) {
      w.Write(fi.name);
      w.Write<int32_t>(fi.type);
      w.Write(fi.idx);
      w.Write(fi.dim);
    }
  }
  for (const auto* tab : {&node_types, &edge_types}) {
    w.Write<uint32_t>(static_cast<uint32_t>(tab->size()));
    for (const auto& kv : *tab) {
      w.Write(kv.first);
      w.Write(kv.second);
    }
  }
  return w.str();
}

const FeatureInfo* GraphMeta::NodeFeature(const std::string& n) const {
  for (const auto& f : node_features)
    if (f.name == n) return &f;
  return nullptr;
}
const FeatureInfo* GraphMeta::EdgeFeature(const std::string& n) const {
  for (const auto& f : edge_features)
    if (f.name == n) return &f;
  return nullptr;
}
int GraphMeta::NodeTypeId(const std::string& n) const {
  for (const auto& kv : node_types)
    if (kv.first == n) return static_cast<int>(kv.second);
  return -1;
}
int GraphMeta::EdgeTypeId(const std::string& n) const {
  for (const auto& kv : edge_types)
    if (kv.first == n) return static_cast<int>(kv.second);
  return -1;
}
int GraphMeta::NumNodeTypes() const {
  int m = 0;
  for (const auto& kv : node_types) m = std::max<int>(m, kv.second + 1);
  return m;
}
int GraphMeta::NumEdgeTypes() const {
  int m = 0;
  for (const auto& kv : edge_types) m = std::max<int>(m, kv.second + 1);
  return m;
}
int GraphMeta::NumColumns(bool node, FeatureType t) const {
  int m = 0;
  for (const auto& f : (node ? node_features : edge_features))
    if (f.type == t) m = std::max(m, f.idx + 1);
  return m;
}
std::string GraphMeta::ToString() const {
  std::ostringstream os;
  os << "GraphMeta(name=" << name << ", nodes=" << node_count << ", edges=" << edge_count
     << ", partitions=" << partitions_num << ", node_features=" << node_features.size()
     << ", edge_features=" << edge_features.size() << ", node_types=" << node_types.size()
     << ", edge_types=" << edge_types.size() << ")";
  return os.str();
}

// ============================================================================ IdMap
void IdMap::Build(const std::vector<uint64_t>& ids) {
  n_ = ids.size();
  identity_ = true;
  for (uint64_t i = 0; i < n_; ++i)
    if (ids[i] != i) {
      identity_ = false;
      break;
    }
  keys_.clear();
  rows_.clear();
  cap_ = 0;
  if (identity_) return;
  cap_ = 16;
  while (cap_ < n_ * 2) cap_ <<= 1;
  keys_.assign(cap_, 0);
  rows_.assign(cap_, -1);
  for (uint64_t i = 0; i < n_; ++i) {
    uint64_t h = Mix(ids[i]) & (cap_ - 1);
    while (rows_[h] >= 0) h = (h + 1) & (cap_ - 1);
    keys_[h] = ids[i];
    rows_[h] = static_cast<int64_t>(i);
  }
}

// ============================================================================ Graph access
static inline void ExpandTypes(const std::vector<int32_t>& in, int T, std::vector<int32_t>* out) {
  out->clear();
  if (in.empty()) {
    for (int t = 0; t < T; ++t) out->push_back(t);
  } else {
    for (int32_t t : in)
      if (t >= 0 && t < T) out->push_back(t);
  }
}

void Graph::SampleNeighbor(int64_t row, const std::vector<int32_t>& etypes, int count, bool out, Rng& rng,
                           std::vector<IdWeightType>* res) const {
  res->clear();
  if (row < 0 || row >= num_nodes() || count <= 0) return;
  const Adjacency& A = adj(out);
  const int T = num_edge_types_;
  const int64_t base = row * T;
  // pick among groups proportionally to their weight sums (reference node.cc:98-161)
  int32_t types[64];
  float tot[64];
  int ng = 0;
  float total = 0.f;
  if (etypes.empty()) {
    for (int t = 0; t < T && ng < 64; ++t) {
      const float g = A.SegTotal(base + t);
      if (g > 0.f) {
        types[ng] = t;
        total += g;
        tot[ng++] = total;
      }
    }
  } else {
    for (int32_t t : etypes) {
      if (t < 0 || t >= T || ng >= 64) continue;
      const float g = A.SegTotal(base + t);
      if (g > 0.f) {
        types[ng] = t;
        total += g;
        tot[ng++] = total;
      }
    }
  }
  if (ng == 0 || total <= 0.f) return;
  res->reserve(count);
  for (int k = 0; k < count; ++k) {
    int gi = 0;
    if (ng > 1) {
      const float u = rng.Uniform() * total;
      while (gi + 1 < ng && tot[gi] <= u) ++gi;
    }
    const int64_t seg = base + types[gi];
    const uint64_t a = A.indptr[seg], b = A.indptr[seg + 1];
    const float u = rng.Uniform() * A.cumw[b - 1];
    const int64_t e = PrefixPick(A.cumw.data(), a, b, u);
    res->push_back({A.nbr[e], A.EdgeWeight(e, a), types[gi]});
  }
}

void Graph::FullNeighbor(int64_t row, const std::vector<int32_t>& etypes, bool out,
                         std::vector<IdWeightType>* res) const {
  res->clear();
  if (row < 0 || row >= num_nodes()) return;
  const Adjacency& A = adj(out);
  std::vector<int32_t> ts;
  ExpandTypes(etypes, num_edge_types_, &ts);
  for (int32_t t : ts) {
    const int64_t seg = row * num_edge_types_ + t;
    const uint64_t a = A.indptr[seg], b = A.indptr[seg + 1];
    for (uint64_t e = a; e < b; ++e) res->push_back({A.nbr[e], A.EdgeWeight(e, a), t});
  }
}

void Graph::SortedFullNeighbor(int64_t row, const std::vector<int32_t>& etypes, bool out,
                               std::vector<IdWeightType>* res) const {
  FullNeighbor(row, etypes, out, res);
  std::stable_sort(res->begin(), res->end(), [](const IdWeightType& x, const IdWeightType& y) { return x.id < y.id; });
}

void Graph::TopKNeighbor(int64_t row, const std::vector<int32_t>& etypes, int k, bool out,
                         std::vector<IdWeightType>* res) const {
  FullNeighbor(row, etypes, out, res);
  auto cmp = [](const IdWeightType& x, const IdWeightType& y) {
    return x.weight != y.weight ? x.weight > y.weight : x.id < y.id;
  };
  if (static_cast<int64_t>(res->size()) > k) {
    std::partial_sort(res->begin(), res->begin() + k, res->end(), cmp);
    res->resize(k);
  } else {
    std::sort(res->begin(), res->end(), cmp);
  }
}

float Graph::EdgeSumWeight(int64_t row, const std::vector<int32_t>& etypes, bool out) const {
  if (row < 0 || row >= num_nodes()) return 0.f;
  const Adjacency& A = adj(out);
  std::vector<int32_t> ts;
  ExpandTypes(etypes, num_edge_types_, &ts);
  float s = 0.f;
  for (int32_t t : ts) s += A.SegTotal(row * num_edge_types_ + t);
  return s;
}

void Graph::SampleNode(int node_type, int64_t count, Rng& rng, std::vector<uint64_t>* out) const {
  out->clear();
  const int idx = (node_type < 0 || node_type >= num_node_types_) ? num_node_types_ : node_type;
  if (node_type >= num_node_types_) return;
  const AliasTable& at = node_sampler_[idx];
  if (at.empty() || at.total() <= 0) return;
  const std::vector<int64_t>* rows = idx == num_node_types_ ? nullptr : &node_rows_by_type_[idx];
  out->reserve(count);
  for (int64_t i = 0; i < count; ++i) {
    const int64_t k = at.Sample(rng);
    out->push_back(node_ids_[rows ? (*rows)[k] : k]);
  }
}

void Graph::SampleEdge(int edge_type, int64_t count, Rng& rng, std::vector<int64_t>* rows_out) const {
  rows_out->clear();
  const int ne = static_cast<int>(edge_sampler_.size()) - 1;
  const int idx = (edge_type < 0) ? ne : edge_type;
  if (idx > ne || ne < 0) return;
  const AliasTable& at = edge_sampler_[idx];
  if (at.empty() || at.total() <= 0) return;
  const std::vector<int64_t>* rows = idx == ne ? nullptr : &edge_rows_by_type_[idx];
  rows_out->reserve(count);
  for (int64_t i = 0; i < count; ++i) {
    const int64_t k = at.Sample(rng);
    rows_out->push_back(rows ? (*rows)[k] : k);
  }
}

double Graph::NodeWeightSum(int t) const {
  if (t < 0 || t >= num_node_types_) return t < 0 ? node_wsum_.back() : 0.0;
  return node_wsum_[t];
}
double Graph::EdgeWeightSum(int t) const {
  if (edge_wsum_.empty()) return 0.0;
  if (t < 0 || t >= static_cast<int>(edge_wsum_.size()) - 1) return t < 0 ? edge_wsum_.back() : 0.0;
  return edge_wsum_[t];
}
const std::vector<int64_t>& Graph::NodeRowsOfType(int t) const {
  static const std::vector<int64_t> kEmpty;
  if (t < 0 || t >= num_node_types_) return kEmpty;
  return node_rows_by_type_[t];
}

// The (src, dst, type) -> row index is an open-addressing table split into 2^edge_pbits_
// partitions by the key's top bits; each partition probes within its own slots.  Every
// partition is built by one thread scanning the edges in order, so the build is parallel
// and still deterministic (a duplicate key keeps the probe position it would get serially).
int64_t Graph::EdgeRow(uint64_t src, uint64_t dst, int32_t type) const {
  if (edge_slots_.empty()) return -1;
  const uint64_t key = EdgeIdHash(src, dst, type);
  const uint64_t capP = edge_slots_.size() >> edge_pbits_;
  const uint64_t base = edge_pbits_ ? (key >> (64 - edge_pbits_)) * capP : 0;
  uint64_t h = key & (capP - 1);
  for (;;) {
    const int64_t r = edge_slots_[base + h];
    if (r < 0) return -1;
    if (edge_keys_[base + h] == key && edge_src_[r] == src && edge_dst_[r] == dst && edge_type_[r] == type) return r;
    h = (h + 1) & (capP - 1);
  }
}

void Graph::BuildEdgeIndex() {
  const uint64_t n = edge_src_.size();
  edge_pbits_ = n >= (uint64_t{1} << 20) ? 6 : 0;  // 64 partitions for large edge tables
  const uint64_t P = uint64_t{1} << edge_pbits_;
  std::vector<uint64_t> keys(n);
  auto* pool = ThreadPool::Default();
  pool->ParallelFor(static_cast<int64_t>(n), 1 << 16, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) keys[i] = EdgeIdHash(edge_src_[i], edge_dst_[i], edge_type_[i]);
  });
  auto part = [&](uint64_t key) { return edge_pbits_ ? key >> (64 - edge_pbits_) : 0; };
  std::vector<uint64_t> cnt(P, 0);
  for (uint64_t i = 0; i < n; ++i) ++cnt[part(keys[i])];
  uint64_t mx = 1;
  for (uint64_t c : cnt) mx = std::max(mx, c);
  uint64_t capP = 16;
  while (capP < mx * 2) capP <<= 1;  // every partition at most half full
  edge_keys_.assign(capP * P, 0);
  edge_slots_.assign(capP * P, -1);
  // edges bucketed by partition, in edge order (counting sort)
  std::vector<uint64_t> off(P + 1, 0);
  for (uint64_t p = 0; p < P; ++p) off[p + 1] = off[p] + cnt[p];
  std::vector<uint64_t> order(n);
  {
    std::vector<uint64_t> cur(off.begin(), off.end() - 1);
    for (uint64_t i = 0; i < n; ++i) order[cur[part(keys[i])]++] = i;
  }
  pool->ParallelFor(static_cast<int64_t>(P), 1, [&](int64_t b, int64_t e) {
    for (int64_t p = b; p < e; ++p) {
      const uint64_t base = static_cast<uint64_t>(p) * capP;
      for (uint64_t j = off[p]; j < off[p + 1]; ++j) {
        const uint64_t i = order[j];
        const uint64_t key = keys[i];
        uint64_t h = key & (capP - 1);
        while (edge_slots_[base + h] >= 0) h = (h + 1) & (capP - 1);
        edge_keys_[base + h] = key;
        edge_slots_[base + h] = static_cast<int64_t>(i);
      }
    }
  });
}

Status LoadOptions::Parse(const std::string& data, const std::string& sampler, LoadOptions* o) {
  auto two = [](const std::string& v, const char* what, bool* a, bool* b) -> Status {
    if (v == "none") *a = false, *b = false;
    else if (v == "node") *a = true, *b = false;
    else if (v == "edge") *a = false, *b = true;
    else if (v == "all" || v.empty()) *a = true, *b = true;
    else return Status::InvalidArgument(std::string("invalid ") + what + ": '" + v + "' (none, node, edge or all)");
    return Status::OK();
  };
  EULER_RETURN_IF_ERROR(two(data, "load_data_type", &o->load_nodes, &o->load_edges));
  return two(sampler, "global_sampler_type", &o->node_sampler, &o->edge_sampler);
}

std::string LoadOptions::ToString() const {
  auto s = [](bool a, bool b) { return a ? (b ? "all" : "node") : (b ? "edge" : "none"); };
  return std::string("load_data_type=") + s(load_nodes, load_edges) + " global_sampler_type=" +
         s(node_sampler, edge_sampler);
}

void Graph::BuildSamplers(bool node_on, bool edge_on) {
  const int NT = num_node_types_;
  node_rows_by_type_.assign(NT, {});
  for (int64_t r = 0; r < num_nodes(); ++r) {
    const int t = node_type_[r];
    if (t >= 0 && t < NT) node_rows_by_type_[t].push_back(r);
  }
  node_sampler_.assign(NT + 1, AliasTable());
  node_wsum_.assign(NT + 1, 0.0);
  for (int t = 0; t < NT && node_on; ++t) {
    std::vector<float> w;
    w.reserve(node_rows_by_type_[t].size());
    for (int64_t r : node_rows_by_type_[t]) w.push_back(node_weight_[r]);
    node_sampler_[t].Init(w.data(), w.size());
    node_wsum_[t] = node_sampler_[t].total();
  }
  if (node_on) {
    node_sampler_[NT].Init(node_weight_.data(), node_weight_.size());
    node_wsum_[NT] = node_sampler_[NT].total();
  }

  const int ET = num_edge_types_;
  edge_rows_by_type_.assign(ET, {});
  for (int64_t e = 0; e < num_edges(); ++e) {
    const int t = edge_type_[e];
    if (t >= 0 && t < ET) edge_rows_by_type_[t].push_back(e);
  }
  edge_sampler_.assign(ET + 1, AliasTable());
  edge_wsum_.assign(ET + 1, 0.0);
  for (int t = 0; t < ET && edge_on; ++t) {
    std::vector<float> w;
    for (int64_t e : edge_rows_by_type_[t]) w.push_back(edge_weight_[e]);
    edge_sampler_[t].Init(w.data(), w.size());
    edge_wsum_[t] = edge_sampler_[t].total();
  }
  if (edge_on) {
    edge_sampler_[ET].Init(edge_weight_.data(), edge_weight_.size());
    edge_wsum_[ET] = edge_sampler_[ET].total();
  }

  graph_labels_.clear();
  const FeatureInfo* fi = meta_.NodeFeature("binary_graph_label");
  if (fi && fi->type == kBinary) {
    const Column<char>* c = NodeBinary(fi->idx);
    std::set<std::string> s;
    for (int64_t r = 0; c && r < num_nodes(); ++r) {
      const char* p;
      int64_t n;
      c->Get(r, &p, &n);
      if (n > 0) s.insert(std::string(p, n));
    }
    graph_labels_.assign(s.begin(), s.end());
  }
}

std::string Graph::Summary() const {
  std::ostringstream os;
  os << "Graph(shard " << shard_idx_ << "/" << shard_num_ << ", nodes=" << num_nodes() << ", out_adj="
     << out_.nbr.size() << ", in_adj=" << in_.nbr.size() << ", edges=" << num_edges()
     << ", node_types=" << num_node_types_ << ", edge_types=" << num_edge_types_ << ")";
  return os.str();
}

// ============================================================================ GraphBuilder
void GraphBuilder::AddNode(uint64_t id, int32_t type, float weight) { nodes_.push_back({id, type, weight}); }

void GraphBuilder::AddAdj(bool out, uint64_t node, int32_t etype, uint64_t nbr, float weight) {
  have_adj_ = true;
  (out ? adj_out_ : adj_in_).push_back({node, nbr, etype, weight});
}

void GraphBuilder::AddEdge(uint64_t src, uint64_t dst, int32_t type, float weight) {
  edges_.push_back({src, dst, type, weight});
}

int64_t GraphBuilder::EdgeKeyRow(uint64_t src, uint64_t dst, int32_t t) {
  // the (src, dst, type) -> row map is only needed when edge features arrive by key (the
  // API builder); the on-disk loader attaches them by row and never pays for it.  Edges
  // added since the last lookup are indexed in insertion order (a later duplicate wins).
  if (keyed_upto_ < edges_.size()) {
    edge_key_rows_.reserve(edges_.size());
    for (; keyed_upto_ < edges_.size(); ++keyed_upto_) {
      const EdgeRec& e = edges_[keyed_upto_];
      edge_key_rows_[EdgeIdHash(e.src, e.dst, e.type)] = static_cast<int64_t>(keyed_upto_);
    }
  }
  auto it = edge_key_rows_.find(EdgeIdHash(src, dst, t));
  return it == edge_key_rows_.end() ? -1 : it->second;
}

void GraphBuilder::AddNodeDense(uint64_t id, int idx, const float* v, int64_t n) {
  nd_.push_back({id, idx, std::vector<float>(v, v + n)});
}
void GraphBuilder::AddNodeSparse(uint64_t id, int idx, const uint64_t* v, int64_t n) {
  ns_.push_back({id, idx, std::vector<uint64_t>(v, v + n)});
}
void GraphBuilder::AddNodeBinary(uint64_t id, int idx, const char* v, int64_t n) {
  nb_.push_back({id, idx, std::vector<char>(v, v + n)});
}
void GraphBuilder::AddEdgeDense(uint64_t s, uint64_t d, int32_t t, int idx, const float* v, int64_t n) {
  const int64_t r = EdgeKeyRow(s, d, t);
  if (r >= 0) ed_.push_back({static_cast<uint64_t>(r), idx, std::vector<float>(v, v + n)});
}
void GraphBuilder::AddEdgeSparse(uint64_t s, uint64_t d, int32_t t, int idx, const uint64_t* v, int64_t n) {
  const int64_t r = EdgeKeyRow(s, d, t);
  if (r >= 0) es_.push_back({static_cast<uint64_t>(r), idx, std::vector<uint64_t>(v, v + n)});
}
void GraphBuilder::AddEdgeBinary(uint64_t s, uint64_t d, int32_t t, int idx, const char* v, int64_t n) {
  const int64_t r = EdgeKeyRow(s, d, t);
  if (r >= 0) eb_.push_back({static_cast<uint64_t>(r), idx, std::vector<char>(v, v + n)});
}
void GraphBuilder::SetNodeDenseColumn(int idx, std::vector<float>&& values, int64_t width) {
  if (static_cast<int>(dense_cols_.size()) <= idx) dense_cols_.resize(idx + 1);
  dense_cols_[idx] = {std::move(values), width};
}

namespace {
// parse a "<prefix>_<part>.dat" file name; -1 when it does not match
int FilePart(const std::string& name) {
  if (!EndsWith(name, ".dat")) return -1;
  const std::string stem = name.substr(0, name.size() - 4);
  const size_t us = stem.rfind('_');
  int64_t p;
  if (us == std::string::npos || !ParseInt64(stem.substr(us + 1), &p)) return -1;
  return static_cast<int>(p);
}

template <typename T>
void SplitFeatures(uint64_t key, const std::vector<int32_t>& idx, const T* vals, size_t nvals,
                   std::vector<typename std::remove_const<T>::type>* scratch, std::vector<std::pair<int, std::pair<size_t, size_t>>>* spans) {
  spans->clear();
  int32_t prev = 0;
  for (size_t i = 0; i < idx.size(); ++i) {
    const int32_t e = std::min<int32_t>(idx[i], static_cast<int32_t>(nvals));
    spans->push_back({static_cast<int>(i), {static_cast<size_t>(prev), static_cast<size_t>(std::max(prev, e))}});
    prev = e;
  }
}
}  // namespace

Status GraphBuilder::ParseNodeFile(const char* data, size_t n, std::vector<NodeRec>* nodes,
                                   std::vector<AdjRec>* adj_out, std::vector<AdjRec>* adj_in,
                                   std::vector<FeatRec<float>>* fd, std::vector<FeatRec<uint64_t>>* fs,
                                   std::vector<FeatRec<char>>* fb) {
  BytesReader file(data, n);
  std::vector<int32_t> gids, gidx, fidx;
  std::vector<float> gw, nw, fvals;
  std::vector<uint64_t> nbrs, u64vals;
  std::string bin;
  std::vector<std::pair<int, std::pair<size_t, size_t>>> spans;
  while (file.remaining() > 0) {
    uint32_t len = 0;
    if (!file.Read(&len) || file.remaining() < len) return Status::DataLoss("node record framing");
    BytesReader r(file.cur(), len);
    file.skip(len);
    NodeRec nr;
    if (!r.Read(&nr.id) || !r.Read(&nr.type) || !r.Read(&nr.weight)) return Status::DataLoss("node header");
    nodes->push_back(nr);
    for (int dir = 0; dir < 2; ++dir) {
      if (!r.Read(&gids) || !r.Read(&gw) || !r.Read(&gidx) || !r.Read(&nbrs) || !r.Read(&nw))
        return Status::DataLoss("node neighbor block id=" + std::to_string(nr.id));
      // neighbors_weight are prefix sums running across all groups (tools/node.py)
      int32_t start = 0;
      for (size_t g = 0; g < gids.size() && g < gidx.size(); ++g) {
        const int32_t end = std::min<int32_t>(gidx[g], static_cast<int32_t>(nbrs.size()));
        for (int32_t j = start; j < end; ++j) {
          const float w = j > 0 ? nw[j] - nw[j - 1] : nw[j];
          (dir == 0 ? adj_out : adj_in)->push_back({nr.id, nbrs[j], gids[g], w});
        }
        start = end;
      }
    }
    // uint64 / float / binary features
    if (!r.Read(&fidx) || !r.Read(&u64vals)) return Status::DataLoss("node sparse features");
    SplitFeatures<uint64_t>(nr.id, fidx, u64vals.data(), u64vals.size(), nullptr, &spans);
    for (auto& sp : spans)
      if (sp.second.second > sp.second.first)
        fs->push_back({nr.id, sp.first,
                       std::vector<uint64_t>(u64vals.begin() + sp.second.first, u64vals.begin() + sp.second.second)});
    if (!r.Read(&fidx) || !r.Read(&fvals)) return Status::DataLoss("node dense features");
    SplitFeatures<float>(nr.id, fidx, fvals.data(), fvals.size(), nullptr, &spans);
    for (auto& sp : spans)
      fd->push_back({nr.id, sp.first,
                     std::vector<float>(fvals.begin() + sp.second.first, fvals.begin() + sp.second.second)});
    if (!r.Read(&fidx) || !r.Read(&bin)) return Status::DataLoss("node binary features");
    SplitFeatures<char>(nr.id, fidx, bin.data(), bin.size(), nullptr, &spans);
    for (auto& sp : spans)
      if (sp.second.second > sp.second.first)
        fb->push_back({nr.id, sp.first, std::vector<char>(bin.begin() + sp.second.first, bin.begin() + sp.second.second)});
  }
  return Status::OK();
}

Status GraphBuilder::ParseEdgeFile(const char* data, size_t n, std::vector<EdgeRec>* edges,
                                   std::vector<FeatRec<float>>* fd, std::vector<FeatRec<uint64_t>>* fs,
                                   std::vector<FeatRec<char>>* fb) {
  BytesReader file(data, n);
  std::vector<int32_t> fidx;
  std::vector<float> fvals;
  std::vector<uint64_t> u64vals;
  std::string bin;
  std::vector<std::pair<int, std::pair<size_t, size_t>>> spans;
  while (file.remaining() > 0) {
    uint32_t len = 0;
    if (!file.Read(&len) || file.remaining() < len) return Status::DataLoss("edge record framing");
    BytesReader r(file.cur(), len);
    file.skip(len);
    EdgeRec er;
    if (!r.Read(&er.src) || !r.Read(&er.dst) || !r.Read(&er.type) || !r.Read(&er.w))
      return Status::DataLoss("edge header");
    // edge features are keyed by local record ordinal; re-keyed to builder rows later
    const uint64_t key = edges->size();
    edges->push_back(er);
    if (!r.Read(&fidx) || !r.Read(&u64vals)) return Status::DataLoss("edge sparse features");
    SplitFeatures<uint64_t>(key, fidx, u64vals.data(), u64vals.size(), nullptr, &spans);
    for (auto& sp : spans)
      if (sp.second.second > sp.second.first)
        fs->push_back({key, sp.first,
                       std::vector<uint64_t>(u64vals.begin() + sp.second.first, u64vals.begin() + sp.second.second)});
    if (!r.Read(&fidx) || !r.Read(&fvals)) return Status::DataLoss("edge dense features");
    SplitFeatures<float>(key, fidx, fvals.data(), fvals.size(), nullptr, &spans);
    for (auto& sp : spans)
      fd->push_back({key, sp.first, std::vector<float>(fvals.begin() + sp.second.first, fvals.begin() + sp.second.second)});
    if (!r.Read(&fidx) || !r.Read(&bin)) return Status::DataLoss("edge binary features");
    SplitFeatures<char>(key, fidx, bin.data(), bin.size(), nullptr, &spans);
    for (auto& sp : spans)
      if (sp.second.second > sp.second.first)
        fb->push_back({key, sp.first, std::vector<char>(bin.begin() + sp.second.first, bin.begin() + sp.second.second)});
  }
  return Status::OK();
}

Status GraphBuilder::LoadReferenceFormat(const std::string& dir, int shard_idx, int shard_num, bool load_nodes,
                                         bool load_edges, int threads) {
  SetShard(shard_idx, shard_num);
  EULER_RETURN_IF_ERROR(meta_.Load(JoinPath(dir, "euler.meta")));
  struct Task {
    std::string path;
    bool node;
  };
  std::vector<Task> tasks;
  for (int kind = 0; kind < 2; ++kind) {
    if ((kind == 0 && !load_nodes) || (kind == 1 && !load_edges)) continue;
    const std::string sub = JoinPath(dir, kind == 0 ? "Node" : "Edge");
    std::vector<std::string> names;
    if (!ListDir(sub, &names).ok()) continue;
    for (const auto& nm : names) {
      const int part = FilePart(nm);
      if (part < 0 || part % shard_num != shard_idx) continue;  // reference graph.cc:90-98
      tasks.push_back({JoinPath(sub, nm), kind == 0});
    }
  }
  struct Out {
    std::vector<NodeRec> nodes;
    std::vector<AdjRec> ao, ai;
    std::vector<EdgeRec> edges;
    std::vector<FeatRec<float>> nd, ed;
    std::vector<FeatRec<uint64_t>> ns, es;
    std::vector<FeatRec<char>> nb, eb;
    Status st;
  };
  std::vector<Out> outs(tasks.size());
  LoadTimer lt;
  {
    ThreadPool pool(std::max(1, std::min<int>(threads, static_cast<int>(tasks.size()))));
    Latch done(static_cast<int64_t>(tasks.size()));
    for (size_t i = 0; i < tasks.size(); ++i) {
      pool.Schedule([&, i] {
        std::unique_ptr<FileView> f;
        Out& o = outs[i];
        o.st = FileView::Open(tasks[i].path, &f);
        if (o.st.ok()) {
          if (tasks[i].node)
            o.st = ParseNodeFile(f->data(), f->size(), &o.nodes, &o.ao, &o.ai, &o.nd, &o.ns, &o.nb);
          else
            o.st = ParseEdgeFile(f->data(), f->size(), &o.edges, &o.ed, &o.es, &o.eb);
        }
        done.CountDown();
      });
    }
    done.Wait();
  }
  lt.Mark("parse files (parallel)");
  {  // one allocation per builder array for the merge below
    size_t nn = 0, nao = 0, nai = 0, ne = 0, nnd = 0, nns = 0, nnb = 0, ned = 0, nes = 0, neb = 0;
    for (const Out& o : outs) {
      nn += o.nodes.size(), nao += o.ao.size(), nai += o.ai.size(), ne += o.edges.size();
      nnd += o.nd.size(), nns += o.ns.size(), nnb += o.nb.size();
      ned += o.ed.size(), nes += o.es.size(), neb += o.eb.size();
    }
    nodes_.reserve(nodes_.size() + nn), adj_out_.reserve(adj_out_.size() + nao), adj_in_.reserve(adj_in_.size() + nai);
    edges_.reserve(edges_.size() + ne);
    nd_.reserve(nd_.size() + nnd), ns_.reserve(ns_.size() + nns), nb_.reserve(nb_.size() + nnb);
    ed_.reserve(ed_.size() + ned), es_.reserve(es_.size() + nes), eb_.reserve(eb_.size() + neb);
  }
  for (size_t i = 0; i < outs.size(); ++i) {
    Out& o = outs[i];
    if (!o.st.ok()) return Status(o.st.code(), tasks[i].path + ": " + o.st.message());
    for (auto& x : o.nodes) nodes_.push_back(x);
    for (auto& x : o.ao) adj_out_.push_back(x);
    for (auto& x : o.ai) adj_in_.push_back(x);
    have_adj_ = have_adj_ || !o.nodes.empty();
    for (auto& x : o.nd) nd_.push_back(std::move(x));
    for (auto& x : o.ns) ns_.push_back(std::move(x));
    for (auto& x : o.nb) nb_.push_back(std::move(x));
    const int64_t base = static_cast<int64_t>(edges_.size());
    for (auto& x : o.edges) AddEdge(x.src, x.dst, x.type, x.w);
    for (auto& x : o.ed) ed_.push_back({x.key + base, x.idx, std::move(x.v)});
    for (auto& x : o.es) es_.push_back({x.key + base, x.idx, std::move(x.v)});
    for (auto& x : o.eb) eb_.push_back({x.key + base, x.idx, std::move(x.v)});
    o = Out();  // release this file's records
  }
  lt.Mark("merge parsed records");
  return Status::OK();
}

namespace {
template <typename T, typename Rec, typename KeyToRow>
void FillColumns(std::vector<Rec>& recs, int ncols, int64_t nrows, std::vector<Column<T>>* cols, KeyToRow key_to_row) {
  int maxidx = ncols;
  for (auto& r : recs) maxidx = std::max(maxidx, r.idx + 1);
  cols->assign(maxidx, Column<T>());
  // group records per column, keep the last record per row
  std::vector<std::vector<std::pair<int64_t, size_t>>> per(maxidx);
  for (size_t i = 0; i < recs.size(); ++i) {
    const int64_t row = key_to_row(recs[i].key);
    if (row >= 0) per[recs[i].idx].push_back({row, i});
  }
  for (int c = 0; c < maxidx; ++c) {
    auto& v = per[c];
    std::stable_sort(v.begin(), v.end(), [](const std::pair<int64_t, size_t>& a, const std::pair<int64_t, size_t>& b) {
      return a.first < b.first;
    });
    std::vector<size_t> pick(nrows, SIZE_MAX);
    for (auto& pr : v) pick[pr.first] = pr.second;
    Column<T>& col = (*cols)[c];
    int64_t width = -2;
    bool all = true;
    for (int64_t r = 0; r < nrows; ++r) {
      if (pick[r] == SIZE_MAX) {
        all = false;
        break;
      }
      const int64_t w = static_cast<int64_t>(recs[pick[r]].v.size());
      if (width == -2) width = w;
      else if (width != w) {
        all = false;
        break;
      }
    }
    if (all && nrows > 0 && width >= 0) {
      col.width = width;
      col.values.reserve(nrows * width);
      for (int64_t r = 0; r < nrows; ++r) {
        auto& src = recs[pick[r]].v;
        col.values.insert(col.values.end(), src.begin(), src.end());
      }
    } else {
      col.width = -1;
      col.offsets.assign(nrows + 1, 0);
      for (int64_t r = 0; r < nrows; ++r) {
        const size_t n = pick[r] == SIZE_MAX ? 0 : recs[pick[r]].v.size();
        col.offsets[r + 1] = col.offsets[r] + n;
      }
      col.values.resize(col.offsets[nrows]);
      for (int64_t r = 0; r < nrows; ++r)
        if (pick[r] != SIZE_MAX) std::copy(recs[pick[r]].v.begin(), recs[pick[r]].v.end(), col.values.begin() + col.offsets[r]);
    }
  }
}

void BuildAdjacency(std::vector<std::pair<int64_t, std::pair<int32_t, std::pair<uint64_t, float>>>>& entries,
                    int64_t N, int T, Adjacency* A) {
  // entries: (row, (type, (nbr, weight))) -> CSR segments sorted by neighbor id
  A->indptr.assign(static_cast<size_t>(N) * T + 1, 0);
  for (auto& e : entries) A->indptr[e.first * T + e.second.first + 1]++;
  for (size_t i = 1; i < A->indptr.size(); ++i) A->indptr[i] += A->indptr[i - 1];
  const size_t E = entries.size();
  A->nbr.resize(E);
  A->cumw.resize(E);
  std::vector<uint64_t> pos(A->indptr.begin(), A->indptr.end() - 1);
  std::vector<float> w(E);
  for (auto& e : entries) {
    const uint64_t p = pos[e.first * T + e.second.first]++;
    A->nbr[p] = e.second.second.first;
    w[p] = e.second.second.second;
  }
  ThreadPool::Default()->ParallelFor(static_cast<int64_t>(N) * T, 4096, [&](int64_t b, int64_t en) {
    std::vector<std::pair<uint64_t, float>> tmp;
    for (int64_t s = b; s < en; ++s) {
      const uint64_t a = A->indptr[s], z = A->indptr[s + 1];
      if (z - a > 1) {
        tmp.clear();
        for (uint64_t i = a; i < z; ++i) tmp.push_back({A->nbr[i], w[i]});
        std::stable_sort(tmp.begin(), tmp.end(),
                         [](const std::pair<uint64_t, float>& x, const std::pair<uint64_t, float>& y) {
                           return x.first < y.first;
                         });
        for (uint64_t i = a; i < z; ++i) {
          A->nbr[i] = tmp[i - a].first;
          w[i] = tmp[i - a].second;
        }
      }
      float acc = 0.f;
      for (uint64_t i = a; i < z; ++i) {
        acc += std::max(0.f, w[i]);
        A->cumw[i] = acc;
      }
    }
  });
}
}  // namespace

std::unique_ptr<Graph> GraphBuilder::Finish() {
  std::unique_ptr<Graph> g(new Graph);
  LoadTimer lt;
  g->meta_ = meta_;
  g->shard_idx_ = shard_idx_;
  g->shard_num_ = shard_num_;
  // ---- nodes: sort by id, last write wins
  std::stable_sort(nodes_.begin(), nodes_.end(), [](const NodeRec& a, const NodeRec& b) { return a.id < b.id; });
  std::vector<NodeRec> uniq;
  uniq.reserve(nodes_.size());
  for (auto& n : nodes_) {
    if (!uniq.empty() && uniq.back().id == n.id) uniq.back() = n;
    else uniq.push_back(n);
  }
  const int64_t N = static_cast<int64_t>(uniq.size());
  g->node_ids_.resize(N);
  g->node_type_.resize(N);
  g->node_weight_.resize(N);
  int max_nt = 0, max_et = 0;
  for (int64_t i = 0; i < N; ++i) {
    g->node_ids_[i] = uniq[i].id;
    g->node_type_[i] = uniq[i].type;
    g->node_weight_[i] = uniq[i].weight;
    max_nt = std::max(max_nt, uniq[i].type + 1);
  }
  g->id_map_.Build(g->node_ids_);
  lt.Mark("nodes sorted + id map");
  for (auto& e : edges_) max_et = std::max(max_et, e.type + 1);
  for (auto& e : adj_out_) max_et = std::max(max_et, e.type + 1);
  for (auto& e : adj_in_) max_et = std::max(max_et, e.type + 1);
  g->num_node_types_ = std::max({1, max_nt, meta_.NumNodeTypes(), num_node_types_hint_});
  g->num_edge_types_ = std::max({1, max_et, meta_.NumEdgeTypes(), num_edge_types_hint_});
  const int T = g->num_edge_types_;
  // ---- adjacency
  using Entry = std::pair<int64_t, std::pair<int32_t, std::pair<uint64_t, float>>>;
  for (int dir = 0; dir < 2; ++dir) {
    std::vector<Entry> entries;
    entries.reserve(have_adj_ ? (dir == 0 ? adj_out_.size() : adj_in_.size()) : edges_.size());
    if (have_adj_) {
      for (auto& a : (dir == 0 ? adj_out_ : adj_in_)) {
        const int64_t r = g->Row(a.node);
        if (r >= 0 && a.type >= 0) entries.push_back({r, {a.type, {a.nbr, a.w}}});
      }
    }
    if (!have_adj_ || (dir == 1 && derive_in_from_edges_ && adj_in_.empty())) {
      for (auto& e : edges_) {
        const uint64_t node = dir == 0 ? e.src : e.dst;
        const uint64_t nbr = dir == 0 ? e.dst : e.src;
        if (dir == 1 && have_adj_ && !derive_in_from_edges_) break;
        const int64_t r = g->Row(node);
        if (r >= 0 && e.type >= 0) entries.push_back({r, {e.type, {nbr, e.w}}});
      }
    }
    BuildAdjacency(entries, N, T, dir == 0 ? &g->out_ : &g->in_);
    lt.Mark(dir == 0 ? "out adjacency" : "in adjacency");
  }
  // ---- edges (this shard owns edges whose src row is local, or all when no node filter)
  const int64_t E = static_cast<int64_t>(edges_.size());
  g->edge_src_.resize(E);
  g->edge_dst_.resize(E);
  g->edge_type_.resize(E);
  g->edge_weight_.resize(E);
  for (int64_t e = 0; e < E; ++e) {
    g->edge_src_[e] = edges_[e].src;
    g->edge_dst_[e] = edges_[e].dst;
    g->edge_type_[e] = edges_[e].type;
    g->edge_weight_[e] = edges_[e].w;
  }
  g->BuildEdgeIndex();
  lt.Mark("edge table + index");
  // ---- features
  auto node_row = [&](uint64_t id) { return g->Row(id); };
  auto edge_row = [&](uint64_t key) { return static_cast<int64_t>(key) < E ? static_cast<int64_t>(key) : -1; };
  FillColumns<float>(nd_, meta_.NumColumns(true, kDense), N, &g->node_dense_, node_row);
  FillColumns<uint64_t>(ns_, meta_.NumColumns(true, kSparse), N, &g->node_sparse_, node_row);
  FillColumns<char>(nb_, meta_.NumColumns(true, kBinary), N, &g->node_binary_, node_row);
  FillColumns<float>(ed_, meta_.NumColumns(false, kDense), E, &g->edge_dense_, edge_row);
  FillColumns<uint64_t>(es_, meta_.NumColumns(false, kSparse), E, &g->edge_sparse_, edge_row);
  FillColumns<char>(eb_, meta_.NumColumns(false, kBinary), E, &g->edge_binary_, edge_row);
  for (size_t idx = 0; idx < dense_cols_.size(); ++idx) {
    if (dense_cols_[idx].first.empty()) continue;
    if (g->node_dense_.size() <= idx) g->node_dense_.resize(idx + 1);
    Column<float>& c = g->node_dense_[idx];
    c.width = dense_cols_[idx].second;
    c.offsets.clear();
    c.values = std::move(dense_cols_[idx].first);
  }
  lt.Mark("feature columns");
  g->meta_.node_count = N;
  g->meta_.edge_count = E;
  g->BuildSamplers(node_sampler_on_, edge_sampler_on_);
  lt.Mark("samplers");
  // release builder memory
  nodes_.clear();
  adj_out_.clear();
  adj_in_.clear();
  edges_.clear();
  edge_key_rows_.clear();
  keyed_upto_ = 0;
  nd_.clear(); ns_.clear(); nb_.clear(); ed_.clear(); es_.clear(); eb_.clear();
  return g;
}

// ============================================================================ synthetic
// ============================================================================ on-disk writer
namespace {
// the feature block of one row: per feature type, the cumulative end offsets (int32, one
// per column idx) and the concatenated values (reference tools/node.py / edge.py)
template <typename T>
void WriteCols(BytesWriter* w, const std::vector<const Column<T>*>& cols, int64_t row) {
  std::vector<int32_t> idx;
  std::vector<T> vals;
  for (const Column<T>* c : cols) {
    const T* p = nullptr;
    int64_t n = 0;
    if (c) c->Get(row, &p, &n);
    vals.insert(vals.end(), p, p + n);
    idx.push_back(static_cast<int32_t>(vals.size()));
  }
  w->Write(idx);
  w->Write(vals);
}

void WriteBinaryCols(BytesWriter* w, const std::vector<const Column<char>*>& cols, int64_t row) {
  std::vector<int32_t> idx;
  std::string vals;
  for (const Column<char>* c : cols) {
    const char* p = nullptr;
    int64_t n = 0;
    if (c) c->Get(row, &p, &n);
    vals.append(p ? p : "", static_cast<size_t>(n));
    idx.push_back(static_cast<int32_t>(vals.size()));
  }
  w->Write(idx);
  w->Write(vals);
}

// one direction's neighbour block: group ids, group weight sums, cumulative group ends,
// neighbour ids, and weights as ONE prefix sum over the node's whole list
void WriteAdj(BytesWriter* w, const Adjacency& A, int64_t row, int T) {
  std::vector<int32_t> gids, gidx;
  std::vector<float> gw, nw;
  std::vector<uint64_t> nbrs;
  float run = 0.f;
  if (!A.indptr.empty()) {
    for (int t = 0; t < T; ++t) {
      const uint64_t a = A.indptr[row * T + t], b = A.indptr[row * T + t + 1];
      if (b <= a) continue;
      gids.push_back(t);
      gw.push_back(A.SegTotal(row * T + t));
      for (uint64_t k = a; k < b; ++k) {
        nbrs.push_back(A.nbr[k]);
        run += A.EdgeWeight(k, a);
        nw.push_back(run);
      }
      gidx.push_back(static_cast<int32_t>(nbrs.size()));
    }
  }
  w->Write(gids);
  w->Write(gw);
  w->Write(gidx);
  w->Write(nbrs);
  w->Write(nw);
}
}  // namespace

Status SaveReferenceFormat(const Graph& g, const std::string& dir, int partitions, int threads,
                           const std::string& prefix) {
  if (partitions < 1) return Status::InvalidArgument("partitions must be >= 1");
  EULER_RETURN_IF_ERROR(MakeDirs(JoinPath(dir, "Node")));
  EULER_RETURN_IF_ERROR(MakeDirs(JoinPath(dir, "Edge")));
  GraphMeta m = g.meta();
  m.partitions_num = static_cast<uint32_t>(partitions);
  m.node_count = static_cast<uint64_t>(g.num_nodes());
  m.edge_count = static_cast<uint64_t>(g.num_edges());
  EULER_RETURN_IF_ERROR(WriteFile(JoinPath(dir, "euler.meta"), m.Serialize()));
  const int T = std::max(1, g.num_edge_types());
  auto cols = [&](bool node, FeatureType t) {
    const int n = m.NumColumns(node, t);
    std::vector<const void*> out(n, nullptr);
    for (int i = 0; i < n; ++i) {
      if (node) out[i] = t == kDense ? static_cast<const void*>(g.NodeDense(i))
                                     : t == kSparse ? static_cast<const void*>(g.NodeSparse(i))
                                                    : static_cast<const void*>(g.NodeBinary(i));
      else out[i] = t == kDense ? static_cast<const void*>(g.EdgeDense(i))
                                : t == kSparse ? static_cast<const void*>(g.EdgeSparse(i))
                                               : static_cast<const void*>(g.EdgeBinary(i));
    }
    return out;
  };
  auto cast_f = [](const std::vector<const void*>& v) {
    std::vector<const Column<float>*> o;
    for (auto* p : v) o.push_back(static_cast<const Column<float>*>(p));
    return o;
  };
  auto cast_u = [](const std::vector<const void*>& v) {
    std::vector<const Column<uint64_t>*> o;
    for (auto* p : v) o.push_back(static_cast<const Column<uint64_t>*>(p));
    return o;
  };
  auto cast_b = [](const std::vector<const void*>& v) {
    std::vector<const Column<char>*> o;
    for (auto* p : v) o.push_back(static_cast<const Column<char>*>(p));
    return o;
  };
  const auto nd = cast_f(cols(true, kDense)), ed = cast_f(cols(false, kDense));
  const auto ns = cast_u(cols(true, kSparse)), es = cast_u(cols(false, kSparse));
  const auto nb = cast_b(cols(true, kBinary)), eb = cast_b(cols(false, kBinary));
  const int64_t N = g.num_nodes(), E = g.num_edges();
  std::vector<Status> st(static_cast<size_t>(partitions) * 2);
  ThreadPool pool(std::max(1, std::min(threads, 2 * partitions)));
  Latch done(2 * partitions);
  for (int job = 0; job < 2 * partitions; ++job) {
    pool.Schedule([&, job] {
      const int part = job % partitions;
      const bool node = job < partitions;
      const std::string path = JoinPath(JoinPath(dir, node ? "Node" : "Edge"),
                                        prefix + "_" + std::to_string(part) + ".dat");
      const std::string tmp = path + ".tmp";
      FILE* f = fopen(tmp.c_str(), "wb");
      if (!f) {
        st[job] = Status::Internal("cannot create " + tmp);
        done.CountDown();
        return;
      }
      std::string out;
      bool io_ok = true;
      BytesWriter rec;
      // records stream out in ~32 MB writes: host memory stays one buffer per worker
      auto flush_rec = [&] {
        const uint32_t len = static_cast<uint32_t>(rec.str().size());
        out.append(reinterpret_cast<const char*>(&len), 4);
        out.append(rec.str());
        rec.str().clear();
        if (out.size() >= (size_t{32} << 20)) {
          io_ok = io_ok && fwrite(out.data(), 1, out.size(), f) == out.size();
          out.clear();
        }
      };
      if (node) {
        for (int64_t r = 0; r < N; ++r) {
          if (static_cast<int>(g.Id(r) % static_cast<uint64_t>(partitions)) != part) continue;
          rec.Write(g.Id(r));
          rec.Write(g.NodeType(r));
          rec.Write(g.NodeWeight(r));
          WriteAdj(&rec, g.adj(true), r, T);
          WriteAdj(&rec, g.adj(false), r, T);
          WriteCols(&rec, ns, r);
          WriteCols(&rec, nd, r);
          WriteBinaryCols(&rec, nb, r);
          flush_rec();
        }
      } else {
        for (int64_t e = 0; e < E; ++e) {
          if (static_cast<int>(g.EdgeSrc(e) % static_cast<uint64_t>(partitions)) != part) continue;
          rec.Write(g.EdgeSrc(e));
          rec.Write(g.EdgeDst(e));
          rec.Write(g.EdgeType(e));
          rec.Write(g.EdgeWeight(e));
          WriteCols(&rec, es, e);
          WriteCols(&rec, ed, e);
          WriteBinaryCols(&rec, eb, e);
          flush_rec();
        }
      }
      io_ok = io_ok && (out.empty() || fwrite(out.data(), 1, out.size(), f) == out.size());
      io_ok = (fclose(f) == 0) && io_ok;
      st[job] = io_ok && rename(tmp.c_str(), path.c_str()) == 0 ? Status::OK() : Status::Internal("writing " + path);
      done.CountDown();
    });
  }
  done.Wait();
  for (auto& s : st) EULER_RETURN_IF_ERROR(s);
  return Status::OK();
}

std::unique_ptr<Graph> SyntheticGraph(int64_t N, double avg_degree, int64_t max_degree, int num_node_types,
                                      int num_edge_types, int feature_dim, int label_dim, uint64_t seed,
                                      bool out_only) {
  std::unique_ptr<Graph> g(new Graph);
  const int T = std::max(1, num_edge_types);
  const int NT = std::max(1, num_node_types);
  g->num_edge_types_ = T;
  g->num_node_types_ = NT;
  g->node_ids_.resize(N);
  g->node_type_.resize(N);
  g->node_weight_.assign(N, 1.f);
  for (int64_t i = 0; i < N; ++i) {
    g->node_ids_[i] = static_cast<uint64_t>(i);
    g->node_type_[i] = static_cast<int32_t>(i % NT);
  }
  g->id_map_.Build(g->node_ids_);
  ThreadPool* pool = ThreadPool::Default();
  // degrees per (row, type)
  std::vector<uint64_t>& ip = g->out_.indptr;
  ip.assign(static_cast<size_t>(N) * T + 1, 0);
  pool->ParallelFor(N, 1 << 14, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      Rng r(seed, 0x100000000ULL + i);
      const double u = std::max(1e-7, static_cast<double>(r.Uniform()));
      int64_t d = static_cast<int64_t>(avg_degree * 0.5 / std::sqrt(u));
      d = std::max<int64_t>(1, std::min<int64_t>(d, max_degree));
      for (int t = 0; t < T; ++t) ip[i * T + t + 1] = d / T + (t < d % T ? 1 : 0);
    }
  });
  for (size_t i = 1; i < ip.size(); ++i) ip[i] += ip[i - 1];
  const uint64_t E = ip.back();
  g->out_.nbr.resize(E);
  g->out_.cumw.resize(E);
  pool->ParallelFor(N, 1 << 12, [&](int64_t b, int64_t e) {
    for (int64_t i = b; i < e; ++i) {
      Rng r(seed, 0x200000000ULL + i);
      for (int t = 0; t < T; ++t) {
        const uint64_t a = ip[i * T + t], z = ip[i * T + t + 1];
        for (uint64_t k = a; k < z; ++k) {
          uint64_t v = r.Below(static_cast<uint64_t>(N));
          if (static_cast<int64_t>(v) == i) v = (v + 1) % N;
          g->out_.nbr[k] = v;
        }
        std::sort(g->out_.nbr.begin() + a, g->out_.nbr.begin() + z);
        float acc = 0.f;
        for (uint64_t k = a; k < z; ++k) {
          acc += 0.5f + r.Uniform();
          g->out_.cumw[k] = acc;
        }
      }
    }
  });
  // in-adjacency and the edge table from the out CSR (skipped for out_only graphs: a
  // sampling-only benchmark graph keeps just the out CSR, ~12 bytes per edge)
  if (out_only) {
    g->in_.indptr.assign(static_cast<size_t>(N) * T + 1, 0);
  } else {
    g->edge_src_.resize(E);
    g->edge_dst_.resize(E);
    g->edge_type_.resize(E);
    g->edge_weight_.resize(E);
    std::vector<uint64_t> in_cnt(static_cast<size_t>(N) * T + 1, 0);
    for (int64_t i = 0; i < N; ++i)
      for (int t = 0; t < T; ++t)
        for (uint64_t k = ip[i * T + t]; k < ip[i * T + t + 1]; ++k) {
          g->edge_src_[k] = i;
          g->edge_dst_[k] = g->out_.nbr[k];
          g->edge_type_[k] = t;
          g->edge_weight_[k] = g->out_.EdgeWeight(k, ip[i * T + t]);
          in_cnt[g->out_.nbr[k] * T + t + 1]++;
        }
    for (size_t i = 1; i < in_cnt.size(); ++i) in_cnt[i] += in_cnt[i - 1];
    g->in_.indptr = in_cnt;
    g->in_.nbr.resize(E);
    g->in_.cumw.resize(E);
    {
      std::vector<uint64_t> pos(in_cnt.begin(), in_cnt.end() - 1);
      std::vector<float> w(E);
      for (uint64_t k = 0; k < E; ++k) {
        const uint64_t seg = g->edge_dst_[k] * T + g->edge_type_[k];
        const uint64_t p = pos[seg]++;
        g->in_.nbr[p] = g->edge_src_[k];  // sources visited in ascending order: segments stay sorted
        w[p] = g->edge_weight_[k];
      }
      for (size_t s = 0; s + 1 < in_cnt.size(); ++s) {
        float acc = 0.f;
        for (uint64_t k = in_cnt[s]; k < in_cnt[s + 1]; ++k) {
          acc += w[k];
          g->in_.cumw[k] = acc;
        }
      }
    }
    g->BuildEdgeIndex();
  }
  // meta + features
  GraphMeta& m = g->meta_;
  m.name = "synthetic";
  m.node_count = N;
  m.edge_count = E;
  for (int t = 0; t < NT; ++t) m.node_types.emplace_back(std::to_string(t), t);
  for (int t = 0; t < T; ++t) m.edge_types.emplace_back(std::to_string(t), t);
  int dense_idx = 0;
  if (feature_dim > 0) {
    m.node_features.push_back({"dense_feature", kDense, dense_idx, feature_dim});
    Column<float> c;
    c.width = feature_dim;
    c.values.resize(static_cast<size_t>(N) * feature_dim);
    pool->ParallelFor(N, 1 << 12, [&](int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) {
        Rng r(seed, 0x300000000ULL + i);
        for (int d = 0; d < feature_dim; d += 2) {
          // Box-Muller normal pair
          const float u1 = std::max(1e-7f, r.Uniform()), u2 = r.Uniform();
          const float rad = std::sqrt(-2.f * std::log(u1));
          c.values[i * feature_dim + d] = rad * std::cos(6.2831853f * u2);
          if (d + 1 < feature_dim) c.values[i * feature_dim + d + 1] = rad * std::sin(6.2831853f * u2);
        }
      }
    });
    g->node_dense_.push_back(std::move(c));
    ++dense_idx;
  }
  if (label_dim > 0) {
    m.node_features.push_back({"dense_label", kDense, dense_idx, label_dim});
    Column<float> c;
    c.width = label_dim;
    c.values.assign(static_cast<size_t>(N) * label_dim, 0.f);
    for (int64_t i = 0; i < N; ++i) {
      int best = 0;
      if (feature_dim > 0) {
        const float* f = g->node_dense_[0].values.data() + i * feature_dim;
        for (int d = 1; d < std::min(label_dim, feature_dim); ++d)
          if (f[d] > f[best]) best = d;
      } else {
        best = static_cast<int>(i % label_dim);
      }
      c.values[i * label_dim + best] = 1.f;
    }
    g->node_dense_.push_back(std::move(c));
  }
  g->BuildSamplers();
  return g;
}

}  // namespace euler
