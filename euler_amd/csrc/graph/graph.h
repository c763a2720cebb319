// euler_amd engine — sharded heterogeneous graph store.
//
// Same semantics as the reference's Graph/Node/Edge (euler/core/graph/*: typed,
// weighted adjacency grouped by edge type, sparse uint64 / dense float / binary
// node and edge features, global per-type samplers, shard filter
// part % shard_num == shard_idx), but a columnar, scale-out layout instead of one
// heap object per node (graph.h:190-193, node.h:165-179):
//
//   * rows 0..N-1 sorted by node id; id -> row through an open-addressing table
//     (identity fast path when ids are exactly 0..N-1);
//   * adjacency = CSR per direction with one segment per (row, edge type):
//       indptr[N*T + 1], nbr (raw uint64 ids, may live on other shards),
//       cumw (inclusive prefix sums restarting at each segment);
//     every segment is sorted by neighbor id (fixes SURVEY §2.10: the reference's
//     sorted-merge / node2vec code assumed sorted groups the converter never made);
//   * features are columns, one ragged column per feature index; dense columns with
//     a uniform width store no offsets;
//   * alias tables per node type / edge type for global sampling.
#pragma once

#include <stdint.h>

#include <map>
#include <memory>
#include <set>
#include <string>
#include <unordered_map>
#include <vector>

#include "common/common.h"
#include "common/runtime.h"

namespace euler {

enum FeatureType : int32_t { kSparse = 0, kDense = 1, kBinary = 2 };

struct FeatureInfo {
  std::string name;  // with type prefix, e.g. "dense_f3" (reference json2meta.py:69-86)
  FeatureType type = kDense;
  int32_t idx = 0;  // index within its type's columns
  int64_t dim = 0;
};

// euler.meta (reference graph_builder.cc:230-308, tools/graph_meta.py:71-101)
class GraphMeta {
 public:
  std::string name = "euler_amd", version = "1";
  uint64_t node_count = 0, edge_count = 0;
  uint32_t partitions_num = 1;
  std::vector<FeatureInfo> node_features, edge_features;  // in file order
  std::vector<std::pair<std::string, uint32_t>> node_types, edge_types;

  Status Load(const std::string& path);
  Status Parse(const char* data, size_t n);
  std::string Serialize() const;

  const FeatureInfo* NodeFeature(const std::string& name) const;
  const FeatureInfo* EdgeFeature(const std::string& name) const;
  int NodeTypeId(const std::string& name) const;  // -1 if unknown
  int EdgeTypeId(const std::string& name) const;
  int NumNodeTypes() const;
  int NumEdgeTypes() const;
  int NumColumns(bool node, FeatureType t) const;
  std::string ToString() const;
};

// ragged column: row r -> values[offsets[r] .. offsets[r+1]) (or r*width when uniform)
template <typename T>
struct Column {
  std::vector<uint64_t> offsets;  // empty when uniform width
  int64_t width = -1;             // >= 0 when uniform
  std::vector<T> values;
  inline void Get(int64_t r, const T** p, int64_t* n) const {
    if (width >= 0) {
      *p = values.data() + r * width;
      *n = width;
    } else if (r + 1 < static_cast<int64_t>(offsets.size())) {
      *p = values.data() + offsets[r];
      *n = static_cast<int64_t>(offsets[r + 1] - offsets[r]);
    } else {
      *p = nullptr;
      *n = 0;
    }
  }
};

struct Adjacency {
  std::vector<uint64_t> indptr;  // N*T + 1
  std::vector<uint64_t> nbr;
  std::vector<float> cumw;
  inline float SegTotal(int64_t seg) const {
    const uint64_t a = indptr[seg], b = indptr[seg + 1];
    return b > a ? cumw[b - 1] : 0.f;
  }
  inline float EdgeWeight(uint64_t e, uint64_t seg_begin) const {
    return e > seg_begin ? cumw[e] - cumw[e - 1] : cumw[e];
  }
};

class IdMap {
 public:
  void Build(const std::vector<uint64_t>& sorted_ids);
  inline int64_t Find(uint64_t id) const {
    if (identity_) return id < n_ ? static_cast<int64_t>(id) : -1;
    if (cap_ == 0) return -1;
    uint64_t h = Mix(id) & (cap_ - 1);
    for (;;) {
      const int64_t r = rows_[h];
      if (r < 0) return -1;
      if (keys_[h] == id) return r;
      h = (h + 1) & (cap_ - 1);
    }
  }

 private:
  static inline uint64_t Mix(uint64_t x) {
    x ^= x >> 33;
    x *= 0xff51afd7ed558ccdULL;
    x ^= x >> 33;
    return x;
  }
  bool identity_ = false;
  uint64_t n_ = 0, cap_ = 0;
  std::vector<uint64_t> keys_;
  std::vector<int64_t> rows_;
};

class Graph;
// Write a graph in the Euler on-disk format (euler.meta + Node/<prefix>_<p>.dat +
// Edge/<prefix>_<p>.dat, partition = id % partitions, edges with their source) — the
// byte layout GraphBuilder::LoadReferenceFormat and the reference's loader read
// (reference euler/tools/json2partdat.py, node.py, edge.py).  Partitions are written by
// `threads` workers straight from the columnar store (no per-node objects).
Status SaveReferenceFormat(const Graph& g, const std::string& dir, int partitions, int threads,
                           const std::string& prefix = "graph");
std::unique_ptr<Graph> SyntheticGraph(int64_t num_nodes, double avg_degree, int64_t max_degree, int num_node_types,
                                      int num_edge_types, int feature_dim, int label_dim, uint64_t seed,
                                      bool out_only);

struct IdWeightType {
  uint64_t id;
  float weight;
  int32_t type;
};

class Graph {
 public:
  // ------------------------------------------------------------ shape
  int64_t num_nodes() const { return static_cast<int64_t>(node_ids_.size()); }
  int64_t num_edges() const { return static_cast<int64_t>(edge_src_.size()); }
  int num_edge_types() const { return num_edge_types_; }
  int num_node_types() const { return num_node_types_; }
  const GraphMeta& meta() const { return meta_; }
  GraphMeta& mutable_meta() { return meta_; }
  int shard_idx() const { return shard_idx_; }
  int shard_num() const { return shard_num_; }

  // ------------------------------------------------------------ nodes
  inline int64_t Row(uint64_t id) const { return id_map_.Find(id); }
  inline uint64_t Id(int64_t row) const { return node_ids_[row]; }
  inline int32_t NodeType(int64_t row) const { return node_type_[row]; }
  inline float NodeWeight(int64_t row) const { return node_weight_[row]; }
  const std::vector<uint64_t>& node_ids() const { return node_ids_; }

  // ------------------------------------------------------------ neighbors (row-based, direction: out=true)
  const Adjacency& adj(bool out) const { return out ? out_ : in_; }
  // weighted with-replacement sampling over the given edge types (empty = all)
  void SampleNeighbor(int64_t row, const std::vector<int32_t>& etypes, int count, bool out, Rng& rng,
                      std::vector<IdWeightType>* res) const;
  void FullNeighbor(int64_t row, const std::vector<int32_t>& etypes, bool out, std::vector<IdWeightType>* res) const;
  void SortedFullNeighbor(int64_t row, const std::vector<int32_t>& etypes, bool out,
                          std::vector<IdWeightType>* res) const;
  void TopKNeighbor(int64_t row, const std::vector<int32_t>& etypes, int k, bool out,
                    std::vector<IdWeightType>* res) const;
  float EdgeSumWeight(int64_t row, const std::vector<int32_t>& etypes, bool out) const;

  // ------------------------------------------------------------ global sampling
  // node_type < 0: all nodes.  Weighted by node weight (reference graph.cc:333-403).
  void SampleNode(int node_type, int64_t count, Rng& rng, std::vector<uint64_t>* out) const;
  void SampleEdge(int edge_type, int64_t count, Rng& rng, std::vector<int64_t>* edge_rows) const;
  double NodeWeightSum(int node_type) const;  // node_type < 0: all
  double EdgeWeightSum(int edge_type) const;
  const std::vector<int64_t>& NodeRowsOfType(int t) const;

  // ------------------------------------------------------------ keyed (shard-independent) sampling
  // See keyed.cc.  Nodes are grouped into `buckets` virtual buckets (id % buckets, buckets a
  // multiple of the partition count, so a bucket never spans shards); the per-bucket
  // weight sums (sorted-id order, double) and in-bucket draws come out the same on a shard
  // as on the whole graph.
  std::vector<double> NodeBucketWeights(int node_type, uint64_t buckets) const;
  // one node of `bucket` by node weight (def when the bucket is empty)
  uint64_t SampleNodeInBucket(int node_type, uint64_t buckets, uint64_t bucket, Rng& rng, uint64_t def) const;

  // ------------------------------------------------------------ edges
  int64_t EdgeRow(uint64_t src, uint64_t dst, int32_t type) const;
  inline uint64_t EdgeSrc(int64_t e) const { return edge_src_[e]; }
  inline uint64_t EdgeDst(int64_t e) const { return edge_dst_[e]; }
  inline int32_t EdgeType(int64_t e) const { return edge_type_[e]; }
  inline float EdgeWeight(int64_t e) const { return edge_weight_[e]; }

  // ------------------------------------------------------------ features
  const Column<float>* NodeDense(int idx) const { return ColAt(node_dense_, idx); }
  const Column<uint64_t>* NodeSparse(int idx) const { return ColAt(node_sparse_, idx); }
  const Column<char>* NodeBinary(int idx) const { return ColAt(node_binary_, idx); }
  const Column<float>* EdgeDense(int idx) const { return ColAt(edge_dense_, idx); }
  const Column<uint64_t>* EdgeSparse(int idx) const { return ColAt(edge_sparse_, idx); }
  const Column<char>* EdgeBinary(int idx) const { return ColAt(edge_binary_, idx); }

  // graph labels (node binary feature "binary_graph_label"; reference graph.cc:441-447)
  const std::vector<std::string>& graph_labels() const { return graph_labels_; }
  std::string Summary() const;

 private:
  friend class GraphBuilder;
  friend std::unique_ptr<Graph> SyntheticGraph(int64_t, double, int64_t, int, int, int, int, uint64_t, bool);
  template <typename T>
  static const Column<T>* ColAt(const std::vector<Column<T>>& v, int idx) {
    return (idx >= 0 && idx < static_cast<int>(v.size())) ? &v[idx] : nullptr;
  }
  void BuildSamplers(bool node = true, bool edge = true);
  void BuildEdgeIndex();

  GraphMeta meta_;
  int shard_idx_ = 0, shard_num_ = 1;
  int num_edge_types_ = 1, num_node_types_ = 1;
  std::vector<uint64_t> node_ids_;
  IdMap id_map_;
  std::vector<int32_t> node_type_;
  std::vector<float> node_weight_;
  Adjacency out_, in_;
  std::vector<Column<float>> node_dense_, edge_dense_;
  std::vector<Column<uint64_t>> node_sparse_, edge_sparse_;
  std::vector<Column<char>> node_binary_, edge_binary_;
  std::vector<uint64_t> edge_src_, edge_dst_;
  std::vector<int32_t> edge_type_;
  std::vector<float> edge_weight_;
  // edge lookup: open addressing on EdgeIdHash
  std::vector<uint64_t> edge_keys_;
  std::vector<int64_t> edge_slots_;
  int edge_pbits_ = 0;  // log2 of the edge index's partitions (BuildEdgeIndex)
  // samplers
  std::vector<std::vector<int64_t>> node_rows_by_type_;
  std::vector<AliasTable> node_sampler_;  // per type; index num_node_types_ = all
  std::vector<double> node_wsum_;
  std::vector<std::vector<int64_t>> edge_rows_by_type_;
  std::vector<AliasTable> edge_sampler_;
  std::vector<double> edge_wsum_;
  std::vector<std::string> graph_labels_;
  // lazily built per-(type, buckets) samplers of SampleNodeInBucket (keyed.cc)
  struct BucketCache;
  static std::shared_ptr<BucketCache> NewBucketCache();
  std::shared_ptr<BucketCache> bucket_cache_ = NewBucketCache();
  const void* BucketSampler(int node_type, uint64_t buckets) const;
};

// Keyed sampling used by the native pipeline so that a batch is a function of
// (seed, batch, hop) only — identical whether the graph is in-process or on shard servers
// (the reference seeds its samplers from time(0), euler/common/random.cc:21-28):
//   KeyedBuckets(P)        the virtual bucket count for P data partitions (multiple of P)
//   KeyedKey(seed, b, h)   the Philox key of batch b, hop h (h = 0: roots)
//   root i                 bucket  = alias over the bucket weights, Philox (key, 2i)
//                          node    = SampleNodeInBucket(...), Philox (key, 2i + 1)
//   neighbours of ids[i]   Philox (key, KeyedStream(id, occurrence of id in ids[0..i]))
uint64_t KeyedBuckets(uint32_t partitions);
uint64_t KeyedKey(uint64_t seed, uint64_t batch, uint64_t hop);
uint64_t KeyedStream(uint64_t id, uint64_t occurrence);
// occurrence index of every ids[i] among ids[0..i]
void KeyedOccurrences(const uint64_t* ids, int64_t n, std::vector<uint32_t>* occ);
// k keyed draws per id over etypes (out edges), occ from KeyedOccurrences (any sub-range of
// a request may be drawn on its own); a node without edges / missing gets def (weight 0,
// type -1); out_w / out_t may be null
void SampleNeighborsKeyed(const Graph& g, const uint64_t* ids, const uint32_t* occ, int64_t n,
                          const std::vector<int32_t>& etypes, int k, uint64_t key, uint64_t def, uint64_t* out_id,
                          float* out_w, int32_t* out_t);

// ---------------------------------------------------------------------------
// GraphBuilder: accumulate nodes / adjacency entries / edges / features from any
// source (reference-format .dat files, numpy arrays, JSON via Python, synthetic
// generator), then Finish() sorts into the columnar layout.
// ---------------------------------------------------------------------------
// What a shard loads and which global samplers it builds (reference start_service.py:33-80
// Module NODE / EDGE / NODE_SAMPLER / EDGE_SAMPLER and graph.cc:39-70): load_data_type
// and global_sampler_type are each "none", "node", "edge" or "all".
struct LoadOptions {
  bool load_nodes = true, load_edges = true;
  bool node_sampler = true, edge_sampler = true;
  static Status Parse(const std::string& load_data_type, const std::string& global_sampler_type, LoadOptions* o);
  std::string ToString() const;
};

// Random walks [n][L + 1] over out edges (walk.cc): p = q = 1 plain weighted walks,
// otherwise node2vec-biased; etypes[s] = edge types of step s (empty = all); walk i uses
// the Philox stream (seed, i).
void RandomWalk(const Graph& g, const uint64_t* starts, int64_t n, const std::vector<std::vector<int32_t>>& etypes,
                float p, float q, int64_t default_node, uint64_t seed, int64_t* out);

class GraphBuilder {
 public:
  GraphBuilder() = default;
  void SetMeta(const GraphMeta& m) { meta_ = m; }
  GraphMeta& meta() { return meta_; }
  void SetShard(int idx, int num) {
    shard_idx_ = idx;
    shard_num_ = num;
  }
  void SetNumEdgeTypes(int t) { num_edge_types_hint_ = t; }
  void SetNumNodeTypes(int t) { num_node_types_hint_ = t; }
  void SetDeriveInFromEdges(bool v) { derive_in_from_edges_ = v; }

  // node + its feature values (features given per column index of each type)
  void AddNode(uint64_t id, int32_t type, float weight);
  void AddAdj(bool out, uint64_t node, int32_t etype, uint64_t nbr, float weight);
  void AddEdge(uint64_t src, uint64_t dst, int32_t type, float weight);
  void AddNodeDense(uint64_t id, int idx, const float* v, int64_t n);
  void AddNodeSparse(uint64_t id, int idx, const uint64_t* v, int64_t n);
  void AddNodeBinary(uint64_t id, int idx, const char* v, int64_t n);
  void AddEdgeDense(uint64_t src, uint64_t dst, int32_t t, int idx, const float* v, int64_t n);
  void AddEdgeSparse(uint64_t src, uint64_t dst, int32_t t, int idx, const uint64_t* v, int64_t n);
  void AddEdgeBinary(uint64_t src, uint64_t dst, int32_t t, int idx, const char* v, int64_t n);
  // bulk dense column in node insertion order (fast path for large synthetic graphs)
  void SetNodeDenseColumn(int idx, std::vector<float>&& values, int64_t width);

  // reference on-disk format: <dir>/euler.meta, Node/*.dat, Edge/*.dat
  Status LoadReferenceFormat(const std::string& dir, int shard_idx, int shard_num, bool load_nodes = true,
                             bool load_edges = true, int threads = 8);

  std::unique_ptr<Graph> Finish();
  // which global samplers Finish() builds (reference global_sampler_type, graph.cc:39-53)
  void SetSamplers(bool node, bool edge) {
    node_sampler_on_ = node;
    edge_sampler_on_ = edge;
  }

  int64_t pending_nodes() const { return static_cast<int64_t>(nodes_.size()); }

 private:
  bool node_sampler_on_ = true, edge_sampler_on_ = true;
  struct NodeRec {
    uint64_t id;
    int32_t type;
    float weight;
  };
  struct AdjRec {
    uint64_t node, nbr;
    int32_t type;
    float w;
  };
  struct EdgeRec {
    uint64_t src, dst;
    int32_t type;
    float w;
  };
  template <typename T>
  struct FeatRec {
    uint64_t key;  // node id or edge row
    int idx;
    std::vector<T> v;
  };
  int64_t EdgeKeyRow(uint64_t src, uint64_t dst, int32_t t);
  Status ParseNodeFile(const char* data, size_t n, std::vector<NodeRec>* nodes, std::vector<AdjRec>* adj_out,
                       std::vector<AdjRec>* adj_in, std::vector<FeatRec<float>>* fd,
                       std::vector<FeatRec<uint64_t>>* fs, std::vector<FeatRec<char>>* fb);
  Status ParseEdgeFile(const char* data, size_t n, std::vector<EdgeRec>* edges, std::vector<FeatRec<float>>* fd,
                       std::vector<FeatRec<uint64_t>>* fs, std::vector<FeatRec<char>>* fb);

  GraphMeta meta_;
  int shard_idx_ = 0, shard_num_ = 1;
  int num_edge_types_hint_ = 0, num_node_types_hint_ = 0;
  bool derive_in_from_edges_ = false;
  std::vector<NodeRec> nodes_;
  std::vector<AdjRec> adj_out_, adj_in_;
  std::vector<EdgeRec> edges_;
  std::unordered_map<uint64_t, int64_t> edge_key_rows_;  // hash -> index into edges_ (builder only)
  size_t keyed_upto_ = 0;  // edges_[0 .. keyed_upto_) are in edge_key_rows_ (built on first lookup)
  std::vector<FeatRec<float>> nd_, ed_;
  std::vector<FeatRec<uint64_t>> ns_, es_;
  std::vector<FeatRec<char>> nb_, eb_;
  std::vector<std::pair<std::vector<float>, int64_t>> dense_cols_;  // bulk columns by idx
  bool have_adj_ = false;
};

// Power-law synthetic graph built straight into the columnar layout (no builder
// sort): ids 0..N-1, node types round-robin, edges uniform targets, weights in
// [0.5, 1.5), optional dense feature "dense_feature" and label "dense_label".


}  // namespace euler
