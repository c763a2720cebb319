// pybind11 module `euler_amd._engine`: the C++ graph engine as seen from Python.
// Plays the role of the reference's C ABI + TF custom ops (SURVEY §2.1 N25,
// tf_euler/utils/init_query_proxy.cc, euler/service/python_api.cc): numpy in,
// numpy out, the GIL released around every engine call.
#include <cstring>
#include <vector>

#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "framework/framework.h"
#include "framework/udf.h"
#include "gql/gql.h"
#include "graph/graph.h"
#include "index/index.h"
#include "pipeline/pipeline.h"
#include "rpc/rpc.h"

namespace py = pybind11;
using namespace euler;

namespace {

void Throw(const Status& st) {
  if (!st.ok()) throw std::runtime_error(st.message());
}

// ------------------------------------------------------------------ numpy <-> Tensor
Tensor FromPy(const py::handle& obj) {
  if (py::isinstance<py::str>(obj) || py::isinstance<py::bytes>(obj))
    return Tensor::Strings({obj.cast<std::string>()});
  if (py::isinstance<py::list>(obj) || py::isinstance<py::tuple>(obj)) {
    py::sequence seq = obj.cast<py::sequence>();
    bool all_str = seq.size() > 0;
    for (auto it : seq) all_str = all_str && (py::isinstance<py::str>(it) || py::isinstance<py::bytes>(it));
    if (all_str) {
      std::vector<std::string> v;
      for (auto it : seq) v.push_back(it.cast<std::string>());
      return Tensor::Strings(v);
    }
  }
  py::array arr = py::array::ensure(obj);
  if (!arr) throw std::runtime_error("cannot convert input to an array");
  if (arr.dtype().kind() == 'U' || arr.dtype().kind() == 'S' || arr.dtype().kind() == 'O') {
    std::vector<std::string> v;
    for (auto it : arr.attr("reshape")(-1)) v.push_back(py::str(it).cast<std::string>());
    std::vector<int64_t> shape(arr.shape(), arr.shape() + arr.ndim());
    return Tensor::Strings(v, shape.empty() ? std::vector<int64_t>{1} : shape);
  }
  arr = py::array::ensure(arr, py::array::c_style);
  std::vector<int64_t> shape(arr.shape(), arr.shape() + arr.ndim());
  if (shape.empty()) shape = {1};
  DType dt;
  const char k = arr.dtype().kind();
  const int sz = static_cast<int>(arr.dtype().itemsize());
  if (k == 'f') dt = sz == 4 ? DType::kFloat : DType::kDouble;
  else if (k == 'i') dt = sz == 1 ? DType::kInt8 : sz == 2 ? DType::kInt16 : sz == 4 ? DType::kInt32 : DType::kInt64;
  else if (k == 'u') dt = sz == 1 ? DType::kUInt8 : sz == 2 ? DType::kUInt16 : sz == 4 ? DType::kUInt32 : DType::kUInt64;
  else if (k == 'b') dt = DType::kBool;
  else throw std::runtime_error("unsupported numpy dtype");
  Tensor t(dt, shape);
  if (t.nbytes()) memcpy(t.raw(), arr.data(), t.nbytes());
  return t;
}

py::object ToPy(const Tensor& t) {
  std::vector<py::ssize_t> shape(t.shape().begin(), t.shape().end());
  if (t.dtype() == DType::kString) {
    py::list l;
    for (auto& s : t.strings()) l.append(py::bytes(s));
    return std::move(l);
  }
  auto mk = [&](auto tag) -> py::object {
    using T = decltype(tag);
    py::array_t<T> a(shape);
    if (t.nbytes()) memcpy(a.mutable_data(), t.raw(), t.nbytes());
    return std::move(a);
  };
  switch (t.dtype()) {
    case DType::kInt8: return mk(int8_t());
    case DType::kInt16: return mk(int16_t());
    case DType::kInt32: return mk(int32_t());
    case DType::kInt64: return mk(int64_t());
    case DType::kUInt8: case DType::kBool: return mk(uint8_t());
    case DType::kUInt16: return mk(uint16_t());
    case DType::kUInt32: return mk(uint32_t());
    case DType::kUInt64: return mk(uint64_t());
    case DType::kFloat: return mk(float());
    case DType::kDouble: return mk(double());
    default: break;
  }
  throw std::runtime_error("unsupported tensor dtype");
}

// ------------------------------------------------------------------ dataflow helpers
// tf.unique (first-occurrence order) in one pass over an open-addressing table
// (multiplicative hash, linear probing, key and slot on one cache line)
void UniqueFirst(const int64_t* xs, int64_t n, std::vector<int64_t>* uniq, int64_t* inv) {
  uint64_t cap = 16;
  while (cap < static_cast<uint64_t>(2 * n)) cap <<= 1;
  const uint64_t mask = cap - 1;
  struct Cell {
    int64_t key;
    int64_t slot;
  };
  std::vector<Cell> table(cap, Cell{0, -1});
  uniq->clear();
  uniq->reserve(static_cast<size_t>(n));
  for (int64_t i = 0; i < n; ++i) {
    const int64_t v = xs[i];
    const uint64_t z = static_cast<uint64_t>(v) * 0x9e3779b97f4a7c15ull;
    uint64_t h = (z ^ (z >> 29)) & mask;
    while (true) {
      Cell& c = table[h];
      if (c.slot < 0) {
        c.slot = static_cast<int64_t>(uniq->size());
        c.key = v;
        uniq->push_back(v);
        break;
      }
      if (c.key == v) break;
      h = (h + 1) & mask;
    }
    inv[i] = table[h].slot;
  }
}

py::array_t<int64_t> I64(const std::vector<int64_t>& v) {
  py::array_t<int64_t> a(static_cast<py::ssize_t>(v.size()));
  if (!v.empty()) memcpy(a.mutable_data(), v.data(), v.size() * sizeof(int64_t));
  return a;
}

// ------------------------------------------------------------------ Engine (QueryProxy)
class Engine {
 public:
  Engine() : proxy_(new QueryProxy) {}
  explicit Engine(std::unique_ptr<QueryProxy> p) : proxy_(std::move(p)) {}

  static std::shared_ptr<Engine> FromConfig(const std::map<std::string, std::string>& cfg) {
    auto e = std::make_shared<Engine>();
    Status st;
    {
      py::gil_scoped_release nogil;
      st = e->proxy_->Init(cfg);
    }
    Throw(st);
    return e;
  }

  py::list Run(const std::string& gql, py::dict inputs, const std::vector<std::string>& outputs) {
    std::vector<std::pair<std::string, Tensor>> in;
    for (auto kv : inputs) in.emplace_back(kv.first.cast<std::string>(), FromPy(kv.second));
    std::vector<Tensor> res;
    Status st;
    {
      py::gil_scoped_release nogil;
      st = proxy_->Run(gql, in, outputs, &res);
    }
    Throw(st);
    py::list out;
    for (auto& t : res) out.append(ToPy(t));
    return out;
  }

  py::list RunOp(const std::string& op, py::dict inputs, const std::vector<std::string>& input_names,
                 const std::vector<std::string>& attrs, int output_num) {
    std::vector<std::pair<std::string, Tensor>> in;
    for (auto kv : inputs) in.emplace_back(kv.first.cast<std::string>(), FromPy(kv.second));
    std::vector<Tensor> res;
    Status st;
    {
      py::gil_scoped_release nogil;
      st = proxy_->RunOp(op, input_names, attrs, output_num, in, &res);
    }
    Throw(st);
    py::list out;
    for (auto& t : res) out.append(ToPy(t));
    return out;
  }

  // one shard's whole graph (API_EXPORT_SHARD): ids, types, weights, indptr, neighbour ids,
  // edge weights, then one [n][dim] table per dense feature
  py::list ExportShard(int shard, const std::vector<std::string>& names, const std::vector<int64_t>& dims) {
    if (names.size() != dims.size()) throw std::invalid_argument("export_shard: one width per feature");
    std::vector<std::string> attrs(names);
    for (int64_t d : dims) attrs.push_back(std::to_string(d));
    std::vector<Tensor> res;
    Status st;
    {
      py::gil_scoped_release nogil;
      st = proxy_->RunOnShard(shard, "API_EXPORT_SHARD", attrs, 6 + static_cast<int>(names.size()), &res);
    }
    Throw(st);
    py::list out;
    for (auto& t : res) out.append(ToPy(t));
    return out;
  }

  std::string Explain(const std::string& gql) {
    std::string s;
    Throw(proxy_->Explain(gql, &s));
    return s;
  }

  py::dict Meta() const {
    const GraphMeta& m = proxy_->meta();
    py::dict d;
    d["name"] = m.name;
    d["version"] = m.version;
    d["node_count"] = m.node_count;
    d["edge_count"] = m.edge_count;
    d["partitions_num"] = m.partitions_num;
    auto feats = [](const std::vector<FeatureInfo>& v) {
      py::dict f;
      for (auto& fi : v) f[py::str(fi.name)] = py::make_tuple(static_cast<int>(fi.type), fi.idx, fi.dim);
      return f;
    };
    d["node_features"] = feats(m.node_features);
    d["edge_features"] = feats(m.edge_features);
    py::dict nt, et;
    for (auto& kv : m.node_types) nt[py::str(kv.first)] = kv.second;
    for (auto& kv : m.edge_types) et[py::str(kv.first)] = kv.second;
    d["node_types"] = nt;
    d["edge_types"] = et;
    d["mode"] = proxy_->mode();
    d["shard_num"] = proxy_->shard_num();
    d["graph_labels"] = proxy_->env()->graph_labels;
    d["index_info"] = proxy_->env()->index_info;
    return d;
  }

  QueryProxy* Proxy() const { return proxy_.get(); }
  Graph& LocalGraph() const {
    Graph* g = proxy_->local_graph();
    if (!g) throw std::runtime_error("this engine has no in-process graph (remote mode)");
    return *g;
  }

  // ---- fast local paths for the training input pipeline (no GQL, numpy in/out)
  py::array_t<uint64_t> SampleNode(int type, int64_t count) {
    Graph& g = LocalGraph();
    std::vector<uint64_t> out;
    {
      py::gil_scoped_release nogil;
      Rng rng(GlobalSeed() ^ 0x77ULL, NextOpEpoch());
      g.SampleNode(type, count, rng, &out);
    }
    py::array_t<uint64_t> a(out.size());
    if (!out.empty()) memcpy(a.mutable_data(), out.data(), out.size() * 8);
    return a;
  }

  py::tuple SampleNeighbor(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> ids,
                           std::vector<int32_t> etypes, int count, uint64_t def) {
    Graph& g = LocalGraph();
    const int64_t n = ids.size();
    py::array_t<uint64_t> oid({n, static_cast<int64_t>(count)});
    py::array_t<float> ow({n, static_cast<int64_t>(count)});
    py::array_t<int32_t> ot({n, static_cast<int64_t>(count)});
    const uint64_t* pid = ids.data();
    uint64_t* po = oid.mutable_data();
    float* pw = ow.mutable_data();
    int32_t* pt = ot.mutable_data();
    {
      py::gil_scoped_release nogil;
      const uint64_t seed = GlobalSeed() * 0x9E3779B97F4A7C15ULL + NextOpEpoch();
      const int64_t chunk = 512, nchunks = (n + chunk - 1) / chunk;
      ThreadPool::Default()->ParallelFor(nchunks, 1, [&](int64_t cb, int64_t ce) {
        std::vector<IdWeightType> tmp;
        for (int64_t c = cb; c < ce; ++c) {
          Rng rng(seed, static_cast<uint64_t>(c));
          for (int64_t i = c * chunk; i < std::min(n, (c + 1) * chunk); ++i) {
            g.SampleNeighbor(g.Row(pid[i]), etypes, count, true, rng, &tmp);
            for (int k = 0; k < count; ++k) {
              const bool ok = k < static_cast<int>(tmp.size());
              po[i * count + k] = ok ? tmp[k].id : def;
              pw[i * count + k] = ok ? tmp[k].weight : 0.f;
              pt[i * count + k] = ok ? tmp[k].type : -1;
            }
          }
        }
      });
    }
    return py::make_tuple(oid, ow, ot);
  }

  // SageDataFlow (dataflow/dataflows.py) in one call with the GIL released: per hop,
  // fixed-fanout sampling of the current node set, tf.unique of [neighbours | nodes], the
  // previous set's positions and the [2, E] edge index (+ self loops).  Returns a list of
  // (n_id, res_n_id, edge_index) int64 arrays, innermost hop first.
  py::list SageFlow(py::array_t<int64_t, py::array::c_style | py::array::forcecast> roots,
                    std::vector<std::vector<int32_t>> etypes, std::vector<int> counts, int64_t def,
                    bool self_loops) {
    Graph& g = LocalGraph();
    if (etypes.size() != counts.size()) throw std::runtime_error("one fanout per hop");
    struct Hop {
      std::vector<int64_t> n_id, res, src, dst;
    };
    std::vector<Hop> hops(etypes.size());
    std::vector<int64_t> cur(roots.data(), roots.data() + roots.size());
    {
      py::gil_scoped_release nogil;
      const uint64_t seed = GlobalSeed() * 0x9E3779B97F4A7C15ULL + NextOpEpoch();
      for (size_t h = 0; h < etypes.size(); ++h) {
        const int64_t n = static_cast<int64_t>(cur.size());
        const int k = counts[h];
        std::vector<int64_t> cat(static_cast<size_t>(n * k + n));
        const int64_t chunk = 512, nchunks = (n + chunk - 1) / chunk;
        ThreadPool::Default()->ParallelFor(nchunks, 1, [&](int64_t cb, int64_t ce) {
          std::vector<IdWeightType> tmp;
          for (int64_t c = cb; c < ce; ++c) {
            Rng rng(seed + h * 0x51ED27ULL, static_cast<uint64_t>(c));
            for (int64_t i = c * chunk; i < std::min(n, (c + 1) * chunk); ++i) {
              g.SampleNeighbor(g.Row(static_cast<uint64_t>(cur[i])), etypes[h], k, true, rng, &tmp);
              for (int j = 0; j < k; ++j)
                cat[i * k + j] = j < static_cast<int>(tmp.size()) ? static_cast<int64_t>(tmp[j].id) : def;
            }
          }
        });
        std::copy(cur.begin(), cur.end(), cat.begin() + n * k);
        Hop& o = hops[h];
        std::vector<int64_t> inv(cat.size());
        UniqueFirst(cat.data(), static_cast<int64_t>(cat.size()), &o.n_id, inv.data());
        o.res.assign(inv.end() - n, inv.end());
        const int64_t e = self_loops ? n * k + n : n * k;
        o.src.resize(static_cast<size_t>(e));
        for (int64_t i = 0; i < n * k; ++i) o.src[i] = i / k;
        if (self_loops)
          for (int64_t i = 0; i < n; ++i) o.src[n * k + i] = i;
        o.dst.assign(inv.begin(), inv.begin() + e);
        cur = o.n_id;
      }
    }
    py::list out;
    for (auto& o : hops) {
      const py::ssize_t e = static_cast<py::ssize_t>(o.src.size());
      py::array_t<int64_t> ei({static_cast<py::ssize_t>(2), e});
      if (e) {
        memcpy(ei.mutable_data(), o.src.data(), e * sizeof(int64_t));
        memcpy(ei.mutable_data() + e, o.dst.data(), e * sizeof(int64_t));
      }
      out.append(py::make_tuple(I64(o.n_id), I64(o.res), ei));
    }
    return out;
  }

  std::map<int, std::vector<std::string>> Endpoints() const { return proxy_->Endpoints(); }
  void SetReplicas(int shard, const std::vector<std::string>& eps) { Throw(proxy_->SetReplicas(shard, eps)); }

  // random walks [n, L + 1] (node2vec-biased unless p = q = 1), GIL released
  py::array_t<int64_t> RandomWalkPy(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> starts,
                                    std::vector<std::vector<int32_t>> etypes, double p, double q,
                                    int64_t default_node, uint64_t seed) {
    Graph& g = LocalGraph();
    const int64_t n = starts.size();
    const int64_t L = static_cast<int64_t>(etypes.size());
    if (p <= 0.0 || q <= 0.0) throw std::invalid_argument("random_walk: p and q must be positive");
    py::array_t<int64_t> out({n, L + 1});
    {
      py::gil_scoped_release nogil;
      RandomWalk(g, starts.data(), n, etypes, static_cast<float>(p), static_cast<float>(q), default_node, seed,
                 out.mutable_data());
    }
    return out;
  }

  // dense node feature rows (missing ids / shorter rows -> zeros), [n, dim] float32
  py::array_t<float> DenseFeature(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> ids,
                                  const std::string& name, int64_t dim) {
    Graph& g = LocalGraph();
    const FeatureInfo* fi = g.meta().NodeFeature(name);
    if (!fi || fi->type != kDense) throw std::runtime_error("no dense node feature named " + name);
    const Column<float>* c = g.NodeDense(fi->idx);
    const int64_t n = ids.size();
    py::array_t<float> out({n, dim});
    float* po = out.mutable_data();
    const uint64_t* pid = ids.data();
    {
      py::gil_scoped_release nogil;
      ThreadPool::Default()->ParallelFor(n, 1024, [&](int64_t b, int64_t e) {
        for (int64_t i = b; i < e; ++i) {
          const int64_t r = g.Row(pid[i]);
          const float* p = nullptr;
          int64_t k = 0;
          if (c && r >= 0) c->Get(r, &p, &k);
          const int64_t m = std::min(k, dim);
          if (m > 0) memcpy(po + i * dim, p, m * 4);
          if (m < dim) memset(po + i * dim + m, 0, (dim - m) * 4);
        }
      });
    }
    return out;
  }

  // whole CSR (out direction) for moving the shard into HBM: indptr, nbr rows (int32), raw weights
  py::tuple ExportCsr() {
    Graph& g = LocalGraph();
    const Adjacency& A = g.adj(true);
    py::array_t<int64_t> indptr(A.indptr.size());
    memcpy(indptr.mutable_data(), A.indptr.data(), A.indptr.size() * 8);
    py::array_t<int64_t> nbr(A.nbr.size());
    py::array_t<float> w(A.nbr.size());
    int64_t* pn = nbr.mutable_data();
    float* pw = w.mutable_data();
    {
      py::gil_scoped_release nogil;
      ThreadPool::Default()->ParallelFor(static_cast<int64_t>(g.num_nodes()) * g.num_edge_types(), 4096,
                                         [&](int64_t b, int64_t e) {
                                           for (int64_t s = b; s < e; ++s)
                                             for (uint64_t k = A.indptr[s]; k < A.indptr[s + 1]; ++k) {
                                               pn[k] = g.Row(A.nbr[k]);
                                               pw[k] = A.EdgeWeight(k, A.indptr[s]);
                                             }
                                         });
    }
    py::array_t<uint64_t> ids(g.num_nodes());
    memcpy(ids.mutable_data(), g.node_ids().data(), g.num_nodes() * 8);
    py::array_t<float> nw(g.num_nodes());
    for (int64_t r = 0; r < g.num_nodes(); ++r) nw.mutable_data()[r] = g.NodeWeight(r);
    return py::make_tuple(indptr, nbr, w, g.num_edge_types(), ids, nw);
  }

  // every edge of `etype` (-1: all) as (src ids, dst ids, weights, dense edge feature
  // `name` [n][dim] or an empty [n][0] when name is empty), edge-row order, for HBM upload
  // of a triple table (knowledge-graph trainers)
  py::tuple ExportEdges(int etype, const std::string& name, int64_t dim) {
    Graph& g = LocalGraph();
    const Column<float>* c = nullptr;
    if (!name.empty()) {
      const FeatureInfo* fi = g.meta().EdgeFeature(name);
      if (!fi || fi->type != kDense) throw std::runtime_error("no dense edge feature named " + name);
      c = g.EdgeDense(fi->idx);
    } else {
      dim = 0;
    }
    std::vector<int64_t> rows;
    for (int64_t e = 0; e < g.num_edges(); ++e)
      if (etype < 0 || g.EdgeType(e) == etype) rows.push_back(e);
    const int64_t n = static_cast<int64_t>(rows.size());
    py::array_t<uint64_t> src(n), dst(n);
    py::array_t<float> w(n);
    py::array_t<float> feat({n, dim});
    uint64_t *ps = src.mutable_data(), *pd = dst.mutable_data();
    float *pw = w.mutable_data(), *pf = feat.mutable_data();
    for (int64_t i = 0; i < n; ++i) {
      const int64_t e = rows[i];
      ps[i] = g.EdgeSrc(e);
      pd[i] = g.EdgeDst(e);
      pw[i] = g.EdgeWeight(e);
      if (dim > 0) {
        const float* p = nullptr;
        int64_t k = 0;
        if (c) c->Get(e, &p, &k);
        const int64_t m = std::min(k, dim);
        if (m > 0) memcpy(pf + i * dim, p, m * 4);
        if (m < dim) memset(pf + i * dim + m, 0, (dim - m) * 4);
      }
    }
    return py::make_tuple(src, dst, w, feat);
  }

  // per-row node ids, types and weights (row order of ExportCsr), for HBM upload
  py::tuple ExportNodes() {
    Graph& g = LocalGraph();
    const int64_t n = g.num_nodes();
    py::array_t<uint64_t> ids(n);
    py::array_t<int32_t> types(n);
    py::array_t<float> w(n);
    memcpy(ids.mutable_data(), g.node_ids().data(), n * 8);
    int32_t* pt = types.mutable_data();
    float* pw = w.mutable_data();
    for (int64_t r = 0; r < n; ++r) {
      pt[r] = g.NodeType(r);
      pw[r] = g.NodeWeight(r);
    }
    return py::make_tuple(ids, types, w);
  }

  std::string Summary() const {
    Graph* g = proxy_->local_graph();
    return g ? g->Summary() : std::string("remote engine (") + proxy_->mode() + ")";
  }

  QueryProxy* proxy() { return proxy_.get(); }

 private:
  std::unique_ptr<QueryProxy> proxy_;
};

// ------------------------------------------------------------------ builder
class PyBuilder {
 public:
  void SetMeta(const std::string& serialized) { Throw(b_.meta().Parse(serialized.data(), serialized.size())); }
  void AddNodes(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> ids,
                py::array_t<int32_t, py::array::c_style | py::array::forcecast> types,
                py::array_t<float, py::array::c_style | py::array::forcecast> weights) {
    for (py::ssize_t i = 0; i < ids.size(); ++i) b_.AddNode(ids.at(i), types.at(i), weights.at(i));
  }
  void AddEdges(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> src,
                py::array_t<uint64_t, py::array::c_style | py::array::forcecast> dst,
                py::array_t<int32_t, py::array::c_style | py::array::forcecast> types,
                py::array_t<float, py::array::c_style | py::array::forcecast> weights) {
    for (py::ssize_t i = 0; i < src.size(); ++i) b_.AddEdge(src.at(i), dst.at(i), types.at(i), weights.at(i));
  }
  void NodeDense(uint64_t id, int idx, py::array_t<float, py::array::c_style | py::array::forcecast> v) {
    b_.AddNodeDense(id, idx, v.data(), v.size());
  }
  void NodeDenseMatrix(py::array_t<uint64_t, py::array::c_style | py::array::forcecast> ids, int idx,
                       py::array_t<float, py::array::c_style | py::array::forcecast> m) {
    const int64_t d = m.ndim() == 2 ? m.shape(1) : 1;
    for (py::ssize_t i = 0; i < ids.size(); ++i) b_.AddNodeDense(ids.at(i), idx, m.data() + i * d, d);
  }
  void NodeSparse(uint64_t id, int idx, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> v) {
    b_.AddNodeSparse(id, idx, v.data(), v.size());
  }
  void NodeBinary(uint64_t id, int idx, const std::string& v) { b_.AddNodeBinary(id, idx, v.data(), v.size()); }
  void EdgeDense(uint64_t s, uint64_t d, int32_t t, int idx, py::array_t<float, py::array::c_style | py::array::forcecast> v) {
    b_.AddEdgeDense(s, d, t, idx, v.data(), v.size());
  }
  void EdgeSparse(uint64_t s, uint64_t d, int32_t t, int idx, py::array_t<uint64_t, py::array::c_style | py::array::forcecast> v) {
    b_.AddEdgeSparse(s, d, t, idx, v.data(), v.size());
  }
  void EdgeBinary(uint64_t s, uint64_t d, int32_t t, int idx, const std::string& v) {
    b_.AddEdgeBinary(s, d, t, idx, v.data(), v.size());
  }
  void DeriveIn(bool v) { b_.SetDeriveInFromEdges(v); }
  std::shared_ptr<Engine> Finish() {
    std::unique_ptr<Graph> g;
    {
      py::gil_scoped_release nogil;
      g = b_.Finish();
    }
    std::unique_ptr<QueryProxy> p(new QueryProxy);
    Throw(p->InitWithGraph(std::move(g), nullptr));
    return std::make_shared<Engine>(std::move(p));
  }

 private:
  GraphBuilder b_;
};

// ------------------------------------------------------------------ server
class PyServer {
 public:
  PyServer(const std::string& data_path, int shard_idx, int shard_num, const std::string& registry, int port,
           int threads, const std::string& host, const std::string& load_data_type,
           const std::string& global_sampler_type, int heartbeat_ms) {
    LoadOptions lopt;
    Throw(LoadOptions::Parse(load_data_type, global_sampler_type, &lopt));
    Status st;
    {
      py::gil_scoped_release nogil;
      st = LoadShard(data_path, shard_idx, shard_num, &g_, &idx_, 8, lopt);
    }
    Throw(st);
    env_ = QueryProxy::MakeEnv(g_.get(), idx_.get(), shard_num);
    ServerOptions opt;
    opt.port = port;
    opt.num_threads = threads;
    opt.registry = registry;
    opt.host = host;
    opt.heartbeat_ms = heartbeat_ms;
    if (const char* e = std::getenv("EULER_RPC_IO_THREADS")) opt.io_threads = std::max(1, std::atoi(e));
    server_.reset(new GraphServer(env_.get(), shard_idx, shard_num, opt));
    Throw(server_->Start());
  }
  int port() const { return server_->port(); }
  int64_t requests() const { return server_->requests(); }
  void Stop() {
    py::gil_scoped_release nogil;
    server_->Stop();
  }

 private:
  std::unique_ptr<Graph> g_;
  std::unique_ptr<IndexManager> idx_;
  std::unique_ptr<EngineEnv> env_;
  std::unique_ptr<GraphServer> server_;
};

// Native batch pipeline (pipeline/pipeline.h) over an engine's in-process graph; the
// slot buffers are caller-owned (pinned torch tensors), passed as raw addresses.
SageBatchSpec MakeSpec(const Graph& g, int batch, int node_type, const std::vector<std::vector<int32_t>>& etypes,
                       const std::vector<int>& fanouts, int64_t def, bool self_loops,
                       const std::vector<std::string>& dense, const std::vector<int>& dims, const std::string& label,
                       int label_dim) {
  SageBatchSpec s;
  s.batch = batch;
  s.node_type = node_type;
  s.etypes = etypes;
  s.fanouts = fanouts;
  s.default_node = def;
  s.self_loops = self_loops;
  auto dense_idx = [&](const std::string& n) {
    const FeatureInfo* fi = g.meta().NodeFeature(n);
    if (!fi || fi->type != kDense) throw std::runtime_error("no dense node feature named " + n);
    return fi->idx;
  };
  for (auto& n : dense) s.dense_idx.push_back(dense_idx(n));
  s.dense_dims = dims;
  if (!label.empty()) s.label_idx = dense_idx(label);
  s.label_dim = label.empty() ? 0 : label_dim;
  return s;
}

class PySagePipeline {
 public:
  PySagePipeline(std::shared_ptr<Engine> e, int batch, int node_type, std::vector<std::vector<int32_t>> etypes,
                 std::vector<int> fanouts, int64_t def, bool self_loops, std::vector<std::string> dense,
                 std::vector<int> dims, std::string label, int label_dim, std::vector<uintptr_t> ints,
                 std::vector<uintptr_t> floats, int workers, uint64_t seed)
      : e_(std::move(e)) {
    std::vector<int64_t*> ip;
    std::vector<float*> fp;
    for (auto a : ints) ip.push_back(reinterpret_cast<int64_t*>(a));
    for (auto a : floats) fp.push_back(reinterpret_cast<float*>(a));
    QueryProxy* q = e_->Proxy();
    if (q->mode() == "graph_partition") {
      // keyed root draws assume bucket (id % B) lives on shard (bucket % P) % S, which only an
      // id-hash partition guarantees; an arbitrary partition_fn would bias the roots
      throw std::invalid_argument("the native pipeline's keyed remote sampling needs an id-hash partition; "
                                  "graph_partition sessions train on the per-op engine path");
    }
    if (q->mode() == "remote" || q->mode() == "local_sharded") {
      // the graph lives on shard servers (or in-process shards): batches through the
      // distribute-mode GQL plans (pipeline.h RemoteSource)
      SageBatchSpec spec;
      spec.batch = batch;
      spec.node_type = node_type;
      spec.etypes = etypes;
      spec.fanouts = fanouts;
      spec.default_node = def;
      spec.self_loops = self_loops;
      spec.dense_names = dense;
      spec.dense_dims = dims;
      spec.label_name = label;
      spec.label_dim = label.empty() ? 0 : label_dim;
      p_.reset(new SagePipeline(MakeRemoteSource(q), spec, ip, fp, workers, seed));
      return;
    }
    const Graph& g = e_->LocalGraph();
    SageBatchSpec spec = MakeSpec(g, batch, node_type, etypes, fanouts, def, self_loops, dense, dims, label, label_dim);
    p_.reset(new SagePipeline(&g, spec, ip, fp, workers, seed));
  }
  ~PySagePipeline() {
    py::gil_scoped_release nogil;
    p_.reset();
  }
  int Next() {
    py::gil_scoped_release nogil;
    return p_->Next();
  }
  void Release(int slot) { p_->Release(slot); }
  void Stop() {
    py::gil_scoped_release nogil;
    p_->Stop();
  }
  int64_t batches() const { return p_->batches(); }

 private:
  std::shared_ptr<Engine> e_;
  std::unique_ptr<SagePipeline> p_;
};

}  // namespace

PYBIND11_MODULE(_engine, m) {
  m.doc() = "euler_amd C++ graph engine";
  LinkGraphOps();
  LinkDistOps();
  LinkRemoteOp();

  py::class_<Engine, std::shared_ptr<Engine>>(m, "Engine")
      .def_static("from_config", &Engine::FromConfig)
      .def("run", &Engine::Run, py::arg("gql"), py::arg("inputs"), py::arg("outputs"))
      .def("explain", &Engine::Explain)
      .def("run_op", &Engine::RunOp, py::arg("op"), py::arg("inputs"), py::arg("input_names"), py::arg("attrs"),
           py::arg("output_num"))
      .def("meta", &Engine::Meta)
      .def("summary", &Engine::Summary)
      .def("sample_node", &Engine::SampleNode)
      .def("sample_neighbor", &Engine::SampleNeighbor)
      .def("sage_flow", &Engine::SageFlow, py::arg("roots"), py::arg("edge_types"), py::arg("counts"),
           py::arg("default_node"), py::arg("self_loops") = true)
      .def("random_walk", &Engine::RandomWalkPy, py::arg("starts"), py::arg("edge_types"), py::arg("p"),
           py::arg("q"), py::arg("default_node"), py::arg("seed"))
      .def("dense_feature", &Engine::DenseFeature)
      .def("export_csr", &Engine::ExportCsr)
      .def(
          "save",
          [](Engine& e, const std::string& dir, int partitions, int threads, const std::string& prefix) {
            Graph& g = e.LocalGraph();
            Status st;
            {
              py::gil_scoped_release nogil;
              st = SaveReferenceFormat(g, dir, partitions, threads, prefix);
            }
            Throw(st);
          },
          py::arg("dir"), py::arg("partitions") = 1, py::arg("threads") = 8, py::arg("prefix") = "graph",
          "write the in-process graph in the Euler on-disk format (euler.meta + Node/Edge partitions)")
      .def("endpoints", [](Engine& e) { return e.Endpoints(); })
      .def("set_replicas", &Engine::SetReplicas, py::arg("shard"), py::arg("endpoints"))
      .def("export_nodes", &Engine::ExportNodes)
      .def("export_shard", &Engine::ExportShard, py::arg("shard"), py::arg("names") = std::vector<std::string>(),
           py::arg("dims") = std::vector<int64_t>())
      .def_property_readonly("shard_num", [](Engine& e) { return e.Proxy()->shard_num(); })
      .def_property_readonly("mode", [](Engine& e) { return e.Proxy()->mode(); })
      .def("export_edges", &Engine::ExportEdges, py::arg("edge_type"), py::arg("name") = "", py::arg("dim") = 0);

  py::class_<PySagePipeline>(m, "SagePipeline")
      .def(py::init<std::shared_ptr<Engine>, int, int, std::vector<std::vector<int32_t>>, std::vector<int>, int64_t,
                    bool, std::vector<std::string>, std::vector<int>, std::string, int, std::vector<uintptr_t>,
                    std::vector<uintptr_t>, int, uint64_t>(),
           py::arg("engine"), py::arg("batch"), py::arg("node_type"), py::arg("edge_types"), py::arg("fanouts"),
           py::arg("default_node"), py::arg("self_loops"), py::arg("dense_features"), py::arg("dense_dims"),
           py::arg("label"), py::arg("label_dim"), py::arg("ints"), py::arg("floats"), py::arg("workers"),
           py::arg("seed"))
      .def("next", &PySagePipeline::Next)
      .def("release", &PySagePipeline::Release)
      .def("stop", &PySagePipeline::Stop)
      .def_property_readonly("batches", &PySagePipeline::batches);
  m.def(
      "sage_pipeline_layout",
      [](int batch, std::vector<int> fanouts, bool self_loops, std::vector<int> dims, int label_dim) {
        SageBatchSpec s;
        s.batch = batch;
        s.fanouts = fanouts;
        s.self_loops = self_loops;
        s.dense_dims = dims;
        s.label_dim = label_dim;
        SageSlotLayout l = SageSlotLayout::Make(s);
        py::dict d;
        d["ints"] = l.ints;
        d["floats"] = l.floats;
        d["feat_dim"] = l.feat_dim;
        d["off_labels"] = l.off_labels;
        d["cap"] = l.cap;
        d["ecap"] = l.ecap;
        d["off_nid"] = l.off_nid;
        d["off_res"] = l.off_res;
        d["off_src"] = l.off_src;
        d["off_nbr"] = l.off_nbr;
        return d;
      },
      py::arg("batch"), py::arg("fanouts"), py::arg("self_loops"), py::arg("dense_dims"), py::arg("label_dim"));

  py::class_<PyBuilder>(m, "GraphBuilder")
      .def(py::init<>())
      .def("set_meta", &PyBuilder::SetMeta)
      .def("add_nodes", &PyBuilder::AddNodes)
      .def("add_edges", &PyBuilder::AddEdges)
      .def("node_dense", &PyBuilder::NodeDense)
      .def("node_dense_matrix", &PyBuilder::NodeDenseMatrix)
      .def("node_sparse", &PyBuilder::NodeSparse)
      .def("node_binary", &PyBuilder::NodeBinary)
      .def("edge_dense", &PyBuilder::EdgeDense)
      .def("edge_sparse", &PyBuilder::EdgeSparse)
      .def("edge_binary", &PyBuilder::EdgeBinary)
      .def("derive_in_from_edges", &PyBuilder::DeriveIn)
      .def("finish", &PyBuilder::Finish);

  py::class_<PyServer>(m, "GraphServer")
      .def(py::init<const std::string&, int, int, const std::string&, int, int, const std::string&, const std::string&,
                    const std::string&, int>(),
           py::arg("data_path"), py::arg("shard_idx"), py::arg("shard_num"), py::arg("registry") = "",
           py::arg("port") = 0, py::arg("threads") = 32, py::arg("host") = "127.0.0.1",
           py::arg("load_data_type") = "all", py::arg("global_sampler_type") = "all", py::arg("heartbeat_ms") = 1000)
      .def_property_readonly("port", &PyServer::port)
      .def_property_readonly("requests", &PyServer::requests)
      .def("stop", &PyServer::Stop);

  py::class_<RegistryServer>(m, "RegistryServer")
      .def(py::init([](int port) {
             auto r = std::make_unique<RegistryServer>(port);
             Throw(r->Start());
             return r;
           }),
           py::arg("port") = 0)
      .def_property_readonly("port", &RegistryServer::port)
      .def("size", &RegistryServer::size)
      .def("stop", [](RegistryServer& r) {
        py::gil_scoped_release nogil;
        r.Stop();
      });

  // (unique values in first-occurrence order, inverse) of an int64 array: tf.unique
  // semantics for the CPU dataflows (every hop of SageDataFlow / NeighborDataFlow), GIL
  // released.
  m.def(
      "unique_first",
      [](py::array_t<int64_t, py::array::c_style | py::array::forcecast> x) {
        const int64_t n = static_cast<int64_t>(x.size());
        py::array_t<int64_t> inv(n);
        std::vector<int64_t> uniq;
        {
          py::gil_scoped_release nogil;
          UniqueFirst(x.data(), n, &uniq, inv.mutable_data());
        }
        return py::make_tuple(I64(uniq), inv);
      },
      py::arg("x"));

  m.def(
      "synthetic",
      [](int64_t n, double avg_deg, int64_t max_deg, int node_types, int edge_types, int feature_dim, int label_dim,
         uint64_t seed, bool out_only) {
        std::unique_ptr<Graph> g;
        {
          py::gil_scoped_release nogil;
          g = SyntheticGraph(n, avg_deg, max_deg, node_types, edge_types, feature_dim, label_dim, seed, out_only);
        }
        std::unique_ptr<QueryProxy> p(new QueryProxy);
        Throw(p->InitWithGraph(std::move(g), nullptr));
        return std::make_shared<Engine>(std::move(p));
      },
      py::arg("num_nodes"), py::arg("avg_degree"), py::arg("max_degree"), py::arg("node_types"),
      py::arg("edge_types"), py::arg("feature_dim"), py::arg("label_dim"), py::arg("seed"),
      py::arg("out_only") = false);
  m.def("parse_gql", [](const std::string& q) {
    std::vector<GqlStep> steps;
    Throw(ParseGql(q, &steps));
    py::list out;
    for (auto& s : steps) {
      py::dict d;
      d["op"] = s.op;
      d["params"] = s.params;
      d["dnf"] = s.dnf;
      d["post"] = s.post;
      d["alias"] = s.alias;
      out.append(d);
    }
    return out;
  });
  m.def("compile_gql", [](const std::string& q, const std::string& mode, int shards, std::vector<std::string> nbr_idx,
                          bool fuse) {
    CompileOptions o;
    o.mode = mode == "local" ? CompileMode::kLocal : CompileMode::kDistribute;
    o.graph_partition = mode == "graph_partition";
    o.shard_num = shards;
    o.neighbor_indexes = nbr_idx;
    o.fuse = fuse;
    std::shared_ptr<const DAGDef> d;
    Throw(Compiler::Get().Compile(q, o, &d));
    py::list nodes;
    for (auto& n : d->nodes) {
      py::dict x;
      x["name"] = n.name();
      x["op"] = n.op;
      x["inputs"] = n.inputs;
      x["attrs"] = n.attrs;
      x["shard"] = n.shard_idx;
      std::vector<std::string> inner;
      for (auto& c : n.inner) inner.push_back(c.op);
      x["inner"] = inner;
      nodes.append(x);
    }
    return nodes;
  }, py::arg("query"), py::arg("mode") = "local", py::arg("shard_num") = 1,
     py::arg("neighbor_indexes") = std::vector<std::string>{}, py::arg("fuse") = true);
  // the REMOTE fusion pass on a hand-built DAG: nodes = [(op, id, inputs, shard)] in
  // topological order; returns [(name, op, shard, inputs, [inner op names])]
  m.def("fuse_remote_nodes", [](std::vector<std::tuple<std::string, int, std::vector<std::string>, int>> spec) {
    DAGDef d;
    for (auto& t : spec) {
      NodeDef n;
      n.op = std::get<0>(t);
      n.id = std::get<1>(t);
      n.inputs = std::get<2>(t);
      n.shard_idx = std::get<3>(t);
      if (n.op == "REMOTE") {
        NodeDef inner;
        inner.op = "INNER_" + std::to_string(n.id);
        inner.id = n.id;
        n.inner.push_back(inner);
        n.output_list.push_back(inner.Output(0));
      }
      d.nodes.push_back(n);
    }
    FuseRemoteNodes(&d);
    py::list out;
    for (auto& n : d.nodes) {
      std::vector<std::string> inner;
      for (auto& c : n.inner) inner.push_back(c.op);
      out.append(py::make_tuple(n.name(), n.op, n.shard_idx, n.inputs, inner));
    }
    return out;
  });
  m.def(
      "registry_list",
      [](const std::string& spec, double ttl) {
        std::map<int, std::vector<std::pair<Endpoint, ShardMeta>>> listing;
        Throw(Registry::Open(spec)->List(&listing, ttl));
        std::map<int, std::vector<std::string>> out;
        for (auto& kv : listing)
          for (auto& e : kv.second) out[kv.first].push_back(e.first.ToString());
        return out;
      },
      py::arg("spec"), py::arg("ttl") = 0.0);
  m.def("set_seed", [](uint64_t s) { SetGlobalSeed(s); });
  m.def("hash64", [](py::bytes b) {
    std::string s = b;
    return Hash64(s.data(), static_cast<int>(s.size()));
  });
  m.def("edge_id_hash", &EdgeIdHash);
  m.def("registered_ops", [] { return KernelRegistry::Get().Ops(); });
  m.def("registered_udfs", [] { return RegisteredUdfs(); });
  m.def("stats", [] {
    auto& c = EngineCounters::Get();
    py::dict d;
    d["queries"] = c.queries.load();
    d["compile_us"] = c.compile_us.load();
    d["exec_us"] = c.exec_us.load();
    d["dag_nodes"] = c.dag_nodes.load();
    d["remote_calls"] = c.remote_calls.load();
    d["local_connections"] = c.local_connections.load();
    d["tcp_connections"] = c.tcp_connections.load();
    d["shm_channels"] = c.shm_channels.load();
    d["shm_bytes"] = c.shm_bytes.load();
    d["rpc_attempts"] = c.rpc_attempts.load();
    d["rpc_failures"] = c.rpc_failures.load();
    d["rpc_bytes_out"] = c.rpc_bytes_out.load();
    d["rpc_bytes_in"] = c.rpc_bytes_in.load();
    d["server_requests"] = c.server_requests.load();
    d["server_us"] = c.server_us.load();
    return d;
  }, "per-stage engine counters (process-wide)");
  m.def("reset_stats", [] { EngineCounters::Get().Reset(); });
  m.def("set_op_profile", [](bool on) { SetOpProfile(on); }, py::arg("on") = true);
  m.def("op_profile", [] {
    py::dict d;
    for (auto& kv : OpProfileSnapshot()) d[py::str(kv.first)] = py::make_tuple(kv.second.first, kv.second.second);
    return d;
  });
  m.def("reset_op_profile", [] { OpProfileReset(); });
}
