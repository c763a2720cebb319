// Graph-access kernels (run on a shard server, or locally in local mode).
// Reference catalog: SURVEY §2.5 "Graph access kernels" (euler/core/kernels/*.cc).
// Input / attribute conventions (our IR):
//   API_GET_NODE            in [ids]?            dnf            -> 0 ids
//   API_GET_EDGE            in [edges n x 3]?    dnf            -> 0 edges
//   API_SAMPLE_NODE         attrs [type, count]  dnf            -> 0 ids
//   API_SAMPLE_N_WITH_TYPES attrs [types, counts]               -> 0 idx[T,2] 1 ids
//   API_SAMPLE_EDGE         attrs [type, count]                 -> 0 edges [count,3]
//   API_GET_NODE_T          in [ids]                            -> 0 types
//   API_GET_P               in [ids | edges] attrs [feature names...] udf -> 2i idx, 2i+1 values
//   API_GET_NB_NODE / API_GET_RNB_NODE  in [ids] attrs [etypes] dnf pp -> idx ids weights types
//   API_GET_NB_EDGE         in [ids] attrs [etypes]             -> 0 idx 1 edges 2 weights
//   API_SAMPLE_NB           in [ids] attrs [etypes, count, default, (key)] dnf pp -> idx ids weights types
//                           (with key: keyed draws, SampleNeighborsKeyed — shard-independent)
//   API_SAMPLE_NODE_AT      in [codes = pos * buckets + bucket] attrs [type, buckets, key, default]
//                           -> 0 ids (one per code: the keyed in-bucket draw of root pos)
//   API_NODE_BUCKET_WEIGHT  attrs [type, buckets]                -> 0 double [buckets]
//   API_GET_EDGE_SUM_WEIGHT in [ids] attrs [etypes]             -> 0 float
//   API_SAMPLE_L            in [ids] attrs [etypes, default]    -> 0 ids (one neighbor each)
//   API_SPARSE_GET_ADJ      in [roots, candidates] attrs [etypes, batch_n] -> 0 idx 1 col (int64)
//   API_GET_ADJ             in [src, dst] attrs [etypes]        -> 0 int32 exists
//   API_GET_GRAPH_BY_LABEL  in [labels]                         -> 0 idx 1 ids
#include <cmath>
#include <unordered_set>

#include "framework/udf.h"
#include "ops/ops_util.h"

namespace euler {
namespace {

Graph& G(OpContext* ctx) {
  if (!ctx->env() || !ctx->env()->graph) EULER_THROW("no graph loaded in this engine");
  return *ctx->env()->graph;
}

bool HasDnf(const NodeDef& nd) { return !nd.dnf.empty(); }

// DNF values may name query input tensors (e.g. has(price gt p0)): substitute them
Dnf GetDnf(const NodeDef& nd, OpContext* ctx) {
  Dnf d;
  Status st = ParseDnf(nd.dnf, &d);
  if (!st.ok()) EULER_THROW(st.message());
  for (auto& conj : d)
    for (auto& t : conj) {
      std::vector<std::string> vals;
      for (auto& v : t.values) {
        Tensor x;
        if (ctx->TryGet(v, &x)) {
          for (auto& s : x.ToStrings()) vals.push_back(s);
        } else {
          vals.push_back(v);
        }
      }
      t.values.swap(vals);
    }
  return d;
}

IndexResult QueryIndex(OpContext* ctx, const Dnf& d) {
  if (!ctx->env()->index) EULER_THROW("condition given but no index is loaded");
  IndexResult r;
  Status st = ctx->env()->index->Query(d, &r);
  if (!st.ok()) EULER_THROW(st.message());
  return r;
}

bool DnfUsesNeighborIndex(OpContext* ctx, const Dnf& d) {
  if (!ctx->env()->index) return false;
  for (auto& c : d)
    for (auto& t : c)
      if (ctx->env()->index->IsNeighborIndex(t.field)) return true;
  return false;
}

// ---------------------------------------------------------------- nodes
class GetNodeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    std::vector<uint64_t> out;
    const bool dnf = HasDnf(nd);
    IndexResult ir;
    if (dnf) ir = QueryIndex(ctx, GetDnf(nd, ctx));
    if (!nd.inputs.empty()) {
      for (uint64_t id : IdsOf(ctx->Get(nd.inputs[0])))
        if (g.Row(id) >= 0 && (!dnf || ir.Contains(id))) out.push_back(id);
    } else if (dnf) {
      // index scan (fixes the reference's out-of-bounds copy)
      for (uint64_t id : ir.ids())
        if (g.Row(id) >= 0) out.push_back(id);
    } else {
      out = g.node_ids();
    }
    PostProcess pp = PostProcess::Parse(nd.post_process);
    if (!pp.empty()) {
      std::vector<IdWeightType> v;
      for (uint64_t id : out) v.push_back({id, g.NodeWeight(g.Row(id)), g.NodeType(g.Row(id))});
      pp.Apply(&v);
      out.clear();
      for (auto& x : v) out.push_back(x.id);
    }
    ctx->Set(nd.Output(0), Tensor::FromVector(out));
  }
};

class GetEdgeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    std::vector<uint64_t> out;
    const bool dnf = HasDnf(nd);
    IndexResult ir;
    if (dnf) ir = QueryIndex(ctx, GetDnf(nd, ctx));  // edge index ids are EdgeIdHash values
    auto keep = [&](uint64_t s, uint64_t d, int32_t t) {
      return g.EdgeRow(s, d, t) >= 0 && (!dnf || ir.Contains(EdgeIdHash(s, d, t)));
    };
    if (!nd.inputs.empty()) {
      for (auto& e : EdgesOf(ctx->Get(nd.inputs[0])))
        if (keep(e.src, e.dst, e.type)) out.insert(out.end(), {e.src, e.dst, static_cast<uint64_t>(e.type)});
    } else {
      for (int64_t e = 0; e < g.num_edges(); ++e)
        if (!dnf || ir.Contains(EdgeIdHash(g.EdgeSrc(e), g.EdgeDst(e), g.EdgeType(e))))
          out.insert(out.end(), {g.EdgeSrc(e), g.EdgeDst(e), static_cast<uint64_t>(g.EdgeType(e))});
    }
    const int64_t m = static_cast<int64_t>(out.size() / 3);
    ctx->Set(nd.Output(0), Tensor::FromVector(out, {m, 3}));
  }
};

class SampleNodeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    if (nd.attrs.size() < 2) EULER_THROW("API_SAMPLE_NODE needs [node_type, count]");
    const int type = static_cast<int>(ctx->AttrInt(nd.attrs[0]));
    const int64_t count = ctx->AttrInt(nd.attrs[1]);
    std::vector<uint64_t> out;
    Rng rng(GlobalSeed() ^ 0x51ULL, NextEpoch());
    if (HasDnf(nd)) {
      // sample inside the filtered set, weighted by node weight (the reference used
      // the id as the weight here)
      IndexResult ir = QueryIndex(ctx, GetDnf(nd, ctx));
      std::vector<IdWeight> cand;
      for (auto& x : ir.items()) {
        const int64_t r = g.Row(x.id);
        if (r >= 0 && (type < 0 || g.NodeType(r) == type)) cand.push_back({x.id, g.NodeWeight(r)});
      }
      if (!cand.empty()) {
        IndexResult c(std::move(cand), true);
        std::vector<IdWeight> s;
        c.Sample(count, rng, &s);
        for (auto& x : s) out.push_back(x.id);
      }
    } else {
      g.SampleNode(type, count, rng, &out);
    }
    ctx->Set(nd.Output(0), Tensor::FromVector(out));
  }
};

class SampleNWithTypesOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    if (nd.attrs.size() < 2) EULER_THROW("API_SAMPLE_N_WITH_TYPES needs [types, counts]");
    auto types = ctx->AttrInts(nd.attrs[0]);
    auto counts = ctx->AttrInts(nd.attrs[1]);
    if (counts.size() == 1 && types.size() > 1) counts.assign(types.size(), counts[0]);
    Rng rng(GlobalSeed() ^ 0x52ULL, NextEpoch());
    std::vector<int64_t> cnt;
    std::vector<uint64_t> all, tmp;
    for (size_t i = 0; i < types.size(); ++i) {
      g.SampleNode(types[i], i < counts.size() ? counts[i] : 0, rng, &tmp);
      cnt.push_back(tmp.size());
      all.insert(all.end(), tmp.begin(), tmp.end());
    }
    ctx->Set(nd.Output(0), MakeIdx(cnt));
    ctx->Set(nd.Output(1), Tensor::FromVector(all));
  }
};

class SampleEdgeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    if (nd.attrs.size() < 2) EULER_THROW("API_SAMPLE_EDGE needs [edge_type, count]");
    const int type = static_cast<int>(ctx->AttrInt(nd.attrs[0]));
    const int64_t count = ctx->AttrInt(nd.attrs[1]);
    Rng rng(GlobalSeed() ^ 0x53ULL, NextEpoch());
    std::vector<int64_t> rows;
    g.SampleEdge(type, count, rng, &rows);
    std::vector<uint64_t> out;
    out.reserve(rows.size() * 3);
    for (int64_t e : rows) out.insert(out.end(), {g.EdgeSrc(e), g.EdgeDst(e), static_cast<uint64_t>(g.EdgeType(e))});
    ctx->Set(nd.Output(0), Tensor::FromVector(out, {static_cast<int64_t>(rows.size()), 3}));
  }
};

class GetNodeTypeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    auto ids = IdsOf(ctx->Get(nd.inputs.at(0)));
    std::vector<int32_t> out(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
      const int64_t r = g.Row(ids[i]);
      out[i] = r >= 0 ? g.NodeType(r) : -1;
    }
    ctx->Set(nd.Output(0), Tensor::FromVector(out));
  }
};

// ---------------------------------------------------------------- features
// values() UDFs come from the registry (framework/udf.h; built-ins in ops/udfs.cc)
std::shared_ptr<const ValuesUdf> UdfOf(const NodeDef& nd) {
  const std::string name = StartsWith(nd.udf_name, "udf_") ? nd.udf_name : "udf_" + nd.udf_name;
  auto u = FindUdf(name);
  if (!u) EULER_THROW("unknown udf " << nd.udf_name << " (registered: " << Join(RegisteredUdfs(), ", ") << ")");
  return u;
}

class GetFeatureOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    const Tensor& in = ctx->Get(nd.inputs.at(0));
    // rank-2 input with 3 columns = edges (reference get_feature_op.cc:169-240)
    const bool edges = in.shape().size() == 2 && in.dim(1) == 3;
    std::vector<int64_t> rows;
    if (edges) {
      for (auto& e : EdgesOf(in)) rows.push_back(g.EdgeRow(e.src, e.dst, e.type));
    } else {
      for (uint64_t id : IdsOf(in)) rows.push_back(g.Row(id));
    }
    const int64_t n = static_cast<int64_t>(rows.size());
    std::set<std::string> udf_feats(nd.udf_str_params.begin(), nd.udf_str_params.end());
    for (size_t f = 0; f < nd.attrs.size(); ++f) {
      const std::string fname = ctx->AttrStr(nd.attrs[f]);
      const FeatureInfo* fi = edges ? g.meta().EdgeFeature(fname) : g.meta().NodeFeature(fname);
      std::vector<int64_t> counts(n, 0);
      if (!fi) {
        // unknown feature: empty rows (graphs without that feature on this shard)
        ctx->Set(nd.Output(2 * f), MakeIdx(counts));
        ctx->Set(nd.Output(2 * f + 1), Tensor(DType::kFloat, {0}));
        continue;
      }
      const bool apply_udf = !nd.udf_name.empty() &&
                             (udf_feats.empty() || udf_feats.count(fname) || udf_feats.count(nd.attrs[f]));
      if (fi->type == kDense) {
        const Column<float>* c = edges ? g.EdgeDense(fi->idx) : g.NodeDense(fi->idx);
        if (!apply_udf) {
          // size pass, then one memcpy per row straight into the output tensor
          std::vector<const float*> src(n, nullptr);
          int64_t total = 0;
          for (int64_t i = 0; i < n; ++i) {
            int64_t k = 0;
            if (c && rows[i] >= 0) c->Get(rows[i], &src[i], &k);
            counts[i] = k;
            total += k;
          }
          Tensor out = Tensor::Uninit(DType::kFloat, {total});
          float* dst = out.data<float>();
          for (int64_t i = 0; i < n; ++i) {
            if (counts[i]) memcpy(dst, src[i], counts[i] * sizeof(float));
            dst += counts[i];
          }
          ctx->Set(nd.Output(2 * f), MakeIdx(counts));
          ctx->Set(nd.Output(2 * f + 1), out);
          continue;
        }
        UdfColumn col;
        col.kind = UdfColumn::kDense;
        col.counts.assign(n, 0);
        for (int64_t i = 0; i < n; ++i) {
          const float* p = nullptr;
          int64_t k = 0;
          if (c && rows[i] >= 0) c->Get(rows[i], &p, &k);
          col.f.insert(col.f.end(), p, p + k);
          col.counts[i] = k;
        }
        UdfColumn res;
        UdfOf(nd)->Compute(col, nd.udf_num_params, &res);
        if (static_cast<int64_t>(res.counts.size()) != n || res.kind != UdfColumn::kDense)
          EULER_THROW("udf " << nd.udf_name << " returned a malformed column");
        ctx->Set(nd.Output(2 * f), MakeIdx(res.counts));
        ctx->Set(nd.Output(2 * f + 1), Tensor::FromVector(res.f));
      } else if (fi->type == kSparse) {
        const Column<uint64_t>* c = edges ? g.EdgeSparse(fi->idx) : g.NodeSparse(fi->idx);
        std::vector<uint64_t> vals;
        for (int64_t i = 0; i < n; ++i) {
          const uint64_t* p = nullptr;
          int64_t k = 0;
          if (c && rows[i] >= 0) c->Get(rows[i], &p, &k);
          vals.insert(vals.end(), p, p + k);
          counts[i] = k;
        }
        if (apply_udf) {
          UdfColumn col, res;
          col.kind = UdfColumn::kSparse;
          col.counts = counts;
          col.u.swap(vals);
          UdfOf(nd)->Compute(col, nd.udf_num_params, &res);
          if (static_cast<int64_t>(res.counts.size()) != n || res.kind != UdfColumn::kSparse)
            EULER_THROW("udf " << nd.udf_name << " returned a malformed column");
          counts.swap(res.counts);
          vals.swap(res.u);
        }
        ctx->Set(nd.Output(2 * f), MakeIdx(counts));
        ctx->Set(nd.Output(2 * f + 1), Tensor::FromVector(vals));
      } else {
        const Column<char>* c = edges ? g.EdgeBinary(fi->idx) : g.NodeBinary(fi->idx);
        std::vector<std::string> vals;
        for (int64_t i = 0; i < n; ++i) {
          const char* p = nullptr;
          int64_t k = 0;
          if (c && rows[i] >= 0) c->Get(rows[i], &p, &k);
          if (rows[i] >= 0) {
            vals.emplace_back(p ? p : "", k);
            counts[i] = 1;
          }
        }
        ctx->Set(nd.Output(2 * f), MakeIdx(counts));
        ctx->Set(nd.Output(2 * f + 1), Tensor::Strings(vals));
      }
    }
  }
};

// ---------------------------------------------------------------- neighbors
std::vector<int32_t> EdgeTypes(const NodeDef& nd, OpContext* ctx, size_t i = 0) {
  if (nd.attrs.size() <= i) return {};
  auto v = ctx->AttrInts(nd.attrs[i]);
  // "-1" means all edge types
  if (v.size() == 1 && v[0] < 0) return {};
  return v;
}

// filter a neighbor list by the node's DNF (neighbor index when the DNF names one,
// otherwise membership in the attribute-index result)
void FilterNeighbors(OpContext* ctx, uint64_t root, const Dnf& d, bool neighbor_idx, const IndexResult* global,
                     std::vector<IdWeightType>* v) {
  IndexResult allowed;
  const IndexResult* ref = global;
  if (neighbor_idx) {
    Status st = ctx->env()->index->QueryNeighbors(root, d, &allowed);
    if (!st.ok()) EULER_THROW(st.message());
    ref = &allowed;
  }
  std::vector<IdWeightType> keep;
  for (auto& x : *v)
    if (ref && ref->Contains(x.id)) keep.push_back(x);
  v->swap(keep);
}

class GetNeighborOp : public OpKernel {
 public:
  explicit GetNeighborOp(bool out) : out_(out) {}
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    auto ids = IdsOf(ctx->Get(nd.inputs.at(0)));
    auto et = EdgeTypes(nd, ctx);
    PostProcess pp = PostProcess::Parse(nd.post_process);
    const bool dnf = HasDnf(nd);
    Dnf d;
    bool nbr_idx = false;
    IndexResult global;
    if (dnf) {
      d = GetDnf(nd, ctx);
      nbr_idx = DnfUsesNeighborIndex(ctx, d);
      if (!nbr_idx) global = QueryIndex(ctx, d);
    }
    std::vector<std::vector<IdWeightType>> rows(ids.size());
    ThreadPool::Default()->ParallelFor(static_cast<int64_t>(ids.size()), 256, [&](int64_t b, int64_t e) {
      for (int64_t i = b; i < e; ++i) {
        g.FullNeighbor(g.Row(ids[i]), et, out_, &rows[i]);
        if (dnf) FilterNeighbors(ctx, ids[i], d, nbr_idx, &global, &rows[i]);
        pp.Apply(&rows[i]);
      }
    });
    EmitNeighbors(nd, ctx, rows);
  }

 private:
  bool out_;
};
class GetOutNeighborOp : public GetNeighborOp {
 public:
  GetOutNeighborOp() : GetNeighborOp(true) {}
};
class GetInNeighborOp : public GetNeighborOp {
 public:
  GetInNeighborOp() : GetNeighborOp(false) {}
};

class GetNeighborEdgeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    auto ids = IdsOf(ctx->Get(nd.inputs.at(0)));
    auto et = EdgeTypes(nd, ctx);
    const bool dnf = HasDnf(nd);
    IndexResult ir;
    if (dnf) ir = QueryIndex(ctx, GetDnf(nd, ctx));
    std::vector<int64_t> counts(ids.size());
    std::vector<uint64_t> edges;
    std::vector<float> w;
    std::vector<IdWeightType> tmp;
    for (size_t i = 0; i < ids.size(); ++i) {
      g.FullNeighbor(g.Row(ids[i]), et, true, &tmp);
      int64_t k = 0;
      for (auto& x : tmp) {
        if (dnf && !ir.Contains(EdgeIdHash(ids[i], x.id, x.type))) continue;
        edges.insert(edges.end(), {ids[i], x.id, static_cast<uint64_t>(x.type)});
        w.push_back(x.weight);
        ++k;
      }
      counts[i] = k;
    }
    ctx->Set(nd.Output(0), MakeIdx(counts));
    ctx->Set(nd.Output(1), Tensor::FromVector(edges, {static_cast<int64_t>(w.size()), 3}));
    ctx->Set(nd.Output(2), Tensor::FromVector(w));
  }
};

class SampleNeighborOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    auto ids = IdsOf(ctx->Get(nd.inputs.at(0)));
    auto et = EdgeTypes(nd, ctx, 0);
    const int count = nd.attrs.size() > 1 ? static_cast<int>(ctx->AttrInt(nd.attrs[1])) : 1;
    const uint64_t def = nd.attrs.size() > 2 ? static_cast<uint64_t>(ctx->AttrInt(nd.attrs[2])) : kDefaultNode;
    PostProcess pp = PostProcess::Parse(nd.post_process);
    const bool dnf = HasDnf(nd);
    Dnf d;
    bool nbr_idx = false;
    IndexResult global;
    if (dnf) {
      d = GetDnf(nd, ctx);
      nbr_idx = DnfUsesNeighborIndex(ctx, d);
      if (!nbr_idx) global = QueryIndex(ctx, d);
    }
    const int64_t n = static_cast<int64_t>(ids.size());
    if (nd.attrs.size() > 3 && !dnf) {
      // keyed: the draws of ids[i] depend on (key, id, occurrence) only
      const uint64_t key = static_cast<uint64_t>(ctx->AttrInt(nd.attrs[3]));
      std::vector<uint32_t> occ;
      KeyedOccurrences(ids.data(), n, &occ);
      Tensor oid(DType::kUInt64, {n * count}), ow(DType::kFloat, {n * count}), ot(DType::kInt32, {n * count});
      uint64_t* pid = oid.data<uint64_t>();
      float* pw = ow.data<float>();
      int32_t* pt = ot.data<int32_t>();
      ParallelChunks(n, 512, [&](int64_t b, int64_t e, Rng&) {
        SampleNeighborsKeyed(g, ids.data() + b, occ.data() + b, e - b, et, count, key, def, pid + b * count,
                             pw + b * count, pt + b * count);
      });
      if (pp.empty()) {
        ctx->Set(nd.Output(0), MakeUniformIdx(n, count));
        ctx->Set(nd.Output(1), oid);
        ctx->Set(nd.Output(2), ow);
        ctx->Set(nd.Output(3), ot);
        return;
      }
      std::vector<std::vector<IdWeightType>> rows(n);
      for (int64_t i = 0; i < n; ++i) {
        for (int k = 0; k < count; ++k) rows[i].push_back({pid[i * count + k], pw[i * count + k], pt[i * count + k]});
        pp.Apply(&rows[i]);
      }
      EmitNeighbors(nd, ctx, rows);
      return;
    }
    if (!dnf && pp.empty()) {
      // fast path: dense [n, count] outputs written in parallel
      Tensor oid(DType::kUInt64, {n * count}), ow(DType::kFloat, {n * count}), ot(DType::kInt32, {n * count});
      uint64_t* pid = oid.data<uint64_t>();
      float* pw = ow.data<float>();
      int32_t* pt = ot.data<int32_t>();
      ParallelChunks(n, 512, [&](int64_t b, int64_t e, Rng& rng) {
        std::vector<IdWeightType> tmp;
        for (int64_t i = b; i < e; ++i) {
          g.SampleNeighbor(g.Row(ids[i]), et, count, true, rng, &tmp);
          for (int k = 0; k < count; ++k) {
            const int64_t o = i * count + k;
            if (k < static_cast<int>(tmp.size())) {
              pid[o] = tmp[k].id;
              pw[o] = tmp[k].weight;
              pt[o] = tmp[k].type;
            } else {
              pid[o] = def;
              pw[o] = 0.f;
              pt[o] = -1;
            }
          }
        }
      });
      ctx->Set(nd.Output(0), MakeUniformIdx(n, count));
      ctx->Set(nd.Output(1), oid);
      ctx->Set(nd.Output(2), ow);
      ctx->Set(nd.Output(3), ot);
      return;
    }
    std::vector<std::vector<IdWeightType>> rows(n);
    ParallelChunks(n, 256, [&](int64_t b, int64_t e, Rng& rng) {
      std::vector<IdWeightType> full;
      for (int64_t i = b; i < e; ++i) {
        auto& r = rows[i];
        if (dnf) {
          g.FullNeighbor(g.Row(ids[i]), et, true, &full);
          FilterNeighbors(ctx, ids[i], d, nbr_idx, &global, &full);
          if (!full.empty()) {
            std::vector<float> cum(full.size());
            float acc = 0.f;
            for (size_t j = 0; j < full.size(); ++j) cum[j] = (acc += full[j].weight);
            for (int k = 0; k < count; ++k)
              r.push_back(full[PrefixPick(cum.data(), 0, static_cast<int64_t>(cum.size()), rng.Uniform() * acc)]);
          }
        } else {
          g.SampleNeighbor(g.Row(ids[i]), et, count, true, rng, &r);
        }
        if (r.empty())
          for (int k = 0; k < count; ++k) r.push_back({def, 0.f, -1});
        pp.Apply(&r);
      }
    });
    EmitNeighbors(nd, ctx, rows);
  }
};

class SampleNodeAtOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    if (nd.attrs.size() < 3) EULER_THROW("API_SAMPLE_NODE_AT needs [node_type, buckets, key, (default)]");
    auto codes = IdsOf(ctx->Get(nd.inputs.at(0)));
    const int type = static_cast<int>(ctx->AttrInt(nd.attrs[0]));
    const uint64_t B = static_cast<uint64_t>(ctx->AttrInt(nd.attrs[1]));
    const uint64_t key = static_cast<uint64_t>(ctx->AttrInt(nd.attrs[2]));
    const uint64_t def = nd.attrs.size() > 3 ? static_cast<uint64_t>(ctx->AttrInt(nd.attrs[3])) : kDefaultNode;
    if (B == 0) EULER_THROW("API_SAMPLE_NODE_AT: zero buckets");
    std::vector<uint64_t> out(codes.size());
    for (size_t i = 0; i < codes.size(); ++i) {
      Rng rng(key, 2 * (codes[i] / B) + 1);
      out[i] = g.SampleNodeInBucket(type, B, codes[i] % B, rng, def);
    }
    ctx->Set(nd.Output(0), Tensor::FromVector(out));
  }
};

class NodeBucketWeightOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    if (nd.attrs.size() < 2) EULER_THROW("API_NODE_BUCKET_WEIGHT needs [node_type, buckets]");
    const int type = static_cast<int>(ctx->AttrInt(nd.attrs[0]));
    const uint64_t B = static_cast<uint64_t>(ctx->AttrInt(nd.attrs[1]));
    ctx->Set(nd.Output(0), Tensor::FromVector(g.NodeBucketWeights(type, B)));
  }
};

class EdgeSumWeightOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    auto ids = IdsOf(ctx->Get(nd.inputs.at(0)));
    auto et = EdgeTypes(nd, ctx);
    std::vector<float> out(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) out[i] = g.EdgeSumWeight(g.Row(ids[i]), et, true);
    ctx->Set(nd.Output(0), Tensor::FromVector(out));
  }
};

class SampleLayerOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    auto ids = IdsOf(ctx->Get(nd.inputs.at(0)));
    auto et = EdgeTypes(nd, ctx, 0);
    const uint64_t def = nd.attrs.size() > 1 ? static_cast<uint64_t>(ctx->AttrInt(nd.attrs[1])) : kDefaultNode;
    std::vector<uint64_t> out(ids.size(), def);
    ParallelChunks(static_cast<int64_t>(ids.size()), 512, [&](int64_t b, int64_t e, Rng& rng) {
      std::vector<IdWeightType> tmp;
      for (int64_t i = b; i < e; ++i) {
        if (ids[i] == def) continue;
        g.SampleNeighbor(g.Row(ids[i]), et, 1, true, rng, &tmp);
        if (!tmp.empty()) out[i] = tmp[0].id;
      }
    });
    ctx->Set(nd.Output(0), Tensor::FromVector(out));
  }
};

// For root i (batch b = i / batch_n, or all candidates when batch_n <= 0) list the
// candidate positions that are out-neighbors of the root (reference
// sparse_get_adj_op.cc; the (root, batch) pairs of API_SPARSE_GEN_ADJ are implied).
class SparseGetAdjOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    auto roots = IdsOf(ctx->Get(nd.inputs.at(0)));
    auto cands = IdsOf(ctx->Get(nd.inputs.at(1)));
    auto et = EdgeTypes(nd, ctx, 0);
    const int64_t bn = nd.attrs.size() > 1 ? ctx->AttrInt(nd.attrs[1]) : -1;
    // original row positions (distribute mode: roots arrive split by shard)
    std::vector<int64_t> pos(roots.size());
    for (size_t i = 0; i < roots.size(); ++i) pos[i] = static_cast<int64_t>(i);
    int64_t total_roots = static_cast<int64_t>(roots.size());
    if (nd.inputs.size() > 2) {
      pos = ctx->Get(nd.inputs[2]).ToInt64();
      total_roots = 0;
      for (int64_t p : pos) total_roots = std::max(total_roots, p + 1);
    }
    const int64_t nbatches = bn > 0 ? std::max<int64_t>(1, (total_roots + bn - 1) / bn) : 1;
    // attrs[2] = candidates per batch (m); otherwise inferred from the local root count
    const int64_t per_batch_cands =
        nd.attrs.size() > 2 ? ctx->AttrInt(nd.attrs[2]) : static_cast<int64_t>(cands.size()) / nbatches;
    std::vector<std::vector<int64_t>> cols(roots.size());
    ThreadPool::Default()->ParallelFor(static_cast<int64_t>(roots.size()), 64, [&](int64_t b, int64_t e) {
      std::vector<IdWeightType> nb;
      for (int64_t i = b; i < e; ++i) {
        g.SortedFullNeighbor(g.Row(roots[i]), et, true, &nb);
        const int64_t c0 = bn > 0 ? (pos[i] / bn) * per_batch_cands : 0;
        const int64_t c1 = bn > 0 ? std::min<int64_t>(c0 + per_batch_cands, cands.size()) : cands.size();
        for (int64_t c = c0; c < c1; ++c) {
          auto it = std::lower_bound(nb.begin(), nb.end(), cands[c],
                                     [](const IdWeightType& x, uint64_t v) { return x.id < v; });
          if (it != nb.end() && it->id == cands[c]) cols[i].push_back(c);
        }
      }
    });
    std::vector<int64_t> counts, flat;
    for (auto& c : cols) {
      counts.push_back(c.size());
      flat.insert(flat.end(), c.begin(), c.end());
    }
    ctx->Set(nd.Output(0), MakeIdx(counts));
    ctx->Set(nd.Output(1), Tensor::FromVector(flat));
  }
};

class GetAdjOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    auto src = IdsOf(ctx->Get(nd.inputs.at(0)));
    auto dst = IdsOf(ctx->Get(nd.inputs.at(1)));
    auto et = EdgeTypes(nd, ctx, 0);
    std::vector<int32_t> out(src.size(), 0);
    std::vector<IdWeightType> nb;
    for (size_t i = 0; i < src.size() && i < dst.size(); ++i) {
      g.SortedFullNeighbor(g.Row(src[i]), et, true, &nb);
      auto it = std::lower_bound(nb.begin(), nb.end(), dst[i], [](const IdWeightType& x, uint64_t v) { return x.id < v; });
      out[i] = (it != nb.end() && it->id == dst[i]) ? 1 : 0;
    }
    ctx->Set(nd.Output(0), Tensor::FromVector(out));
  }
};

class GetGraphByLabelOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    auto labels = ctx->Get(nd.inputs.at(0)).ToStrings();
    std::vector<std::vector<IdWeightType>> rows(labels.size());
    const FeatureInfo* fi = g.meta().NodeFeature("binary_graph_label");
    const IndexManager* im = ctx->env()->index;
    const SampleIndex* gi = im ? im->Get("graph_label") : nullptr;
    for (size_t i = 0; i < labels.size(); ++i) {
      if (gi) {
        IndexResult r = gi->Search(CmpOp::EQ, {IndexValue::Parse(labels[i], gi->string_values())});
        for (auto& x : r.items())
          if (g.Row(x.id) >= 0) rows[i].push_back({x.id, x.weight, 0});
      } else if (fi) {
        const Column<char>* c = g.NodeBinary(fi->idx);
        for (int64_t r = 0; c && r < g.num_nodes(); ++r) {
          const char* p;
          int64_t k;
          c->Get(r, &p, &k);
          if (static_cast<size_t>(k) == labels[i].size() && std::equal(p, p + k, labels[i].begin()))
            rows[i].push_back({g.Id(r), g.NodeWeight(r), g.NodeType(r)});
        }
      }
    }
    std::vector<int64_t> counts;
    std::vector<uint64_t> flat;
    for (auto& r : rows) {
      counts.push_back(r.size());
      for (auto& x : r) flat.push_back(x.id);
    }
    ctx->Set(nd.Output(0), MakeIdx(counts));
    ctx->Set(nd.Output(1), Tensor::FromVector(flat));
  }
};

}  // namespace

// ---------------------------------------------------------------- whole-shard export
// Every node of this shard with its out-adjacency and dense features, for assembling the
// whole graph in HBM from a sharded / remote cluster (DeviceGraph.from_engine over
// QueryProxy::RunOnShard).  attrs: dense node feature names followed by as many widths.
// Outputs: 0 node ids u64 [n], 1 types i32 [n], 2 weights f32 [n], 3 indptr i64 [n*T + 1]
// over (row, edge type) segments, 4 neighbour ids u64 [E], 5 edge weights f32 [E],
// 6.. one f32 [n][width] table per feature (missing rows / short rows zero-filled).
class ExportShardOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Graph& g = G(ctx);
    const int64_t n = g.num_nodes(), T = g.num_edge_types();
    if (nd.attrs.size() % 2 != 0) EULER_THROW("API_EXPORT_SHARD: attrs = feature names then widths");
    const Adjacency& A = g.adj(true);
    std::vector<int32_t> types(n);
    std::vector<float> nw(n);
    for (int64_t r = 0; r < n; ++r) {
      types[r] = g.NodeType(r);
      nw[r] = g.NodeWeight(r);
    }
    std::vector<int64_t> indptr(A.indptr.begin(), A.indptr.end());
    std::vector<float> w(A.nbr.size());
    ThreadPool::Default()->ParallelFor(n * T, 4096, [&](int64_t b, int64_t e) {
      for (int64_t s = b; s < e; ++s)
        for (uint64_t k = A.indptr[s]; k < A.indptr[s + 1]; ++k) w[k] = A.EdgeWeight(k, A.indptr[s]);
    });
    ctx->Set(nd.Output(0), Tensor::FromVector(g.node_ids()));
    ctx->Set(nd.Output(1), Tensor::FromVector(types));
    ctx->Set(nd.Output(2), Tensor::FromVector(nw));
    ctx->Set(nd.Output(3), Tensor::FromVector(indptr));
    ctx->Set(nd.Output(4), Tensor::FromVector(A.nbr));
    ctx->Set(nd.Output(5), Tensor::FromVector(w));
    const size_t nf = nd.attrs.size() / 2;
    for (size_t f = 0; f < nf; ++f) {
      const int64_t dim = std::stoll(nd.attrs[nf + f]);
      const FeatureInfo* fi = g.meta().NodeFeature(nd.attrs[f]);
      if (!fi || fi->type != kDense) EULER_THROW("no dense node feature named " + nd.attrs[f]);
      const Column<float>* c = g.NodeDense(fi->idx);
      std::vector<float> out(static_cast<size_t>(n * dim), 0.f);
      ThreadPool::Default()->ParallelFor(n, 1024, [&](int64_t b, int64_t e) {
        for (int64_t r = b; r < e; ++r) {
          const float* p = nullptr;
          int64_t k = 0;
          if (c) c->Get(r, &p, &k);
          if (k > dim) k = dim;
          if (k > 0) memcpy(out.data() + r * dim, p, k * 4);
        }
      });
      ctx->Set(nd.Output(6 + static_cast<int>(f)), Tensor::FromVector(out, {n, dim}));
    }
  }
};

REGISTER_OP_KERNEL("API_EXPORT_SHARD", ExportShardOp);
REGISTER_OP_KERNEL("API_GET_NODE", GetNodeOp);
REGISTER_OP_KERNEL("API_GET_EDGE", GetEdgeOp);
REGISTER_OP_KERNEL("API_SAMPLE_NODE", SampleNodeOp);
REGISTER_OP_KERNEL("API_SAMPLE_N_WITH_TYPES", SampleNWithTypesOp);
REGISTER_OP_KERNEL("API_SAMPLE_EDGE", SampleEdgeOp);
REGISTER_OP_KERNEL("API_GET_NODE_T", GetNodeTypeOp);
REGISTER_OP_KERNEL("API_GET_P", GetFeatureOp);
REGISTER_OP_KERNEL("API_GET_NB_NODE", GetOutNeighborOp);
REGISTER_OP_KERNEL("API_GET_RNB_NODE", GetInNeighborOp);
REGISTER_OP_KERNEL("API_GET_NB_EDGE", GetNeighborEdgeOp);
REGISTER_OP_KERNEL("API_SAMPLE_NB", SampleNeighborOp);
REGISTER_OP_KERNEL("API_SAMPLE_NODE_AT", SampleNodeAtOp);
REGISTER_OP_KERNEL("API_NODE_BUCKET_WEIGHT", NodeBucketWeightOp);
REGISTER_OP_KERNEL("API_GET_EDGE_SUM_WEIGHT", EdgeSumWeightOp);
REGISTER_OP_KERNEL("API_SAMPLE_L", SampleLayerOp);
REGISTER_OP_KERNEL("API_SPARSE_GET_ADJ", SparseGetAdjOp);
REGISTER_OP_KERNEL("API_GET_ADJ", GetAdjOp);
REGISTER_OP_KERNEL("API_GET_GRAPH_BY_LABEL", GetGraphByLabelOp);

void LinkGraphOps() {}

}  // namespace euler
