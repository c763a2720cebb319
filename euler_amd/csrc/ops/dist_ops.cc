// Client-side distribution kernels: split -> REMOTE x shards -> merge, unique/gather,
// aliasing, post-processing and the layer-wise sampling helpers that stay local.
// Reference catalog: SURVEY §2.5 "Distribution kernels" and "Misc kernels".
//
//   ID_SPLIT                   in [ids|edges]               -> 2s ids_s, 2s+1 merge_idx_s
//   BROAD_CAST_SPLIT           in [x]                       -> s: x
//   SAMPLE_NODE_SPLIT          attrs [type, count]          -> s: count_s      (by node weight sums)
//   SAMPLE_EDGE_SPLIT          attrs [type, count]          -> s: count_s      (by edge weight sums)
//   SAMPLE_N_WITH_TYPES_SPLIT  attrs [types, counts]        -> s: counts_s
//   APPEND_MERGE               in [d_0..d_S-1]              -> concat rows
//   IDX_MERGE                  in [idx_s, merge_s]*         -> idx in original order
//   DATA_MERGE                 in [d_s, idx_s, merge_s]*    -> data in original order
//   REGULAR_DATA_MERGE         in [d_s, merge_s]*           -> fixed-width rows in original order
//   MULTI_TYPE_IDX_MERGE / IDX_ROW_APPEND_MERGE   in [idx_s]*        -> per-row counts summed
//   MULTI_TYPE_DATA_MERGE / DATA_ROW_APPEND_MERGE in [d_s, idx_s]*   -> per-row concat over shards
//   ID_UNIQUE                  in [ids]                     -> 0 unique, 1 gather_idx
//   IDX_GATHER                 in [idx_u, gather]           -> idx of the original rows
//   DATA_GATHER                in [d_u, idx_u, gather]      -> data of the original rows
//   AS                         in [x_i...] attrs [alias]    -> "alias:i"
//   POST_PROCESS               in [idx, ids, w, t] | [ids]  -> same, order_by / limit per row
//   API_GET_NB_FILTER          in [idx, ids, w, t, allowed] -> neighbors in allowed, then pp
//   API_SAMPLE_ROOT            in [roots, weights] attrs [n, m, default] -> m roots per batch of n
//   API_LOCAL_SAMPLE_L         in [idx, ids, w, t] attrs [n, m, weight_func, default]
//   API_SAMPLE_GRAPH_LABEL     attrs [count]                -> labels (strings)
//   GP_*_MERGE                 graph-partition names of the merges; GP_UNIQUE_MERGE row unique
//   API_SPARSE_GEN_ADJ         in [roots, l_nb, n]          -> (root, batch) rows, l_nb
//   API_GATHER_RESULT          in [x_i...]                  -> aliases
//   API_RESHAPE                in [x] attrs ["d0,?,..."]    -> x with that shape
#include <cmath>
#include <unordered_map>
#include <unordered_set>

#include <stdexcept>
#include "ops/ops_util.h"

namespace euler {
namespace {

int Shards(OpContext* ctx) { return std::max(1, ctx->env() ? ctx->env()->shard_num : 1); }

// rows of a tensor: shape[0] when rank >= 1
int64_t Rows(const Tensor& t) { return t.shape().empty() ? t.numel() : t.dim(0); }
int64_t RowWidth(const Tensor& t) {
  const int64_t r = Rows(t);
  return r > 0 ? t.numel() / r : (t.shape().size() > 1 ? t.dim(1) : 1);
}

// gather rows of t (any dtype) into a new tensor; runs of consecutive rows are one memcpy
Tensor TakeRows(const Tensor& t, const std::vector<int64_t>& rows, int64_t width) {
  std::vector<int64_t> shape = t.shape();
  if (shape.empty()) shape = {static_cast<int64_t>(rows.size())};
  shape[0] = static_cast<int64_t>(rows.size());
  Tensor out(t.dtype(), shape);
  if (t.dtype() == DType::kString) {
    for (size_t i = 0; i < rows.size(); ++i)
      for (int64_t k = 0; k < width; ++k) out.strings()[i * width + k] = t.strings()[rows[i] * width + k];
  } else {
    const size_t es = DTypeSize(t.dtype()) * width;
    const char* src = static_cast<const char*>(t.raw());
    char* dst = static_cast<char*>(out.raw());
    for (size_t i = 0; i < rows.size();) {
      size_t j = i + 1;
      while (j < rows.size() && rows[j] == rows[j - 1] + 1) ++j;
      memcpy(dst + i * es, src + rows[i] * es, (j - i) * es);
      i = j;
    }
  }
  return out;
}

// g == 0, 1, ..., rows-1 (a gather that keeps every row in place)
bool IsIdentity(const Tensor& g, int64_t rows) {
  if (g.numel() != rows) return false;
  for (int64_t i = 0; i < rows; ++i)
    if (g.AsInt(i) != i) return false;
  return true;
}

// open-addressing id -> first position map (linear probing, power-of-two capacity)
class IdPosMap {
 public:
  explicit IdPosMap(size_t n) {
    size_t cap = 16;
    while (cap < 2 * n) cap <<= 1;
    mask_ = cap - 1;
    keys_.resize(cap);
    pos_.assign(cap, -1);
  }
  // position of `id`, inserting `next` when absent (returns next then)
  int32_t FindOrInsert(uint64_t id, int32_t next) {
    size_t h = static_cast<size_t>((id * 0x9E3779B97F4A7C15ull) >> 17) & mask_;
    for (;;) {
      if (pos_[h] < 0) {
        keys_[h] = id;
        pos_[h] = next;
        return next;
      }
      if (keys_[h] == id) return pos_[h];
      h = (h + 1) & mask_;
    }
  }

 private:
  size_t mask_;
  std::vector<uint64_t> keys_;
  std::vector<int32_t> pos_;
};

Tensor Concat(const std::vector<const Tensor*>& parts, DType fallback, int64_t width_hint) {
  int64_t rows = 0, width = width_hint > 0 ? width_hint : 1;
  DType dt = fallback;
  std::vector<int64_t> shape_tail;
  for (auto* p : parts) {
    rows += Rows(*p);
    if (p->numel() > 0) {
      dt = p->dtype();
      width = RowWidth(*p);
      shape_tail.assign(p->shape().begin() + (p->shape().empty() ? 0 : 1), p->shape().end());
    }
  }
  std::vector<int64_t> shape{rows};
  if (width > 1) {
    if (shape_tail.empty()) shape_tail = {width};
    shape.insert(shape.end(), shape_tail.begin(), shape_tail.end());
  }
  Tensor out(dt, shape);
  int64_t off = 0;
  for (auto* p : parts) {
    const int64_t n = p->numel();
    if (n == 0) continue;
    if (dt == DType::kString) {
      for (int64_t i = 0; i < n; ++i) out.strings()[off + i] = p->strings()[i];
    } else {
      memcpy(static_cast<char*>(out.raw()) + off * DTypeSize(dt), p->raw(), n * DTypeSize(dt));
    }
    off += n;
  }
  return out;
}

// ---------------------------------------------------------------- splits
class IdSplitOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const Tensor& in = ctx->Get(nd.inputs.at(0));
    const int S = Shards(ctx);
    const uint32_t P = ctx->env()->num_partitions;
    const bool edges = in.shape().size() == 2 && in.dim(1) == 3;
    const int64_t n = edges ? in.dim(0) : in.numel();
    const int64_t width = edges ? 3 : 1;
    if (S == 1) {  // one shard: the ids as they are, identity merge index
      Tensor part = in;
      if (!edges) part.Reshape({n});
      ctx->Set(nd.Output(0), part);
      std::vector<int32_t> mi(n);
      for (int64_t i = 0; i < n; ++i) mi[i] = static_cast<int32_t>(i);
      ctx->Set(nd.Output(1), Tensor::FromVector(mi));
      return;
    }
    std::vector<std::vector<int64_t>> rows(S);
    for (int64_t i = 0; i < n; ++i) {
      // edges are split by their source (reference id_split_op.cc:46-49)
      const uint64_t id = static_cast<uint64_t>(in.AsInt(i * width));
      rows[ShardOf(id, P, S)].push_back(i);
    }
    for (int s = 0; s < S; ++s) {
      Tensor part = TakeRows(in, rows[s], width);
      if (!edges) part.Reshape({static_cast<int64_t>(rows[s].size())});
      ctx->Set(nd.Output(2 * s), part);
      std::vector<int32_t> mi(rows[s].begin(), rows[s].end());
      ctx->Set(nd.Output(2 * s + 1), Tensor::FromVector(mi));
    }
  }
};

// graph_partition mode: the node ids of an id-routed input (edges [n, 3]: their sources)
class IdSrcOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const Tensor& in = ctx->Get(nd.inputs.at(0));
    const bool edges = in.shape().size() == 2 && in.dim(1) == 3;
    const int64_t n = edges ? in.dim(0) : in.numel();
    std::vector<int64_t> ids(n);
    for (int64_t i = 0; i < n; ++i) ids[i] = in.AsInt(edges ? i * 3 : i);
    ctx->Set(nd.Output(0), Tensor::FromVector(ids));
  }
};

// graph_partition mode: inputs (x, types_0 .. types_{S-1}) with types_s[i] = the type shard
// s reports for row i's node (-1: not held there); row i goes to the first holder, a row
// no shard holds to its hash shard (it reads as missing there, as under hash routing).
// Outputs as ID_SPLIT: 2s = the rows of shard s, 2s + 1 = their positions.
class GpIdSplitOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const Tensor& in = ctx->Get(nd.inputs.at(0));
    const int S = static_cast<int>(nd.inputs.size()) - 1;
    const uint32_t P = ctx->env()->num_partitions;
    const bool edges = in.shape().size() == 2 && in.dim(1) == 3;
    const int64_t n = edges ? in.dim(0) : in.numel();
    const int64_t width = edges ? 3 : 1;
    std::vector<const Tensor*> types(S);
    for (int s = 0; s < S; ++s) {
      types[s] = &ctx->Get(nd.inputs.at(1 + s));
      if (types[s]->numel() != n)
        throw std::runtime_error("GP_ID_SPLIT: shard " + std::to_string(s) + " answered " +
                                 std::to_string(types[s]->numel()) + " types for " + std::to_string(n) + " rows");
    }
    std::vector<std::vector<int64_t>> rows(S);
    for (int64_t i = 0; i < n; ++i) {
      int owner = -1;
      for (int s = 0; s < S && owner < 0; ++s)
        if (types[s]->AsInt(i) >= 0) owner = s;
      if (owner < 0) owner = ShardOf(static_cast<uint64_t>(in.AsInt(i * width)), P, S);
      rows[owner].push_back(i);
    }
    for (int s = 0; s < S; ++s) {
      Tensor part = TakeRows(in, rows[s], width);
      if (!edges) part.Reshape({static_cast<int64_t>(rows[s].size())});
      ctx->Set(nd.Output(2 * s), part);
      std::vector<int32_t> mi(rows[s].begin(), rows[s].end());
      ctx->Set(nd.Output(2 * s + 1), Tensor::FromVector(mi));
    }
  }
};

class BroadcastSplitOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const Tensor& in = ctx->Get(nd.inputs.at(0));
    for (int s = 0; s < Shards(ctx); ++s) ctx->Set(nd.Output(s), in);
  }
};

// split `count` over shards proportionally to their weight sums, remainder at random
// (reference sample_node_split_op.cc:54-85)
std::vector<int64_t> SplitCount(int64_t count, const std::vector<double>& w, Rng& rng) {
  const int S = static_cast<int>(w.size());
  std::vector<int64_t> out(S, 0);
  double total = 0;
  for (double x : w) total += x;
  if (total <= 0 || count <= 0) return out;
  int64_t given = 0;
  for (int s = 0; s < S; ++s) given += (out[s] = static_cast<int64_t>(std::floor(count * w[s] / total)));
  std::vector<float> wf(w.begin(), w.end());
  AliasTable at(wf);
  for (int64_t r = given; r < count; ++r) out[at.Sample(rng)]++;
  return out;
}

std::vector<double> ShardWeights(const std::vector<std::vector<double>>& table, int type, int S) {
  std::vector<double> w(S, 1.0);
  if (table.empty()) return w;
  const int row = (type < 0 || type + 1 >= static_cast<int>(table.size())) ? static_cast<int>(table.size()) - 1 : type;
  for (int s = 0; s < S && s < static_cast<int>(table[row].size()); ++s) w[s] = table[row][s];
  return w;
}

class SampleSplitOp : public OpKernel {
 public:
  explicit SampleSplitOp(bool node) : node_(node) {}
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const int S = Shards(ctx);
    const int type = static_cast<int>(ctx->AttrInt(nd.attrs.at(0)));
    const int64_t count = ctx->AttrInt(nd.attrs.at(1));
    Rng rng(GlobalSeed() ^ 0x5A17ULL, NextEpoch());
    auto w = ShardWeights(node_ ? ctx->env()->node_weight_sums : ctx->env()->edge_weight_sums, type, S);
    auto c = SplitCount(count, w, rng);
    for (int s = 0; s < S; ++s) ctx->Set(nd.Output(s), Tensor::Scalar<int64_t>(c[s]));
  }

 private:
  bool node_;
};
class SampleNodeSplitOp : public SampleSplitOp {
 public:
  SampleNodeSplitOp() : SampleSplitOp(true) {}
};
class SampleEdgeSplitOp : public SampleSplitOp {
 public:
  SampleEdgeSplitOp() : SampleSplitOp(false) {}
};

class SampleNWithTypesSplitOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const int S = Shards(ctx);
    auto types = ctx->AttrInts(nd.attrs.at(0));
    auto counts = ctx->AttrInts(nd.attrs.at(1));
    if (counts.size() == 1 && types.size() > 1) counts.assign(types.size(), counts[0]);
    Rng rng(GlobalSeed() ^ 0x5A18ULL, NextEpoch());
    std::vector<std::vector<int32_t>> per(S, std::vector<int32_t>(types.size(), 0));
    for (size_t t = 0; t < types.size(); ++t) {
      auto c = SplitCount(t < counts.size() ? counts[t] : 0, ShardWeights(ctx->env()->node_weight_sums, types[t], S), rng);
      for (int s = 0; s < S; ++s) per[s][t] = static_cast<int32_t>(c[s]);
    }
    for (int s = 0; s < S; ++s) ctx->Set(nd.Output(s), Tensor::FromVector(per[s]));
  }
};

// ---------------------------------------------------------------- merges
class AppendMergeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    std::vector<const Tensor*> parts;
    std::vector<Tensor> hold;
    hold.reserve(nd.inputs.size());
    for (auto& in : nd.inputs) hold.push_back(ctx->Get(in));
    for (auto& t : hold) parts.push_back(&t);
    ctx->Set(nd.Output(0), Concat(parts, DType::kUInt64, 0));
  }
};

class IdxMergeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const size_t S = nd.inputs.size() / 2;
    int64_t n = 0;
    std::vector<Tensor> idx(S), mi(S);
    for (size_t s = 0; s < S; ++s) {
      idx[s] = ctx->Get(nd.inputs[2 * s]);
      mi[s] = ctx->Get(nd.inputs[2 * s + 1]);
      n += mi[s].numel();
    }
    std::vector<int64_t> counts(n, 0);
    for (size_t s = 0; s < S; ++s) {
      const int32_t* p = idx[s].data<int32_t>();
      for (int64_t i = 0; i < mi[s].numel(); ++i) counts[mi[s].AsInt(i)] = p[2 * i + 1] - p[2 * i];
    }
    ctx->Set(nd.Output(0), MakeIdx(counts));
  }
};

class DataMergeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const size_t S = nd.inputs.size() / 3;
    std::vector<Tensor> d(S), idx(S), mi(S);
    int64_t n = 0, total_rows = 0, width = 1;
    DType dt = DType::kUInt64;
    std::vector<int64_t> tail;
    for (size_t s = 0; s < S; ++s) {
      d[s] = ctx->Get(nd.inputs[3 * s]);
      idx[s] = ctx->Get(nd.inputs[3 * s + 1]);
      mi[s] = ctx->Get(nd.inputs[3 * s + 2]);
      n += mi[s].numel();
      if (d[s].numel() > 0 || s == 0) {
        dt = d[s].dtype();
        width = RowWidth(d[s]);
        tail.assign(d[s].shape().begin() + (d[s].shape().empty() ? 0 : 1), d[s].shape().end());
      }
      total_rows += Rows(d[s]);
    }
    if (S == 1) {  // single shard in original order: the data is already merged
      bool identity = true;
      for (int64_t i = 0; i < mi[0].numel() && identity; ++i) identity = mi[0].AsInt(i) == i;
      if (identity) {
        ctx->Set(nd.Output(0), d[0]);
        return;
      }
    }
    // destination offsets in original order
    std::vector<int64_t> counts(n, 0);
    std::vector<std::pair<int, int64_t>> where(n);  // (shard, local row)
    for (size_t s = 0; s < S; ++s) {
      const int32_t* p = idx[s].data<int32_t>();
      for (int64_t i = 0; i < mi[s].numel(); ++i) {
        const int64_t o = mi[s].AsInt(i);
        counts[o] = p[2 * i + 1] - p[2 * i];
        where[o] = {static_cast<int>(s), i};
      }
    }
    std::vector<int64_t> shape{total_rows};
    shape.insert(shape.end(), tail.begin(), tail.end());
    Tensor out(dt, shape);
    int64_t off = 0;
    for (int64_t o = 0; o < n; ++o) {
      const int s = where[o].first;
      const int64_t i = where[o].second;
      const int32_t b = idx[s].data<int32_t>()[2 * i];
      const int64_t k = counts[o];
      if (k == 0) continue;
      if (dt == DType::kString) {
        for (int64_t j = 0; j < k * width; ++j) out.strings()[off * width + j] = d[s].strings()[b * width + j];
      } else {
        const size_t es = DTypeSize(dt) * width;
        memcpy(static_cast<char*>(out.raw()) + off * es, static_cast<const char*>(d[s].raw()) + b * es, k * es);
      }
      off += k;
    }
    ctx->Set(nd.Output(0), out);
  }
};

class RegularDataMergeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const size_t S = nd.inputs.size() / 2;
    std::vector<Tensor> d(S), mi(S);
    int64_t n = 0, width = 1;
    DType dt = DType::kFloat;
    std::vector<int64_t> tail;
    for (size_t s = 0; s < S; ++s) {
      d[s] = ctx->Get(nd.inputs[2 * s]);
      mi[s] = ctx->Get(nd.inputs[2 * s + 1]);
      n += mi[s].numel();
      if (mi[s].numel() > 0 || s == 0) {
        dt = d[s].dtype();
        width = mi[s].numel() > 0 ? d[s].numel() / mi[s].numel() : 1;
        tail.assign(d[s].shape().begin() + (d[s].shape().empty() ? 0 : 1), d[s].shape().end());
      }
    }
    std::vector<int64_t> shape{n};
    shape.insert(shape.end(), tail.begin(), tail.end());
    Tensor out(dt, shape);
    for (size_t s = 0; s < S; ++s) {
      for (int64_t i = 0; i < mi[s].numel(); ++i) {
        const int64_t o = mi[s].AsInt(i);
        if (dt == DType::kString) {
          for (int64_t j = 0; j < width; ++j) out.strings()[o * width + j] = d[s].strings()[i * width + j];
        } else {
          const size_t es = DTypeSize(dt) * width;
          memcpy(static_cast<char*>(out.raw()) + o * es, static_cast<const char*>(d[s].raw()) + i * es, es);
        }
      }
    }
    ctx->Set(nd.Output(0), out);
  }
};

class RowAppendIdxMergeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    std::vector<int64_t> counts;
    for (auto& in : nd.inputs) {
      const Tensor& t = ctx->Get(in);
      const int64_t rows = Rows(t);
      if (counts.size() < static_cast<size_t>(rows)) counts.resize(rows, 0);
      const int32_t* p = t.data<int32_t>();
      for (int64_t r = 0; r < rows; ++r) counts[r] += p[2 * r + 1] - p[2 * r];
    }
    ctx->Set(nd.Output(0), MakeIdx(counts));
  }
};

class RowAppendDataMergeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const size_t S = nd.inputs.size() / 2;
    std::vector<Tensor> d(S), idx(S);
    int64_t rows = 0;
    for (size_t s = 0; s < S; ++s) {
      d[s] = ctx->Get(nd.inputs[2 * s]);
      idx[s] = ctx->Get(nd.inputs[2 * s + 1]);
      rows = std::max(rows, Rows(idx[s]));
    }
    std::vector<Tensor> pieces;
    for (int64_t r = 0; r < rows; ++r)
      for (size_t s = 0; s < S; ++s) {
        if (r >= Rows(idx[s])) continue;
        const int32_t* p = idx[s].data<int32_t>();
        std::vector<int64_t> take;
        const int64_t w = RowWidth(d[s]);
        for (int32_t k = p[2 * r]; k < p[2 * r + 1]; ++k) take.push_back(k);
        pieces.push_back(TakeRows(d[s], take, w));
      }
    std::vector<const Tensor*> ptrs;
    for (auto& p : pieces) ptrs.push_back(&p);
    ctx->Set(nd.Output(0), Concat(ptrs, S ? d[0].dtype() : DType::kUInt64, 0));
  }
};

// ---------------------------------------------------------------- unique / gather
class IdUniqueOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const Tensor& in = ctx->Get(nd.inputs.at(0));
    const bool edges = in.shape().size() == 2 && in.dim(1) == 3;
    if (edges) {
      // edges are not de-duplicated (pass through with identity gather)
      ctx->Set(nd.Output(0), in);
      std::vector<int32_t> g(in.dim(0));
      for (size_t i = 0; i < g.size(); ++i) g[i] = static_cast<int32_t>(i);
      ctx->Set(nd.Output(1), Tensor::FromVector(g));
      return;
    }
    auto ids = in.ToUInt64();
    IdPosMap pos(ids.size());
    std::vector<uint64_t> uniq;
    uniq.reserve(ids.size());
    std::vector<int32_t> gidx(ids.size());
    for (size_t i = 0; i < ids.size(); ++i) {
      const int32_t next = static_cast<int32_t>(uniq.size());
      gidx[i] = pos.FindOrInsert(ids[i], next);
      if (gidx[i] == next) uniq.push_back(ids[i]);
    }
    ctx->Set(nd.Output(0), Tensor::FromVector(uniq));
    ctx->Set(nd.Output(1), Tensor::FromVector(gidx));
  }
};

class IdxGatherOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const Tensor& idx = ctx->Get(nd.inputs.at(0));
    if (IsIdentity(ctx->Get(nd.inputs.at(1)), Rows(idx))) {  // ids were already distinct
      ctx->Set(nd.Output(0), idx);
      return;
    }
    auto g = ctx->Get(nd.inputs.at(1)).ToInt64();
    const int32_t* p = idx.data<int32_t>();
    std::vector<int64_t> counts(g.size());
    for (size_t i = 0; i < g.size(); ++i) counts[i] = p[2 * g[i] + 1] - p[2 * g[i]];
    ctx->Set(nd.Output(0), MakeIdx(counts));
  }
};

class DataGatherOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const Tensor& d = ctx->Get(nd.inputs.at(0));
    const Tensor& idx = ctx->Get(nd.inputs.at(1));
    if (IsIdentity(ctx->Get(nd.inputs.at(2)), Rows(idx))) {
      ctx->Set(nd.Output(0), d);
      return;
    }
    auto g = ctx->Get(nd.inputs.at(2)).ToInt64();
    const int32_t* p = idx.data<int32_t>();
    const int64_t w = RowWidth(d);
    int64_t total = 0;
    for (int64_t u : g) total += p[2 * u + 1] - p[2 * u];
    std::vector<int64_t> shape = d.shape();
    if (shape.empty()) shape = {0};
    shape[0] = total;
    Tensor out = Tensor::Uninit(d.dtype(), shape);
    int64_t off = 0;
    if (d.dtype() == DType::kString) {
      for (int64_t u : g)
        for (int64_t k = p[2 * u] * w; k < p[2 * u + 1] * w; ++k) out.strings()[off++] = d.strings()[k];
    } else {
      // one memcpy per gathered ragged row
      const size_t es = DTypeSize(d.dtype()) * w;
      const char* src = static_cast<const char*>(d.raw());
      char* dst = static_cast<char*>(out.raw());
      for (int64_t u : g) {
        const int64_t k = p[2 * u + 1] - p[2 * u];
        if (k) memcpy(dst + off * es, src + p[2 * u] * es, k * es);
        off += k;
      }
    }
    ctx->Set(nd.Output(0), out);
  }
};

// ---------------------------------------------------------------- alias / post-process
class AsOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const std::string alias = nd.attrs.empty() ? nd.name() : nd.attrs[0];
    for (size_t i = 0; i < nd.inputs.size(); ++i) ctx->Set(alias + ":" + std::to_string(i), ctx->Get(nd.inputs[i]));
  }
};

// GP_UNIQUE_MERGE: in [d_0, m_0, d_1, m_1, ...] (uint64 rows of equal width; the m_s are
// ignored) -> 0 the distinct rows over all shards in first-seen order, s+1 for each shard
// the int32 position of each of its rows in output 0.  Graph-partition mode: the same
// node can come back from several shards.  Rows are keyed by their full uint64 content
// (the reference keys by concatenated decimal text, so rows {1, 23} and {12, 3} collide).
struct RowKey {
  std::vector<uint64_t> v;
  bool operator==(const RowKey& o) const { return v == o.v; }
};
struct RowKeyHash {
  size_t operator()(const RowKey& k) const {
    uint64_t h = 0x9e3779b97f4a7c15ull;
    for (uint64_t x : k.v) h = (h ^ x) * 0xbf58476d1ce4e5b9ull + (h >> 31);
    return static_cast<size_t>(h);
  }
};

class GpUniqueMergeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    std::vector<Tensor> parts;
    for (size_t i = 0; i < nd.inputs.size(); i += 2) parts.push_back(ctx->Get(nd.inputs[i]));
    if (parts.empty()) EULER_THROW("GP_UNIQUE_MERGE needs at least one shard input");
    const int64_t width = RowWidth(parts[0]);
    std::unordered_map<RowKey, int32_t, RowKeyHash> pos;
    std::vector<uint64_t> uniq;
    std::vector<std::vector<int32_t>> where(parts.size());
    for (size_t s = 0; s < parts.size(); ++s) {
      if (RowWidth(parts[s]) != width && Rows(parts[s]) > 0) EULER_THROW("GP_UNIQUE_MERGE: row widths differ");
      const auto vals = parts[s].ToUInt64();
      const int64_t n = Rows(parts[s]);
      where[s].resize(n);
      for (int64_t r = 0; r < n; ++r) {
        RowKey k{std::vector<uint64_t>(vals.begin() + r * width, vals.begin() + (r + 1) * width)};
        auto it = pos.find(k);
        if (it == pos.end()) {
          it = pos.emplace(k, static_cast<int32_t>(uniq.size() / std::max<int64_t>(width, 1))).first;
          uniq.insert(uniq.end(), k.v.begin(), k.v.end());
        }
        where[s][r] = it->second;
      }
    }
    std::vector<int64_t> shape = parts[0].shape();
    if (shape.empty()) shape = {0};
    shape[0] = static_cast<int64_t>(pos.size());
    ctx->Set(nd.Output(0), Tensor::FromVector(uniq, shape));
    for (size_t s = 0; s < parts.size(); ++s) ctx->Set(nd.Output(static_cast<int>(s) + 1), Tensor::FromVector(where[s]));
  }
};

// API_SPARSE_GEN_ADJ: in [roots (b*n ids), l_nb, n] -> 0 (root id, batch number) uint64
// rows [b*n, 2], 1 l_nb passed through (the two inputs of API_SPARSE_GET_ADJ's split)
class SparseGenAdjOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const Tensor& roots = ctx->Get(nd.inputs.at(0));
    const int64_t n = nd.inputs.size() > 2 ? ctx->AttrInt(nd.inputs[2]) : ctx->AttrInt(nd.attrs.at(0));
    if (n <= 0) EULER_THROW("API_SPARSE_GEN_ADJ: n must be positive");
    const auto ids = roots.ToUInt64();
    const int64_t total = static_cast<int64_t>(ids.size());
    if (total % n != 0) EULER_THROW("API_SPARSE_GEN_ADJ: " << total << " roots are not batches of " << n);
    std::vector<uint64_t> rb(2 * total);
    for (int64_t c = 0; c < total; ++c) {
      rb[2 * c] = ids[c];
      rb[2 * c + 1] = static_cast<uint64_t>(c / n);
    }
    ctx->Set(nd.Output(0), Tensor::FromVector(rb, {total, 2}));
    ctx->Set(nd.Output(1), ctx->Get(nd.inputs.at(1)));
  }
};

// API_GATHER_RESULT: outputs i alias inputs i (collects a sub-DAG's results under one node)
class GatherResultOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    for (size_t i = 0; i < nd.inputs.size(); ++i) ctx->Set(nd.Output(static_cast<int>(i)), ctx->Get(nd.inputs[i]));
  }
};

// API_RESHAPE: in [x] attrs ["d0,d1,..."] (one "?" inferred) -> x viewed with that shape
class ReshapeOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    Tensor x = ctx->Get(nd.inputs.at(0));
    const std::string spec = nd.inputs.size() > 1 ? ctx->AttrStr(nd.inputs[1]) : nd.attrs.at(0);
    std::vector<int64_t> shape;
    int unknown = -1;
    int64_t known = 1;
    for (auto& tok : Split(spec, ",")) {
      const std::string t = Trim(tok);
      if (t == "?" || t == "-1") {
        if (unknown >= 0) EULER_THROW("API_RESHAPE: more than one unknown dimension in '" << spec << "'");
        unknown = static_cast<int>(shape.size());
        shape.push_back(0);
      } else {
        int64_t d;
        if (!ParseInt64(t, &d) || d < 0) EULER_THROW("API_RESHAPE: bad dimension '" << t << "'");
        shape.push_back(d);
        known *= d;
      }
    }
    if (unknown >= 0) {
      if (known == 0 || x.numel() % known != 0) EULER_THROW("API_RESHAPE: " << x.numel() << " elements vs '" << spec << "'");
      shape[unknown] = x.numel() / known;
    } else if (known != x.numel()) {
      EULER_THROW("API_RESHAPE: " << x.numel() << " elements vs '" << spec << "'");
    }
    x.Reshape(shape);  // shares the (immutable) storage
    ctx->Set(nd.Output(0), x);
  }
};

void ReadNeighbors(OpContext* ctx, const NodeDef& nd, std::vector<std::vector<IdWeightType>>* rows) {
  const Tensor& idx = ctx->Get(nd.inputs.at(0));
  const Tensor& ids = ctx->Get(nd.inputs.at(1));
  Tensor w, t;
  const bool hw = nd.inputs.size() > 2 && ctx->TryGet(nd.inputs[2], &w);
  const bool ht = nd.inputs.size() > 3 && ctx->TryGet(nd.inputs[3], &t);
  const int64_t n = Rows(idx);
  rows->assign(n, {});
  const int32_t* p = idx.data<int32_t>();
  for (int64_t r = 0; r < n; ++r)
    for (int32_t k = p[2 * r]; k < p[2 * r + 1]; ++k)
      (*rows)[r].push_back({static_cast<uint64_t>(ids.AsInt(k)), hw ? static_cast<float>(w.AsDouble(k)) : 0.f,
                            ht ? static_cast<int32_t>(t.AsInt(k)) : 0});
}

class PostProcessOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    PostProcess pp = PostProcess::Parse(nd.post_process);
    if (nd.inputs.size() == 1) {  // plain id list
      auto ids = ctx->Get(nd.inputs[0]).ToUInt64();
      std::vector<IdWeightType> v;
      for (auto id : ids) v.push_back({id, 0.f, 0});
      pp.Apply(&v);
      std::vector<uint64_t> out;
      for (auto& x : v) out.push_back(x.id);
      ctx->Set(nd.Output(0), Tensor::FromVector(out));
      return;
    }
    std::vector<std::vector<IdWeightType>> rows;
    ReadNeighbors(ctx, nd, &rows);
    for (auto& r : rows) pp.Apply(&r);
    EmitNeighbors(nd, ctx, rows);
  }
};

class NbFilterOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    std::vector<std::vector<IdWeightType>> rows;
    ReadNeighbors(ctx, nd, &rows);
    auto allowed_v = ctx->Get(nd.inputs.at(4)).ToUInt64();
    std::unordered_set<uint64_t> allowed(allowed_v.begin(), allowed_v.end());
    PostProcess pp = PostProcess::Parse(nd.post_process);
    for (auto& r : rows) {
      std::vector<IdWeightType> keep;
      for (auto& x : r)
        if (allowed.count(x.id)) keep.push_back(x);
      pp.Apply(&keep);
      r.swap(keep);
    }
    EmitNeighbors(nd, ctx, rows);
  }
};

// ---------------------------------------------------------------- layer-wise sampling (client side)
class SampleRootOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    auto roots = ctx->Get(nd.inputs.at(0)).ToUInt64();
    const Tensor& wt = ctx->Get(nd.inputs.at(1));
    const int64_t n = ctx->AttrInt(nd.attrs.at(0)), m = ctx->AttrInt(nd.attrs.at(1));
    const uint64_t def = nd.attrs.size() > 2 ? static_cast<uint64_t>(ctx->AttrInt(nd.attrs[2])) : kDefaultNode;
    Rng rng(GlobalSeed() ^ 0x2007ULL, NextEpoch());
    std::vector<uint64_t> out;
    const int64_t batches = (static_cast<int64_t>(roots.size()) + n - 1) / std::max<int64_t>(1, n);
    for (int64_t b = 0; b < batches; ++b) {
      std::vector<float> w;
      for (int64_t i = b * n; i < std::min<int64_t>((b + 1) * n, roots.size()); ++i)
        w.push_back(static_cast<float>(wt.AsDouble(i)));
      AliasTable at(w);
      for (int64_t k = 0; k < m; ++k)
        out.push_back(at.total() > 0 ? roots[b * n + at.Sample(rng)] : def);
    }
    ctx->Set(nd.Output(0), Tensor::FromVector(out));
  }
};

class LocalSampleLayerOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    std::vector<std::vector<IdWeightType>> rows;
    ReadNeighbors(ctx, nd, &rows);
    const int64_t n = ctx->AttrInt(nd.attrs.at(0)), m = ctx->AttrInt(nd.attrs.at(1));
    const std::string wf = nd.attrs.size() > 2 ? nd.attrs[2] : "";
    const uint64_t def = nd.attrs.size() > 3 ? static_cast<uint64_t>(ctx->AttrInt(nd.attrs[3])) : kDefaultNode;
    Rng rng(GlobalSeed() ^ 0x2008ULL, NextEpoch());
    std::vector<uint64_t> out;
    const int64_t batches = (static_cast<int64_t>(rows.size()) + n - 1) / std::max<int64_t>(1, n);
    for (int64_t b = 0; b < batches; ++b) {
      // dedup (dst, type), sum weights, optional sqrt (reference local_sample_layer_op.cc:42-146)
      std::map<std::pair<uint64_t, int32_t>, double> acc;
      for (int64_t i = b * n; i < std::min<int64_t>((b + 1) * n, rows.size()); ++i)
        for (auto& x : rows[i]) acc[{x.id, x.type}] += x.weight;
      std::vector<uint64_t> ids;
      std::vector<float> w;
      for (auto& kv : acc) {
        ids.push_back(kv.first.first);
        w.push_back(static_cast<float>(wf == "sqrt" ? std::sqrt(kv.second) : kv.second));
      }
      AliasTable at(w);
      for (int64_t k = 0; k < m; ++k) out.push_back(at.total() > 0 ? ids[at.Sample(rng)] : def);
    }
    ctx->Set(nd.Output(0), Tensor::FromVector(out));
  }
};

class SampleGraphLabelOp : public OpKernel {
 public:
  void Compute(const NodeDef& nd, OpContext* ctx) override {
    const int64_t count = ctx->AttrInt(nd.attrs.at(0));
    std::vector<std::string> labels = ctx->env()->graph_labels;
    if (labels.empty() && ctx->env()->graph) labels = ctx->env()->graph->graph_labels();
    if (labels.empty()) EULER_THROW("graph label set is empty");
    Rng rng(GlobalSeed() ^ 0x61ABULL, NextEpoch());
    std::vector<std::string> out;
    for (int64_t i = 0; i < count; ++i) out.push_back(labels[rng.Below(labels.size())]);
    ctx->Set(nd.Output(0), Tensor::Strings(out));
  }
};

}  // namespace

REGISTER_OP_KERNEL("ID_SPLIT", IdSplitOp);
REGISTER_OP_KERNEL("ID_SRC", IdSrcOp);
REGISTER_OP_KERNEL("GP_ID_SPLIT", GpIdSplitOp);
REGISTER_OP_KERNEL("BROAD_CAST_SPLIT", BroadcastSplitOp);
REGISTER_OP_KERNEL("SAMPLE_NODE_SPLIT", SampleNodeSplitOp);
REGISTER_OP_KERNEL("SAMPLE_EDGE_SPLIT", SampleEdgeSplitOp);
REGISTER_OP_KERNEL("SAMPLE_N_WITH_TYPES_SPLIT", SampleNWithTypesSplitOp);
REGISTER_OP_KERNEL("APPEND_MERGE", AppendMergeOp);
REGISTER_OP_KERNEL("IDX_MERGE", IdxMergeOp);
REGISTER_OP_KERNEL("DATA_MERGE", DataMergeOp);
REGISTER_OP_KERNEL("REGULAR_DATA_MERGE", RegularDataMergeOp);
REGISTER_OP_KERNEL("MULTI_TYPE_IDX_MERGE", RowAppendIdxMergeOp);
REGISTER_OP_KERNEL("MULTI_TYPE_DATA_MERGE", RowAppendDataMergeOp);
REGISTER_OP_KERNEL("IDX_ROW_APPEND_MERGE", RowAppendIdxMergeOp);
REGISTER_OP_KERNEL("DATA_ROW_APPEND_MERGE", RowAppendDataMergeOp);
REGISTER_OP_KERNEL("ID_UNIQUE", IdUniqueOp);
REGISTER_OP_KERNEL("IDX_GATHER", IdxGatherOp);
REGISTER_OP_KERNEL("DATA_GATHER", DataGatherOp);
REGISTER_OP_KERNEL("AS", AsOp);
REGISTER_OP_KERNEL("POST_PROCESS", PostProcessOp);
REGISTER_OP_KERNEL("API_GET_NB_FILTER", NbFilterOp);
REGISTER_OP_KERNEL("API_SAMPLE_ROOT", SampleRootOp);
REGISTER_OP_KERNEL("API_LOCAL_SAMPLE_L", LocalSampleLayerOp);
REGISTER_OP_KERNEL("API_SAMPLE_GRAPH_LABEL", SampleGraphLabelOp);
// graph-partition variants: same merges (ids may repeat across partitions; the merges
// never assume disjoint shards), plus the row-level unique merge
REGISTER_OP_KERNEL("GP_APPEND_MERGE", AppendMergeOp);
REGISTER_OP_KERNEL("GP_IDX_MERGE", IdxMergeOp);
REGISTER_OP_KERNEL("GP_DATA_MERGE", DataMergeOp);
REGISTER_OP_KERNEL("GP_REGULAR_DATA_MERGE", RegularDataMergeOp);
REGISTER_OP_KERNEL("GP_UNIQUE_MERGE", GpUniqueMergeOp);
REGISTER_OP_KERNEL("API_SPARSE_GEN_ADJ", SparseGenAdjOp);
REGISTER_OP_KERNEL("API_GATHER_RESULT", GatherResultOp);
REGISTER_OP_KERNEL("API_RESHAPE", ReshapeOp);

void LinkDistOps() {}

}  // namespace euler
