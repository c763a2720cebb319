// Shared helpers for engine kernels: ragged outputs, reproducible parallel
// sampling, DNF / post-process handling.
#pragma once

#include <algorithm>
#include <atomic>

#include "framework/framework.h"
#include "graph/graph.h"
#include "index/index.h"

namespace euler {

constexpr uint64_t kDefaultNode = UINT64_MAX;  // reference DEFAULT_UINT64

// idx tensor [n, 2] int32 (begin, end) from per-row counts
inline Tensor MakeIdx(const std::vector<int64_t>& counts) {
  Tensor t(DType::kInt32, {static_cast<int64_t>(counts.size()), 2});
  int32_t* p = t.data<int32_t>();
  int64_t acc = 0;
  for (size_t i = 0; i < counts.size(); ++i) {
    p[2 * i] = static_cast<int32_t>(acc);
    acc += counts[i];
    p[2 * i + 1] = static_cast<int32_t>(acc);
  }
  return t;
}

inline Tensor MakeUniformIdx(int64_t n, int64_t per) {
  Tensor t(DType::kInt32, {n, 2});
  int32_t* p = t.data<int32_t>();
  for (int64_t i = 0; i < n; ++i) {
    p[2 * i] = static_cast<int32_t>(i * per);
    p[2 * i + 1] = static_cast<int32_t>((i + 1) * per);
  }
  return t;
}

// Reproducible parallel loop: fixed-size chunks, chunk c draws from
// Rng(global seed + epoch, c) whatever thread runs it.
inline uint64_t NextEpoch() { return NextOpEpoch(); }

template <typename Fn>
void ParallelChunks(int64_t n, int64_t chunk, Fn fn) {
  const uint64_t epoch = NextEpoch();
  const uint64_t seed = GlobalSeed() * 0x9E3779B97F4A7C15ULL + epoch;
  const int64_t nchunks = (n + chunk - 1) / chunk;
  auto body = [&](int64_t cb, int64_t ce) {
    for (int64_t c = cb; c < ce; ++c) {
      Rng rng(seed, static_cast<uint64_t>(c));
      fn(c * chunk, std::min(n, (c + 1) * chunk), rng);
    }
  };
  if (nchunks <= 1) {
    body(0, nchunks);
    return;
  }
  ThreadPool::Default()->ParallelFor(nchunks, 1, body);
}

// input ids of a node (1-D u64) — also accepts [n,3] edges (returns src column)
inline std::vector<uint64_t> IdsOf(const Tensor& t) { return t.ToUInt64(); }

struct EdgeKey {
  uint64_t src, dst;
  int32_t type;
};
inline std::vector<EdgeKey> EdgesOf(const Tensor& t) {
  std::vector<EdgeKey> v;
  const int64_t n = t.shape().size() == 2 ? t.dim(0) : t.numel() / 3;
  v.reserve(n);
  for (int64_t i = 0; i < n; ++i)
    v.push_back({static_cast<uint64_t>(t.AsInt(3 * i)), static_cast<uint64_t>(t.AsInt(3 * i + 1)),
                 static_cast<int32_t>(t.AsInt(3 * i + 2))});
  return v;
}

struct PostProcess {
  bool has_order = false, by_id = true, asc = true;
  int64_t limit = -1;
  static PostProcess Parse(const std::vector<std::string>& pp) {
    PostProcess p;
    for (const auto& s : pp) {
      auto parts = Split(s, " \t,()");
      if (parts.empty()) continue;
      if (parts[0] == "order_by" && parts.size() >= 2) {
        p.has_order = true;
        p.by_id = parts[1] == "id";
        p.asc = parts.size() < 3 || parts[2] == "asc";
      } else if (parts[0] == "limit" && parts.size() >= 2) {
        ParseInt64(parts[1], &p.limit);
      }
    }
    return p;
  }
  bool empty() const { return !has_order && limit < 0; }
  void Apply(std::vector<IdWeightType>* v) const {
    if (has_order) {
      if (by_id)
        std::stable_sort(v->begin(), v->end(), [&](const IdWeightType& a, const IdWeightType& b) {
          return asc ? a.id < b.id : a.id > b.id;
        });
      else
        std::stable_sort(v->begin(), v->end(), [&](const IdWeightType& a, const IdWeightType& b) {
          return asc ? a.weight < b.weight : a.weight > b.weight;
        });
    }
    if (limit >= 0 && static_cast<int64_t>(v->size()) > limit) v->resize(limit);
  }
};

// outputs of a neighbor-type op: idx / ids / weights / types
inline void EmitNeighbors(const NodeDef& nd, OpContext* ctx, const std::vector<std::vector<IdWeightType>>& rows) {
  std::vector<int64_t> counts(rows.size());
  int64_t total = 0;
  for (size_t i = 0; i < rows.size(); ++i) total += (counts[i] = rows[i].size());
  Tensor ids(DType::kUInt64, {total}), w(DType::kFloat, {total}), t(DType::kInt32, {total});
  int64_t k = 0;
  for (auto& r : rows)
    for (auto& x : r) {
      ids.data<uint64_t>()[k] = x.id;
      w.data<float>()[k] = x.weight;
      t.data<int32_t>()[k] = x.type;
      ++k;
    }
  ctx->Set(nd.Output(0), MakeIdx(counts));
  ctx->Set(nd.Output(1), ids);
  ctx->Set(nd.Output(2), w);
  ctx->Set(nd.Output(3), t);
}

inline int ShardOf(uint64_t id, uint32_t partitions, int shards) {
  return static_cast<int>((id % std::max<uint32_t>(1, partitions)) % std::max(1, shards));
}

}  // namespace euler
