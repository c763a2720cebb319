// Keyed (shard-independent) sampling — see graph.h.
//
// Why buckets: a weighted draw over the whole node set needs the whole set's weights; on
// shard servers each server only holds its own nodes.  Grouping nodes into B virtual
// buckets by id % B, with B a multiple of the partition count P, puts every bucket on exactly
// one shard (shard = (id % P) % S = (bucket % P) % S), so a draw = (bucket by the global
// bucket weights, node inside the bucket) can run as "client picks the bucket, owning shard
// picks the node" and give the same node as an in-process draw.  Inside a bucket, nodes are
// in row order = sorted-id order and the weight sums are accumulated in double in that order,
// so a shard and the whole graph build bit-identical tables.
#include <algorithm>
#include <mutex>

#include "graph/graph.h"

namespace euler {

namespace {

inline uint64_t Mix64(uint64_t x) {
  x += 0x9E3779B97F4A7C15ULL;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ULL;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBULL;
  return x ^ (x >> 31);
}

struct BucketTables {
  uint64_t buckets = 0;
  std::vector<int64_t> start;  // [buckets + 1] into rows
  std::vector<int64_t> rows;   // rows grouped by bucket, sorted-id order inside
  std::vector<double> wsum;    // [buckets]
  std::vector<AliasTable> alias;
};

}  // namespace

struct Graph::BucketCache {
  std::mutex mu;
  std::map<std::pair<int, uint64_t>, std::shared_ptr<BucketTables>> tables;
};

std::shared_ptr<Graph::BucketCache> Graph::NewBucketCache() { return std::make_shared<BucketCache>(); }

uint64_t KeyedBuckets(uint32_t partitions) {
  const uint64_t p = std::max<uint32_t>(1, partitions);
  return p * ((1024 + p - 1) / p);
}

uint64_t KeyedKey(uint64_t seed, uint64_t batch, uint64_t hop) {
  return Mix64(Mix64(seed ^ 0x6B65796564ULL) + batch * 0x100000001B3ULL + hop);
}

uint64_t KeyedStream(uint64_t id, uint64_t occurrence) { return Mix64(id) + occurrence * 0xD1B54A32D192ED03ULL; }

const void* Graph::BucketSampler(int node_type, uint64_t buckets) const {
  const int t = node_type < 0 ? -1 : node_type;
  std::lock_guard<std::mutex> l(bucket_cache_->mu);
  auto& slot = bucket_cache_->tables[{t, buckets}];
  if (slot) return slot.get();
  auto bt = std::make_shared<BucketTables>();
  bt->buckets = buckets;
  bt->start.assign(buckets + 1, 0);
  auto want = [&](int64_t r) { return t < 0 || node_type_[r] == t; };
  const int64_t N = num_nodes();
  for (int64_t r = 0; r < N; ++r)
    if (want(r)) ++bt->start[node_ids_[r] % buckets + 1];
  for (uint64_t b = 0; b < buckets; ++b) bt->start[b + 1] += bt->start[b];
  bt->rows.resize(bt->start[buckets]);
  std::vector<int64_t> fill(bt->start.begin(), bt->start.end() - 1);
  for (int64_t r = 0; r < N; ++r)  // rows ascend with ids: each bucket stays id-sorted
    if (want(r)) bt->rows[fill[node_ids_[r] % buckets]++] = r;
  bt->wsum.assign(buckets, 0.0);
  bt->alias.resize(buckets);
  std::vector<double> w;
  for (uint64_t b = 0; b < buckets; ++b) {
    const int64_t a = bt->start[b], e = bt->start[b + 1];
    if (a == e) continue;
    w.assign(e - a, 0.0);
    double s = 0.0;
    for (int64_t i = a; i < e; ++i) s += (w[i - a] = node_weight_[bt->rows[i]]);
    bt->wsum[b] = s;
    bt->alias[b].Init(w.data(), w.size());
  }
  slot = bt;
  return slot.get();
}

std::vector<double> Graph::NodeBucketWeights(int node_type, uint64_t buckets) const {
  if (buckets == 0) return {};
  return static_cast<const BucketTables*>(BucketSampler(node_type, buckets))->wsum;
}

uint64_t Graph::SampleNodeInBucket(int node_type, uint64_t buckets, uint64_t bucket, Rng& rng, uint64_t def) const {
  if (buckets == 0 || bucket >= buckets) return def;
  const auto* bt = static_cast<const BucketTables*>(BucketSampler(node_type, buckets));
  const AliasTable& at = bt->alias[bucket];
  if (at.empty() || bt->wsum[bucket] <= 0) return def;
  return node_ids_[bt->rows[bt->start[bucket] + at.Sample(rng)]];
}

void KeyedOccurrences(const uint64_t* ids, int64_t n, std::vector<uint32_t>* occ) {
  occ->assign(n, 0);
  uint64_t cap = 16;
  while (cap < static_cast<uint64_t>(2 * n)) cap <<= 1;
  std::vector<uint64_t> keys(cap);
  std::vector<uint32_t> cnt(cap, 0);  // 0 = empty slot, else occurrences so far
  for (int64_t i = 0; i < n; ++i) {
    uint64_t h = Mix64(ids[i]) & (cap - 1);
    while (cnt[h] && keys[h] != ids[i]) h = (h + 1) & (cap - 1);
    keys[h] = ids[i];
    (*occ)[i] = cnt[h]++;
  }
}

void SampleNeighborsKeyed(const Graph& g, const uint64_t* ids, const uint32_t* occ, int64_t n,
                          const std::vector<int32_t>& etypes, int k, uint64_t key, uint64_t def, uint64_t* out_id,
                          float* out_w, int32_t* out_t) {
  std::vector<IdWeightType> tmp;
  for (int64_t i = 0; i < n; ++i) {
    Rng rng(key, KeyedStream(ids[i], occ[i]));
    g.SampleNeighbor(g.Row(ids[i]), etypes, k, true, rng, &tmp);
    for (int j = 0; j < k; ++j) {
      const bool ok = j < static_cast<int>(tmp.size());
      out_id[i * k + j] = ok ? tmp[j].id : def;
      if (out_w) out_w[i * k + j] = ok ? tmp[j].weight : 0.f;
      if (out_t) out_t[i * k + j] = ok ? tmp[j].type : -1;
    }
  }
}

}  // namespace euler
