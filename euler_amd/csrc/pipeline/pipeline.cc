// Native SageDataFlow + feature batch pipeline (see pipeline.h).
#include "pipeline/pipeline.h"

#include <string.h>

#include <algorithm>
#include <mutex>

#include "rpc/rpc.h"

namespace euler {

namespace {

// tf.unique (first-occurrence order): open addressing, linear probing
void UniqueInto(const int64_t* xs, int64_t n, int64_t* uniq, int64_t* nu, int64_t* inv,
                std::vector<std::pair<int64_t, int64_t>>* table) {
  uint64_t cap = 16;
  while (cap < static_cast<uint64_t>(2 * n)) cap <<= 1;
  const uint64_t mask = cap - 1;
  table->assign(cap, {0, -1});
  int64_t k = 0;
  for (int64_t i = 0; i < n; ++i) {
    const int64_t v = xs[i];
    const uint64_t z = static_cast<uint64_t>(v) * 0x9e3779b97f4a7c15ull;
    uint64_t h = (z ^ (z >> 29)) & mask;
    for (;;) {
      auto& c = (*table)[h];
      if (c.second < 0) {
        c = {v, k};
        uniq[k++] = v;
        break;
      }
      if (c.first == v) break;
      h = (h + 1) & mask;
    }
    inv[i] = (*table)[h].second;
  }
  *nu = k;
}

}  // namespace

SageSlotLayout SageSlotLayout::Make(const SageBatchSpec& s) {
  SageSlotLayout l;
  const int L = static_cast<int>(s.fanouts.size());
  l.cap.assign(L + 1, 0);
  l.ecap.assign(L + 1, 0);
  l.off_nid.assign(L + 1, 0);
  l.off_res.assign(L + 1, 0);
  l.off_src.assign(L + 1, 0);
  l.off_nbr.assign(L + 1, 0);
  l.cap[0] = s.batch;
  int64_t off = 16 + s.batch;
  for (int h = 1; h <= L; ++h) {
    const int64_t f = s.fanouts[h - 1];
    l.cap[h] = l.cap[h - 1] * (f + 1);
    l.ecap[h] = l.cap[h - 1] * f + (s.self_loops ? l.cap[h - 1] : 0);
    l.off_nid[h] = off;
    off += l.cap[h];
    l.off_res[h] = off;
    off += l.cap[h - 1];
    l.off_src[h] = off;
    off += 2 * l.ecap[h];
    l.off_nbr[h] = off;
    off += (l.cap[h - 1] * (f + (s.self_loops ? 1 : 0)) + 1) / 2;
  }
  l.ints = off;
  for (int d : s.dense_dims) l.feat_dim += d;
  l.off_labels = l.cap[L] * l.feat_dim;
  l.floats = l.off_labels + static_cast<int64_t>(s.batch) * s.label_dim;
  return l;
}

namespace {

// the bucket half of a keyed root draw: an alias table over the global bucket weights
// (built once, on first use, from whatever source knows them)
class KeyedRootTable {
 public:
  template <typename Fn>
  void Ensure(Fn weights) {
    std::call_once(once_, [&] {
      std::vector<double> w = weights();
      double t = 0;
      for (double x : w) t += x;
      ok_ = t > 0;
      if (ok_) alias_.Init(w.data(), w.size());
    });
  }
  // bucket of root i, or -1 when the node type has no weight
  int64_t Bucket(uint64_t key, int64_t i) const {
    if (!ok_) return -1;
    Rng rng(key, 2 * static_cast<uint64_t>(i));
    return alias_.Sample(rng);
  }

 private:
  std::once_flag once_;
  bool ok_ = false;
  AliasTable alias_;
};

// the in-process shard: direct column / CSR reads, keyed sampling
class LocalSource : public SageSource {
 public:
  explicit LocalSource(const Graph* g) : g_(*g), buckets_(KeyedBuckets(g->meta().partitions_num)) {}

  void Roots(const SageBatchSpec& s, uint64_t key, int64_t* roots, float* labels) override {
    table_.Ensure([&] { return g_.NodeBucketWeights(s.node_type, buckets_); });
    for (int i = 0; i < s.batch; ++i) {
      const int64_t b = table_.Bucket(key, i);
      Rng rng(key, 2 * static_cast<uint64_t>(i) + 1);
      roots[i] = b < 0 ? s.default_node
                       : static_cast<int64_t>(g_.SampleNodeInBucket(s.node_type, buckets_, b, rng,
                                                                    static_cast<uint64_t>(s.default_node)));
    }
    if (s.label_dim <= 0) return;
    const Column<float>* lc = s.label_idx >= 0 ? g_.NodeDense(s.label_idx) : nullptr;
    for (int i = 0; i < s.batch; ++i) {
      const int64_t row = g_.Row(static_cast<uint64_t>(roots[i]));
      const float* p = nullptr;
      int64_t m = 0;
      if (lc && row >= 0) lc->Get(row, &p, &m);
      m = std::min<int64_t>(m, s.label_dim);
      if (m > 0) memcpy(labels + i * s.label_dim, p, m * sizeof(float));
      if (m < s.label_dim) memset(labels + i * s.label_dim + m, 0, (s.label_dim - m) * sizeof(float));
    }
  }

  void Hop(const SageBatchSpec& s, int hop, const int64_t* ids, int64_t n, uint64_t key, int64_t* out) override {
    const int k = s.fanouts[hop - 1];
    const uint64_t* u = reinterpret_cast<const uint64_t*>(ids);
    std::vector<uint32_t> occ;
    KeyedOccurrences(u, n, &occ);
    std::vector<int32_t> et = s.etypes[hop - 1];
    if (et.size() == 1 && et[0] < 0) et.clear();
    SampleNeighborsKeyed(g_, u, occ.data(), n, et, k, key, static_cast<uint64_t>(s.default_node),
                         reinterpret_cast<uint64_t*>(out), nullptr, nullptr);
  }

  void Features(const SageBatchSpec& s, const int64_t* ids, int64_t n, int64_t fd, float* out) override {
    std::vector<const Column<float>*> cols;
    for (int idx : s.dense_idx) cols.push_back(g_.NodeDense(idx));
    for (int64_t i = 0; i < n; ++i) {
      const int64_t r = g_.Row(static_cast<uint64_t>(ids[i]));
      float* o = out + i * fd;
      int64_t c0 = 0;
      for (size_t f = 0; f < cols.size(); ++f) {
        const int64_t dim = s.dense_dims[f];
        const float* p = nullptr;
        int64_t m = 0;
        if (cols[f] && r >= 0) cols[f]->Get(r, &p, &m);
        m = std::min(m, dim);
        if (m > 0) memcpy(o + c0, p, m * sizeof(float));
        if (m < dim) memset(o + c0 + m, 0, (dim - m) * sizeof(float));
        c0 += dim;
      }
    }
  }

 private:
  const Graph& g_;
  const uint64_t buckets_;
  KeyedRootTable table_;
};

// ragged (idx [n][2], flat data) -> dense rows [n][w], zero / default padded
template <typename T>
void DenseFromRagged(const Tensor& idx, const T* data, int64_t n, int64_t w, T pad, T* out) {
  const std::vector<int64_t> ix = idx.ToInt64();
  for (int64_t i = 0; i < n; ++i) {
    const int64_t b = 2 * i + 1 < static_cast<int64_t>(ix.size()) ? ix[2 * i] : 0;
    const int64_t e = 2 * i + 1 < static_cast<int64_t>(ix.size()) ? ix[2 * i + 1] : 0;
    const int64_t m = std::min(e - b, w);
    for (int64_t j = 0; j < w; ++j) out[i * w + j] = j < m ? data[b + j] : pad;
  }
}

// the shard servers, through the session's distribute-mode plans (see pipeline.h)
class RemoteSource : public SageSource {
 public:
  explicit RemoteSource(QueryProxy* q) : q_(q), buckets_(KeyedBuckets(q->env()->num_partitions)) {}

  void Roots(const SageBatchSpec& s, uint64_t key, int64_t* roots, float* labels) override {
    // bucket weights once: every shard reports its buckets (zeros elsewhere), summed here
    table_.Ensure([&] {
      std::vector<Tensor> res;
      Check(q_->RunOp("API_NODE_BUCKET_WEIGHT", {}, {std::to_string(s.node_type), std::to_string(buckets_)}, 1, {},
                      &res),
            "bucket weights");
      std::vector<double> w(buckets_, 0.0);
      const double* p = res[0].data<double>();
      for (int64_t j = 0; j < res[0].numel(); ++j) w[j % buckets_] += p[j];
      return w;
    });
    // codes pos * buckets + bucket: the owning shard draws the node with Philox (key, 2 pos + 1)
    std::vector<uint64_t> codes;
    std::vector<int> at;
    for (int i = 0; i < s.batch; ++i) {
      const int64_t b = table_.Bucket(key, i);
      roots[i] = s.default_node;
      if (b < 0) continue;
      codes.push_back(static_cast<uint64_t>(i) * buckets_ + b);
      at.push_back(i);
    }
    std::vector<std::pair<std::string, Tensor>> in = {
        {"codes", Tensor::FromVector(codes)},
        {"node_type", Tensor::FromVector(std::vector<int32_t>{s.node_type})},
        {"nb_buckets", Tensor::FromVector(std::vector<int64_t>{static_cast<int64_t>(buckets_)})},
        {"nb_key", Tensor::FromVector(std::vector<int64_t>{static_cast<int64_t>(key)})}};
    std::string gql = "v(codes).sampleNodeAt(node_type, nb_buckets, nb_key, " + std::to_string(s.default_node) +
                      ").as(r)";
    std::vector<std::string> outs = {"r:0"};
    const bool lab = s.label_dim > 0 && !s.label_name.empty();
    if (lab) {
      gql += ".values(__lab).as(lb)";
      in.push_back({"__lab", Tensor::Strings({s.label_name})});
      outs.push_back("lb:0");
      outs.push_back("lb:1");
    }
    std::vector<Tensor> res;
    Check(q_->Run(gql, in, outs, &res), "roots");
    const std::vector<int64_t> r = res[0].ToInt64();
    for (size_t j = 0; j < at.size() && j < r.size(); ++j) roots[at[j]] = r[j];
    if (s.label_dim > 0) {
      memset(labels, 0, sizeof(float) * s.batch * s.label_dim);
      if (lab) {
        std::vector<float> l(at.size() * s.label_dim);
        DenseFromRagged<float>(res[1], res[2].data<float>(), static_cast<int64_t>(at.size()), s.label_dim, 0.f,
                               l.data());
        for (size_t j = 0; j < at.size(); ++j)
          memcpy(labels + at[j] * s.label_dim, l.data() + j * s.label_dim, sizeof(float) * s.label_dim);
      }
    }
  }

  void Hop(const SageBatchSpec& s, int hop, const int64_t* ids, int64_t n, uint64_t key, int64_t* out) override {
    const int k = s.fanouts[hop - 1];
    std::vector<uint64_t> u(ids, ids + n);
    std::vector<int32_t> et = s.etypes[hop - 1];
    if (et.empty()) et.push_back(-1);
    std::vector<std::pair<std::string, Tensor>> in = {{"nodes", Tensor::FromVector(u)},
                                                       {"edge_types", Tensor::FromVector(et)},
                                                       {"nb_count", Tensor::FromVector(std::vector<int64_t>{k})},
                                                       {"nb_key", Tensor::FromVector(std::vector<int64_t>{
                                                                      static_cast<int64_t>(key)})}};
    std::vector<Tensor> res;
    // keyed: the owning shard draws id's neighbours with Philox (key, KeyedStream(id, occurrence));
    // the split keeps each shard's ids in request order, so occurrences match the full list
    const std::string gql =
        "v(nodes).sampleNB(edge_types, nb_count, " + std::to_string(s.default_node) + ", nb_key).as(nb)";
    Check(q_->Run(gql, in, {"nb:0", "nb:1"}, &res), "sampleNB");
    const std::vector<int64_t> flat = res[1].ToInt64();
    DenseFromRagged<int64_t>(res[0], flat.data(), n, k, s.default_node, out);
  }

  void Features(const SageBatchSpec& s, const int64_t* ids, int64_t n, int64_t fd, float* out) override {
    std::vector<uint64_t> u(ids, ids + n);
    std::vector<std::pair<std::string, Tensor>> in = {{"nodes", Tensor::FromVector(u)}};
    std::string keys;
    std::vector<std::string> outs;
    for (size_t f = 0; f < s.dense_names.size(); ++f) {
      const std::string k = "__f" + std::to_string(f);
      in.push_back({k, Tensor::Strings({s.dense_names[f]})});
      keys += (f ? ", " : "") + k;
      outs.push_back("fea:" + std::to_string(2 * f));
      outs.push_back("fea:" + std::to_string(2 * f + 1));
    }
    std::vector<Tensor> res;
    Check(q_->Run("v(nodes).values(" + keys + ").as(fea)", in, outs, &res), "values");
    std::vector<float> col;
    int64_t c0 = 0;
    for (size_t f = 0; f < s.dense_names.size(); ++f) {
      const int64_t dim = s.dense_dims[f];
      col.assign(static_cast<size_t>(n * dim), 0.f);
      DenseFromRagged<float>(res[2 * f], res[2 * f + 1].data<float>(), n, dim, 0.f, col.data());
      for (int64_t i = 0; i < n; ++i) memcpy(out + i * fd + c0, col.data() + i * dim, dim * sizeof(float));
      c0 += dim;
    }
  }

 private:
  static void Check(const Status& st, const char* what) {
    if (!st.ok()) EULER_THROW("SagePipeline remote " << what << ": " << st.ToString());
  }
  QueryProxy* q_;
  const uint64_t buckets_;
  KeyedRootTable table_;
};

}  // namespace

std::unique_ptr<SageSource> MakeLocalSource(const Graph* g) { return std::unique_ptr<SageSource>(new LocalSource(g)); }
std::unique_ptr<SageSource> MakeRemoteSource(QueryProxy* q) {
  return std::unique_ptr<SageSource>(new RemoteSource(q));
}

SagePipeline::SagePipeline(const Graph* g, SageBatchSpec spec, std::vector<int64_t*> ints, std::vector<float*> floats,
                           int workers, uint64_t seed)
    : SagePipeline(MakeLocalSource(g), std::move(spec), std::move(ints), std::move(floats), workers, seed) {}

SagePipeline::SagePipeline(std::unique_ptr<SageSource> src, SageBatchSpec spec, std::vector<int64_t*> ints,
                           std::vector<float*> floats, int workers, uint64_t seed)
    : src_(std::move(src)), spec_(std::move(spec)), ints_(std::move(ints)), floats_(std::move(floats)), seed_(seed) {
  lay_ = SageSlotLayout::Make(spec_);
  if (ints_.size() != floats_.size() || ints_.empty()) EULER_THROW("SagePipeline: one int and one float buffer per slot");
  if (spec_.etypes.size() != spec_.fanouts.size() || spec_.fanouts.empty() || spec_.fanouts.size() > 7)
    EULER_THROW("SagePipeline: 1..7 hops, one edge-type list per fanout");
  if (spec_.dense_dims.size() != std::max(spec_.dense_idx.size(), spec_.dense_names.size()))
    EULER_THROW("SagePipeline: one dimension per feature");
  for (int i = 0; i < static_cast<int>(ints_.size()); ++i) free_.push_back(i);
  Start(workers);
}

void SagePipeline::Start(int workers) {
  const int nw = std::max(1, workers);
  for (int w = 0; w < nw; ++w) threads_.emplace_back([this] { Worker(); });
}

SagePipeline::~SagePipeline() { Stop(); }

void SagePipeline::Stop() {
  {
    std::lock_guard<std::mutex> l(mu_);
    if (stop_ && threads_.empty()) return;
    stop_ = true;
  }
  cv_free_.notify_all();
  cv_ready_.notify_all();
  for (auto& t : threads_)
    if (t.joinable()) t.join();
  threads_.clear();
}

void SagePipeline::Worker() {
  for (;;) {
    int slot;
    uint64_t seq;
    {
      std::unique_lock<std::mutex> l(mu_);
      cv_free_.wait(l, [&] { return stop_ || !free_.empty(); });
      if (stop_) return;
      slot = free_.back();
      free_.pop_back();
      seq = issue_seq_++;
    }
    Fill(slot, seq);
    {
      std::lock_guard<std::mutex> l(mu_);
      ready_[seq] = slot;
    }
    cv_ready_.notify_all();
  }
}

int SagePipeline::Next() {
  std::unique_lock<std::mutex> l(mu_);
  cv_ready_.wait(l, [&] { return stop_ || ready_.count(next_seq_); });
  if (stop_) return -1;
  auto it = ready_.find(next_seq_);
  const int slot = it->second;
  ready_.erase(it);
  ++next_seq_;
  return slot;
}

void SagePipeline::Release(int slot) {
  {
    std::lock_guard<std::mutex> l(mu_);
    free_.push_back(slot);
  }
  cv_free_.notify_one();
}

void SagePipeline::Fill(int slot, uint64_t seq) {
  const SageBatchSpec& s = spec_;
  const SageSlotLayout& lay = lay_;
  int64_t* I = ints_[slot];
  float* Fp = floats_[slot];
  const int L = static_cast<int>(s.fanouts.size());
  // roots (+ labels)
  int64_t* lvl0 = I + 16;
  src_->Roots(s, KeyedKey(seed_, seq, 0), lvl0, s.label_dim > 0 ? Fp + lay.off_labels : nullptr);
  I[0] = L;
  I[1] = s.batch;
  // hops
  std::vector<int64_t> cat, inv;
  std::vector<std::pair<int64_t, int64_t>> table;
  const int64_t* cur = lvl0;
  int64_t n = s.batch;
  for (int h = 1; h <= L; ++h) {
    const int k = s.fanouts[h - 1];
    cat.resize(static_cast<size_t>(n * k + n));
    inv.resize(cat.size());
    src_->Hop(s, h, cur, n, KeyedKey(seed_, seq, h), cat.data());
    std::copy(cur, cur + n, cat.begin() + n * k);
    int64_t* nid = I + lay.off_nid[h];
    int64_t nu = 0;
    UniqueInto(cat.data(), static_cast<int64_t>(cat.size()), nid, &nu, inv.data(), &table);
    int64_t* res = I + lay.off_res[h];
    std::copy(inv.end() - n, inv.end(), res);
    const int64_t e = s.self_loops ? n * k + n : n * k;
    int64_t* src = I + lay.off_src[h];
    int64_t* dst = src + e;  // packed behind src: [2, e] is contiguous
    for (int64_t i = 0; i < n * k; ++i) src[i] = i / k;
    if (s.self_loops)
      for (int64_t i = 0; i < n; ++i) src[n * k + i] = i;
    std::copy(inv.begin(), inv.begin() + e, dst);
    // dense neighbour matrix (int32, self loop last) for the fused SAGE kernel
    int32_t* nb = reinterpret_cast<int32_t*>(I + lay.off_nbr[h]);
    const int w = k + (s.self_loops ? 1 : 0);
    for (int64_t i = 0; i < n; ++i) {
      for (int j = 0; j < k; ++j) nb[i * w + j] = static_cast<int32_t>(inv[i * k + j]);
      if (s.self_loops) nb[i * w + k] = static_cast<int32_t>(inv[n * k + i]);
    }
    // capacity padding: rows past n read the zero row (-1), so fixed-capacity consumers
    // (the graph-captured step) compute exact results for the valid rows
    std::fill(res + n, res + lay.cap[h - 1], int64_t{-1});
    std::fill(nb + n * w, nb + lay.cap[h - 1] * w, int32_t{-1});
    I[1 + h] = nu;
    I[8 + h] = e;
    cur = nid;
    n = nu;
  }
  // dense input features of the outermost node set, row-major [n][feat_dim]
  if (lay.feat_dim > 0) src_->Features(s, cur, n, lay.feat_dim, Fp);
}

}  // namespace euler
