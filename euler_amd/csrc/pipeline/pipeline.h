// Native mini-batch pipeline for the engine (CPU-sampling) GraphSAGE path (SURVEY §7.1,
// §2.7 K13; reference hot loop: tf_euler/kernels/sample_fanout_with_feature_op.cc:43-69,
// get_dense_feature_op.cc:89-116, python/dataflow/sage_dataflow.py:35-50).
//
// Worker threads (GIL-free, one batch per worker at a time) build COMPLETE batches: roots
// by the node-type sampler, every hop of the SageDataFlow (fixed-fanout sampling,
// first-occurrence unique of [neighbours | nodes], target positions, target-major edge
// list + self loops), the dense input features of the outermost node set and the roots'
// labels — straight into caller-provided (pinned) slot buffers of fixed capacity.  Slots
// circulate free -> filling -> ready -> consumer -> free; batches are delivered in sequence
// order and batch b draws from the Philox keys KeyedKey(seed, b, hop) (graph.h), so the
// stream of batches is reproducible for any worker count and for the in-process graph or
// any id-hash sharding of it (keyed root draws assume bucket id % B lives on shard
// (bucket % P) % S; graph_partition sessions with an arbitrary partition_fn are refused).
#pragma once

#include <stdint.h>

#include <condition_variable>
#include <map>
#include <memory>
#include <string>
#include <mutex>
#include <thread>
#include <vector>

#include "graph/graph.h"

namespace euler {

class QueryProxy;

struct SageBatchSpec {
  int batch = 0;
  int node_type = -1;                          // roots: sample_node(batch, node_type)
  std::vector<std::vector<int32_t>> etypes;    // per hop (empty = all types)
  std::vector<int> fanouts;
  int64_t default_node = -1;
  bool self_loops = true;
  std::vector<int> dense_idx, dense_dims;      // input features (concatenated)
  int label_idx = -1, label_dim = 0;           // dense label column of the roots
  std::vector<std::string> dense_names;        // the same columns by name (remote source)
  std::string label_name;
};

// Where a batch's graph lookups go.  LocalSource: the in-process shard.  RemoteSource: the
// shard servers, through the session's compiled distribute-mode plans — per batch one
// roots (+ labels) query, one sampleNB query per hop over the hop's unique frontier and
// one values() query for the outermost node set; each query is one RPC per shard
// (split -> REMOTE -> merge, REMOTE fusion), issued by the worker thread that owns the
// batch, so W workers keep W batches of RPCs in flight.
// Both draw with the keyed samplers of graph.h: batch b, hop h uses the Philox key
// KeyedKey(seed, b, h), roots go through the virtual node buckets and neighbour draws are
// keyed by (id, occurrence), so a batch is the same for any worker count and whether the
// graph is in-process or on any number of shard servers (the remote side runs the same
// code: API_SAMPLE_NODE_AT, keyed API_SAMPLE_NB).
class SageSource {
 public:
  virtual ~SageSource() = default;
  // roots [batch] and, with label_dim > 0, their labels [batch][label_dim]
  virtual void Roots(const SageBatchSpec& s, uint64_t key, int64_t* roots, float* labels) = 0;
  // k neighbour draws per id (default_node where none), out [n * k]
  virtual void Hop(const SageBatchSpec& s, int hop, const int64_t* ids, int64_t n, uint64_t key, int64_t* out) = 0;
  // dense input features [n][feat_dim] (zero-filled when missing)
  virtual void Features(const SageBatchSpec& s, const int64_t* ids, int64_t n, int64_t feat_dim, float* out) = 0;
};

std::unique_ptr<SageSource> MakeLocalSource(const Graph* g);
std::unique_ptr<SageSource> MakeRemoteSource(QueryProxy* proxy);

// Slot layout (int64 words):
//   [0, 16)            header: hdr[0] = L, hdr[1 + h] = |n_id of level h| (h = 0..L),
//                      hdr[8 + h] = |edges of hop h| (h = 1..L, hdr[8] unused)
//   level 0 ids        [batch]
//   per hop h = 1..L:  n_id [cap_h] | res [cap_{h-1}] | edges [2 * ecap_h] (src[e] then dst[e]
//                      packed: the [2, e] edge index is one contiguous view) | nbr: int32
//                      [cap_{h-1}][F_h (+1)] dense neighbour positions (self loop last);
//                      res and nbr are padded with -1 up to cap_{h-1} rows
// float words: features [cap_L][sum dense_dims] | labels [batch][label_dim]
struct SageSlotLayout {
  std::vector<int64_t> cap, ecap;   // per level / hop
  std::vector<int64_t> off_nid, off_res, off_src, off_nbr;  // int64 offsets per hop (index 0 unused)
  int64_t ints = 0, floats = 0, feat_dim = 0, off_labels = 0;
  static SageSlotLayout Make(const SageBatchSpec& s);
};

class SagePipeline {
 public:
  SagePipeline(const Graph* g, SageBatchSpec spec, std::vector<int64_t*> ints, std::vector<float*> floats,
               int workers, uint64_t seed);
  SagePipeline(std::unique_ptr<SageSource> src, SageBatchSpec spec, std::vector<int64_t*> ints,
               std::vector<float*> floats, int workers, uint64_t seed);
  ~SagePipeline();
  // the next batch's slot, in sequence order (blocks; -1 after Stop)
  int Next();
  // the consumer is done with a slot (its H2D copy completed)
  void Release(int slot);
  void Stop();
  const SageSlotLayout& layout() const { return lay_; }
  int64_t batches() const { return next_seq_; }

 private:
  void Start(int workers);
  void Worker();
  void Fill(int slot, uint64_t seq);
  std::unique_ptr<SageSource> src_;
  SageBatchSpec spec_;
  SageSlotLayout lay_;
  std::vector<int64_t*> ints_;
  std::vector<float*> floats_;
  uint64_t seed_;
  std::mutex mu_;
  std::condition_variable cv_free_, cv_ready_;
  std::vector<int> free_;
  std::map<uint64_t, int> ready_;  // sequence -> slot
  uint64_t issue_seq_ = 0, next_seq_ = 0;
  bool stop_ = false;
  std::vector<std::thread> threads_;
};

}  // namespace euler
