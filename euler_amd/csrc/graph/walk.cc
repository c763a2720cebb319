// Random walks on the local shard (SURVEY §2.3 random_walk; reference
// tf_euler/kernels/random_walk_op.cc:70-188).
//
// p = q = 1: chained weighted neighbour sampling.  Otherwise node2vec's second-order
// bias on the edge weights of the current node's candidates: 1/p for the node the walk
// came from, 1 for common neighbours of that node (under the previous step's edge
// types), 1/q for the rest.  As in the reference, the "previous node" of the first step
// is the start node itself with no neighbour set, so step 0 is plain weighted sampling
// except that a self loop gets 1/p.
//
// Reference mechanics replaced: the reference issues one GQL outV query per step for the
// whole batch and biases with a sorted merge over both neighbour lists (which assumed
// sorted groups the converter never produced).  Here every walk is one task
// on the engine pool with its own Philox stream (seed, walk index) — reproducible per
// seed independent of thread count — and membership in the previous node's neighbour
// set is a binary search in its id-sorted segments (graph.h): O(deg log deg) per step.
#include <algorithm>

#include "graph/graph.h"

namespace euler {

namespace {

bool InSegments(const Adjacency& A, int64_t row, int T, const std::vector<int32_t>& etypes, uint64_t id) {
  if (row < 0) return false;
  auto in_seg = [&](int64_t seg) {
    const uint64_t* b = A.nbr.data() + A.indptr[seg];
    const uint64_t* e = A.nbr.data() + A.indptr[seg + 1];
    return std::binary_search(b, e, id);
  };
  if (etypes.empty()) {
    for (int t = 0; t < T; ++t)
      if (in_seg(row * T + t)) return true;
    return false;
  }
  for (int32_t t : etypes)
    if (t >= 0 && t < T && in_seg(row * T + t)) return true;
  return false;
}

}  // namespace

void RandomWalk(const Graph& g, const uint64_t* starts, int64_t n, const std::vector<std::vector<int32_t>>& etypes,
                float p, float q, int64_t default_node, uint64_t seed, int64_t* out) {
  const int L = static_cast<int>(etypes.size());
  const Adjacency& A = g.adj(true);
  const int T = g.num_edge_types();
  const bool biased = p != 1.f || q != 1.f;
  const double inv_p = 1.0 / p, inv_q = 1.0 / q;
  ThreadPool::Default()->ParallelFor(n, 64, [&](int64_t b, int64_t e) {
    std::vector<int64_t> segs;
    std::vector<double> acc;
    for (int64_t i = b; i < e; ++i) {
      Rng rng(seed, static_cast<uint64_t>(i));
      int64_t* o = out + i * (L + 1);
      uint64_t cur = starts[i], prev = starts[i];
      bool alive = true;
      const std::vector<int32_t>* prev_types = nullptr;  // none before the first step
      o[0] = static_cast<int64_t>(starts[i]);
      for (int s = 0; s < L; ++s) {
        int64_t nxt = default_node;
        const int64_t row = alive ? g.Row(cur) : -1;
        if (row >= 0) {
          segs.clear();
          if (etypes[s].empty()) {
            for (int t = 0; t < T; ++t) segs.push_back(row * T + t);
          } else {
            for (int32_t t : etypes[s])
              if (t >= 0 && t < T) segs.push_back(row * T + t);
          }
          // cumulative (biased) weights over the candidate edges of every segment
          acc.clear();
          double tot = 0.0;
          const int64_t prow = biased && prev_types ? g.Row(prev) : -1;
          for (int64_t sg : segs)
            for (uint64_t k = A.indptr[sg]; k < A.indptr[sg + 1]; ++k) {
              double w = A.EdgeWeight(k, A.indptr[sg]);
              if (biased) {
                const uint64_t c = A.nbr[k];
                if (c == prev) w *= inv_p;
                else if (!(prev_types && InSegments(A, prow, T, *prev_types, c))) w *= inv_q;
              }
              tot += w;
              acc.push_back(tot);
            }
          if (tot > 0.0) {
            const double u = rng.UniformD() * tot;
            const size_t pick = std::min<size_t>(std::upper_bound(acc.begin(), acc.end(), u) - acc.begin(),
                                                 acc.size() - 1);
            size_t k = pick;
            for (int64_t sg : segs) {
              const uint64_t len = A.indptr[sg + 1] - A.indptr[sg];
              if (k < len) {
                nxt = static_cast<int64_t>(A.nbr[A.indptr[sg] + k]);
                break;
              }
              k -= len;
            }
          }
        }
        o[s + 1] = nxt;
        alive = row >= 0 && nxt != default_node;
        prev = cur;
        prev_types = &etypes[s];
        cur = static_cast<uint64_t>(nxt);
      }
    }
  });
}

}  // namespace euler
