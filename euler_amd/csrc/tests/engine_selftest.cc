// Concurrency self-test of the C++ engine, built and run under ThreadSanitizer and
// AddressSanitizer + UBSan by tests/test_sanitizers.py (SURVEY §5 "Race detection /
// sanitizers": the reference had none).
//
// Exercises, from many client threads at once:
//   * the GQL compiler + plan cache and the dependency-counting executor (local mode);
//   * a GraphServer (RPC, connection pool, thread pool) and the remote QueryProxy
//     (REMOTE fan-out, retries, replica selection) over the in-memory registry;
//   * the per-stage engine counters.
// Remote results are checked against local execution of the same deterministic query.
#include <atomic>
#include <cstdio>
#include <memory>
#include <string>
#include <thread>
#include <vector>

#include "framework/framework.h"
#include "graph/graph.h"
#include "rpc/rpc.h"

using namespace euler;

namespace {

int g_failures = 0;

void Expect(bool ok, const char* what) {
  if (!ok) {
    std::fprintf(stderr, "FAILED: %s\n", what);
    ++g_failures;
  }
}

std::vector<std::pair<std::string, Tensor>> NbInputs(const std::vector<uint64_t>& nodes, int64_t count) {
  return {{"nodes", Tensor::FromVector<uint64_t>(nodes)},
          {"edge_types", Tensor::FromVector<int32_t>(std::vector<int32_t>{0})},
          {"nb_count", Tensor::FromVector<int64_t>(std::vector<int64_t>{count})}};
}

void Hammer(QueryProxy* qp, QueryProxy* oracle, int threads, int iters, std::atomic<int>* errors) {
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) {
    ts.emplace_back([=] {
      for (int i = 0; i < iters; ++i) {
        std::vector<uint64_t> nodes;
        for (int k = 0; k < 16; ++k) nodes.push_back(static_cast<uint64_t>((t * 7919 + i * 104729 + k * 31) % 5000));
        std::vector<Tensor> r;
        Status st = qp->Run("v(nodes).sampleNB(edge_types, nb_count, -1).as(nb)", NbInputs(nodes, 5),
                            {"nb:0", "nb:1"}, &r);
        if (!st.ok() || r.size() != 2 || r[1].numel() != 16 * 5) {
          errors->fetch_add(1);
          continue;
        }
        std::vector<Tensor> a, b;
        Status s1 = qp->Run("v(nodes).outV(edge_types).as(nb)", NbInputs(nodes, 0), {"nb:0", "nb:1"}, &a);
        Status s2 = oracle->Run("v(nodes).outV(edge_types).as(nb)", NbInputs(nodes, 0), {"nb:0", "nb:1"}, &b);
        if (!s1.ok() || !s2.ok() || a.size() != 2 || b.size() != 2 || a[1].numel() != b[1].numel()) {
          errors->fetch_add(1);
          continue;
        }
        const uint64_t* x = a[1].data<uint64_t>();
        const uint64_t* y = b[1].data<uint64_t>();
        for (int64_t k = 0; k < a[1].numel(); ++k)
          if (x[k] != y[k]) {
            errors->fetch_add(1);
            break;
          }
      }
    });
  }
  for (auto& th : ts) th.join();
}

}  // namespace

int main(int argc, char** argv) {
  LinkGraphOps();
  LinkDistOps();
  LinkRemoteOp();
  const int threads = argc > 1 ? std::atoi(argv[1]) : 8;
  const int iters = argc > 2 ? std::atoi(argv[2]) : 50;

  // local engine over a synthetic graph
  QueryProxy local;
  Expect(local.InitWithGraph(SyntheticGraph(5000, 6.0, 64, 1, 1, 8, 0, 7, false), nullptr).ok(), "local init");

  // one graph server (shard 0 of 1) + a remote client through the in-memory registry
  std::unique_ptr<Graph> served = SyntheticGraph(5000, 6.0, 64, 1, 1, 8, 0, 7, false);
  std::unique_ptr<EngineEnv> env = QueryProxy::MakeEnv(served.get(), nullptr, 1);
  ServerOptions so;
  so.num_threads = 8;
  so.registry = "memory:selftest";
  GraphServer server(env.get(), 0, 1, so);
  Expect(server.Start().ok(), "server start");
  QueryProxy remote;
  Expect(remote.Init({{"mode", "remote"}, {"registry", "memory:selftest"}, {"shard_num", "1"}}).ok(), "remote init");

  std::atomic<int> errors{0};
  Hammer(&local, &local, threads, iters, &errors);
  Hammer(&remote, &local, threads, iters, &errors);
  Expect(errors.load() == 0, "concurrent queries");
  Expect(EngineCounters::Get().queries.load() > 0, "counters");
  Expect(EngineCounters::Get().remote_calls.load() > 0, "remote fan-out counted");
  server.Stop();
  if (g_failures == 0) std::printf("engine_selftest OK (%d threads x %d iterations)\n", threads, iters);
  return g_failures == 0 ? 0 : 1;
}
