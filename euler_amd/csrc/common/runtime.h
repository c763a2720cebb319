// euler_amd engine — concurrency, randomness, weighted samplers, file IO.
// Reference counterparts: N1 env/thread pool (env_posix.cc:98-159),
// N2 sync primitives, N5 file IO (file_io.h, hdfs via dlopen), N6 weighted samplers
// (alias_method.cc, compact_weighted_collection.h) and random.cc.
//
// Differences by design:
//  * one shared work queue + ParallelFor with chunking (no per-thread round-robin
//    queues that stall behind a long job);
//  * counter-based Philox RNG: every draw is f(global seed, stream, counter), so
//    sampling is reproducible per (seed, thread) instead of time(0)-seeded
//    thread-locals (reference random.cc:21-24 defect);
//  * file IO reads whole files through mmap.
#pragma once

#include <stdint.h>

#include <atomic>
#include <map>
#include <condition_variable>
#include <deque>
#include <functional>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "common/common.h"

namespace euler {

// ---------------------------------------------------------------- thread pool
class ThreadPool {
 public:
  explicit ThreadPool(int n, const std::string& name = "euler");
  ~ThreadPool();
  void Schedule(std::function<void()> fn);
  int size() const { return static_cast<int>(workers_.size()); }
  // run fn(begin, end) over [0, n) in chunks on the pool and the caller; blocks.
  void ParallelFor(int64_t n, int64_t min_chunk, const std::function<void(int64_t, int64_t)>& fn);
  static ThreadPool* Default();

 private:
  void Loop();
  std::vector<std::thread> workers_;
  std::deque<std::function<void()>> q_;
  std::mutex mu_;
  std::condition_variable cv_;
  bool stop_ = false;
};

// counts down to zero then releases waiters (reference common/signal.h)
class Latch {
 public:
  explicit Latch(int64_t n) : n_(n) {}
  void CountDown() {
    std::lock_guard<std::mutex> l(mu_);
    if (--n_ == 0) cv_.notify_all();
  }
  void Wait() {
    std::unique_lock<std::mutex> l(mu_);
    cv_.wait(l, [&] { return n_ <= 0; });
  }

 private:
  int64_t n_;
  std::mutex mu_;
  std::condition_variable cv_;
};

// ---------------------------------------------------------------- randomness
struct Philox4x32 {
  static void Gen(uint64_t key, uint64_t ctr_hi, uint64_t ctr_lo, uint32_t out[4]);
};

// A cheap per-thread stream: (seed, stream id, counter) -> Philox words.
class Rng {
 public:
  Rng(uint64_t seed, uint64_t stream) : seed_(seed), stream_(stream) {}
  uint32_t NextU32();
  uint64_t NextU64() { return (static_cast<uint64_t>(NextU32()) << 32) | NextU32(); }
  float Uniform() { return (NextU32() >> 8) * (1.0f / 16777216.0f); }        // [0,1)
  double UniformD() { return (NextU64() >> 11) * (1.0 / 9007199254740992.0); }  // [0,1)
  uint64_t Below(uint64_t n);  // uniform in [0, n)

 private:
  uint64_t seed_, stream_, ctr_ = 0;
  uint32_t buf_[4];
  int left_ = 0;
};

void SetGlobalSeed(uint64_t seed);
uint64_t GlobalSeed();
// Per-call RNG stream counter of the sampling ops; SetGlobalSeed restarts it, so a
// sequence of calls after set_seed(s) draws the same streams in every process.
uint64_t NextOpEpoch();
// thread-local Rng keyed by (global seed, thread ordinal); re-keyed when the seed changes
Rng& ThreadRng();

// ---------------------------------------------------------------- weighted samplers
// Walker/Vose alias table: O(n) build, O(1) draw.
class AliasTable {
 public:
  AliasTable() = default;
  explicit AliasTable(const std::vector<float>& w) { Init(w.data(), w.size()); }
  void Init(const float* w, size_t n);
  void Init(const double* w, size_t n);
  int64_t Sample(Rng& r) const;
  size_t size() const { return prob_.size(); }
  double total() const { return total_; }
  bool empty() const { return prob_.empty(); }

 private:
  template <typename T>
  void InitT(const T* w, size_t n);
  std::vector<float> prob_;
  std::vector<int64_t> alias_;
  double total_ = 0;
};

// binary search on inclusive prefix sums cumw[lo..hi): first index with cumw > u
inline int64_t PrefixPick(const float* cumw, int64_t lo, int64_t hi, float u) {
  int64_t a = lo, b = hi - 1;
  while (a < b) {
    const int64_t m = (a + b) >> 1;
    if (cumw[m] > u) b = m; else a = m + 1;
  }
  return a;
}

// ---------------------------------------------------------------- file IO
// Read-only file view; local files are mmapped, "hdfs://" / "viewfs://" go through
// libhdfs loaded with dlopen when present (reference hdfs_file_io.cc:83).
class FileView {
 public:
  static Status Open(const std::string& path, std::unique_ptr<FileView>* out);
  ~FileView();
  const char* data() const { return data_; }
  size_t size() const { return size_; }

 private:
  const char* data_ = nullptr;
  size_t size_ = 0;
  bool mmapped_ = false;
  std::string owned_;
};

Status ListDir(const std::string& path, std::vector<std::string>* names);
bool FileExists(const std::string& path);
Status WriteFile(const std::string& path, const std::string& content);
Status MakeDirs(const std::string& path);

// ============================================================================ observability
// Process-wide per-stage counters of the engine (query compile / execute, DAG nodes,
// remote fan-out, RPC attempts / failures / bytes, server requests), exported to
// Python as _engine.stats().  Relaxed atomics: cheap enough to stay always on.
struct EngineCounters {
  std::atomic<int64_t> queries{0}, compile_us{0}, exec_us{0}, dag_nodes{0};
  std::atomic<int64_t> remote_calls{0}, rpc_attempts{0}, rpc_failures{0}, rpc_bytes_out{0}, rpc_bytes_in{0};
  std::atomic<int64_t> server_requests{0}, server_us{0};
  std::atomic<int64_t> local_connections{0}, tcp_connections{0};  // client transports
  std::atomic<int64_t> shm_channels{0}, shm_bytes{0};  // same-host shared-memory payloads (both sides)
  static EngineCounters& Get();
  void Reset();
};

// Opt-in per-op kernel profile (EULER_OP_PROFILE=1 or SetOpProfile(true)): wall
// microseconds and calls by op name, both sides of the RPC (server DAGs included).
// Async kernels (REMOTE) are timed from launch to completion callback.
bool OpProfileEnabled();
void SetOpProfile(bool on);
void OpProfileAdd(const std::string& op, int64_t us);
std::map<std::string, std::pair<int64_t, int64_t>> OpProfileSnapshot();  // op -> (us, calls)
void OpProfileReset();

// adds the elapsed microseconds to a counter when it goes out of scope
class ScopedMicros {
 public:
  explicit ScopedMicros(std::atomic<int64_t>* c) : c_(c), t0_(NowMicros()) {}
  ~ScopedMicros() { c_->fetch_add(static_cast<int64_t>(NowMicros() - t0_), std::memory_order_relaxed); }

 private:
  std::atomic<int64_t>* c_;
  uint64_t t0_;
};

}  // namespace euler
