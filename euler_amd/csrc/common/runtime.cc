#include "common/runtime.h"

#include <dirent.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cmath>
#include <fstream>

namespace euler {

// ---------------------------------------------------------------- thread pool
ThreadPool::ThreadPool(int n, const std::string&) {
  if (n <= 0) n = 1;
  for (int i = 0; i < n; ++i) workers_.emplace_back([this] { Loop(); });
}

ThreadPool::~ThreadPool() {
  {
    std::lock_guard<std::mutex> l(mu_);
    stop_ = true;
  }
  cv_.notify_all();
  for (auto& t : workers_) t.join();
}

void ThreadPool::Schedule(std::function<void()> fn) {
  {
    std::lock_guard<std::mutex> l(mu_);
    q_.push_back(std::move(fn));
  }
  cv_.notify_one();
}

void ThreadPool::Loop() {
  for (;;) {
    std::function<void()> fn;
    {
      std::unique_lock<std::mutex> l(mu_);
      cv_.wait(l, [&] { return stop_ || !q_.empty(); });
      if (stop_ && q_.empty()) return;
      fn = std::move(q_.front());
      q_.pop_front();
    }
    fn();
  }
}

void ThreadPool::ParallelFor(int64_t n, int64_t min_chunk, const std::function<void(int64_t, int64_t)>& fn) {
  if (n <= 0) return;
  const int64_t workers = size() + 1;
  int64_t chunk = std::max<int64_t>(min_chunk, (n + workers * 4 - 1) / (workers * 4));
  const int64_t nchunks = (n + chunk - 1) / chunk;
  if (nchunks <= 1) {
    fn(0, n);
    return;
  }
  // shared state: a helper that starts after the loop finished only touches `next`
  struct State {
    std::atomic<int64_t> next{0};
    Latch done;
    explicit State(int64_t k) : done(k) {}
  };
  auto st = std::make_shared<State>(nchunks);
  const std::function<void(int64_t, int64_t)>* fnp = &fn;
  auto worker = [st, fnp, nchunks, chunk, n] {
    for (;;) {
      const int64_t c = st->next.fetch_add(1);
      if (c >= nchunks) return;
      const int64_t b = c * chunk, e = std::min(n, b + chunk);
      (*fnp)(b, e);  // fn outlives every claimed chunk: the caller waits on `done`
      st->done.CountDown();
    }
  };
  const int64_t helpers = std::min<int64_t>(size(), nchunks - 1);
  for (int64_t i = 0; i < helpers; ++i) Schedule(worker);
  worker();
  st->done.Wait();
}

ThreadPool* ThreadPool::Default() {
  static ThreadPool* pool = [] {
    int n = static_cast<int>(std::thread::hardware_concurrency());
    if (const char* e = getenv("EULER_NUM_THREADS")) n = atoi(e);
    if (n <= 0) n = 8;
    n = std::min(n, 64);
    return new ThreadPool(n, "euler-default");
  }();
  return pool;
}

// ---------------------------------------------------------------- Philox
void Philox4x32::Gen(uint64_t key, uint64_t hi, uint64_t lo, uint32_t out[4]) {
  uint32_t c0 = static_cast<uint32_t>(lo), c1 = static_cast<uint32_t>(lo >> 32);
  uint32_t c2 = static_cast<uint32_t>(hi), c3 = static_cast<uint32_t>(hi >> 32);
  uint32_t k0 = static_cast<uint32_t>(key), k1 = static_cast<uint32_t>(key >> 32);
  for (int r = 0; r < 10; ++r) {
    const uint64_t p0 = static_cast<uint64_t>(0xD2511F53u) * c0;
    const uint64_t p1 = static_cast<uint64_t>(0xCD9E8D57u) * c2;
    const uint32_t n0 = static_cast<uint32_t>(p1 >> 32) ^ c1 ^ k0;
    const uint32_t n1 = static_cast<uint32_t>(p1);
    const uint32_t n2 = static_cast<uint32_t>(p0 >> 32) ^ c3 ^ k1;
    const uint32_t n3 = static_cast<uint32_t>(p0);
    c0 = n0; c1 = n1; c2 = n2; c3 = n3;
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

uint32_t Rng::NextU32() {
  if (left_ == 0) {
    Philox4x32::Gen(seed_, stream_, ctr_++, buf_);
    left_ = 4;
  }
  return buf_[--left_];
}

uint64_t Rng::Below(uint64_t n) {
  if (n <= 1) return 0;
  const unsigned __int128 m = static_cast<unsigned __int128>(NextU64()) * n;
  return static_cast<uint64_t>(m >> 64);
}

static std::atomic<uint64_t> g_seed{0x5eed5eedULL};
static std::atomic<uint64_t> g_epoch{1};
static std::atomic<uint64_t> g_op_epoch{1};
static std::atomic<uint64_t> g_thread_ordinal{0};

void SetGlobalSeed(uint64_t seed) {
  g_seed.store(seed);
  g_op_epoch.store(1);
  g_epoch.fetch_add(1);
}
uint64_t NextOpEpoch() { return g_op_epoch.fetch_add(1); }
uint64_t GlobalSeed() { return g_seed.load(); }

Rng& ThreadRng() {
  thread_local uint64_t ordinal = g_thread_ordinal.fetch_add(1);
  thread_local uint64_t epoch = 0;
  thread_local std::unique_ptr<Rng> rng;
  const uint64_t e = g_epoch.load(std::memory_order_relaxed);
  if (!rng || epoch != e) {
    rng.reset(new Rng(g_seed.load(), (ordinal << 20) ^ 0xA5A5ULL));
    epoch = e;
  }
  return *rng;
}

// ---------------------------------------------------------------- alias table
template <typename T>
void AliasTable::InitT(const T* w, size_t n) {
  prob_.assign(n, 1.f);
  alias_.resize(n);
  total_ = 0;
  for (size_t i = 0; i < n; ++i) total_ += std::max<double>(0.0, static_cast<double>(w[i]));
  for (size_t i = 0; i < n; ++i) alias_[i] = static_cast<int64_t>(i);
  if (n == 0 || total_ <= 0) return;
  std::vector<double> p(n);
  std::vector<int64_t> small, large;
  small.reserve(n);
  large.reserve(n);
  for (size_t i = 0; i < n; ++i) {
    p[i] = std::max<double>(0.0, static_cast<double>(w[i])) * n / total_;
    (p[i] < 1.0 ? small : large).push_back(static_cast<int64_t>(i));
  }
  while (!small.empty() && !large.empty()) {
    const int64_t s = small.back();
    small.pop_back();
    const int64_t l = large.back();
    prob_[s] = static_cast<float>(p[s]);
    alias_[s] = l;
    p[l] -= (1.0 - p[s]);
    if (p[l] < 1.0) {
      large.pop_back();
      small.push_back(l);
    }
  }
  for (int64_t i : small) prob_[i] = 1.f;
  for (int64_t i : large) prob_[i] = 1.f;
}

void AliasTable::Init(const float* w, size_t n) { InitT(w, n); }
void AliasTable::Init(const double* w, size_t n) { InitT(w, n); }

int64_t AliasTable::Sample(Rng& r) const {
  const uint64_t k = r.Below(prob_.size());
  return r.Uniform() < prob_[k] ? static_cast<int64_t>(k) : alias_[k];
}

// ---------------------------------------------------------------- file IO
namespace {
// minimal libhdfs surface (loaded lazily; absent on most hosts)
struct Hdfs {
  void* lib = nullptr;
  void* (*connect)(const char*, uint16_t) = nullptr;
  void* (*open)(void*, const char*, int, int, short, int32_t) = nullptr;
  int32_t (*read)(void*, void*, void*, int32_t) = nullptr;
  int (*close)(void*, void*) = nullptr;
  bool Load() {
    if (lib) return true;
    const char* names[] = {"libhdfs.so", "libhdfs.so.0.0.0"};
    for (auto n : names) {
      lib = dlopen(n, RTLD_NOW);
      if (lib) break;
    }
    if (!lib) return false;
    connect = reinterpret_cast<decltype(connect)>(dlsym(lib, "hdfsConnect"));
    open = reinterpret_cast<decltype(open)>(dlsym(lib, "hdfsOpenFile"));
    read = reinterpret_cast<decltype(read)>(dlsym(lib, "hdfsRead"));
    close = reinterpret_cast<decltype(close)>(dlsym(lib, "hdfsCloseFile"));
    return connect && open && read && close;
  }
};
}  // namespace

Status FileView::Open(const std::string& path, std::unique_ptr<FileView>* out) {
  std::unique_ptr<FileView> fv(new FileView);
  if (StartsWith(path, "hdfs://") || StartsWith(path, "viewfs://")) {
    static Hdfs hdfs;
    if (!hdfs.Load()) return Status::Unavailable("libhdfs not available for " + path);
    void* fs = hdfs.connect("default", 0);
    if (!fs) return Status::Unavailable("hdfsConnect failed");
    void* f = hdfs.open(fs, path.c_str(), O_RDONLY, 0, 0, 0);
    if (!f) return Status::NotFound(path);
    char buf[1 << 16];
    for (;;) {
      int32_t n = hdfs.read(fs, f, buf, sizeof(buf));
      if (n <= 0) break;
      fv->owned_.append(buf, n);
    }
    hdfs.close(fs, f);
    fv->data_ = fv->owned_.data();
    fv->size_ = fv->owned_.size();
    *out = std::move(fv);
    return Status::OK();
  }
  std::string p = StartsWith(path, "file://") ? path.substr(7) : path;
  int fd = ::open(p.c_str(), O_RDONLY);
  if (fd < 0) return Status::NotFound("cannot open " + p + ": " + strerror(errno));
  struct stat st;
  if (fstat(fd, &st) != 0) {
    ::close(fd);
    return Status::Internal("fstat failed: " + p);
  }
  fv->size_ = static_cast<size_t>(st.st_size);
  if (fv->size_ > 0) {
    void* m = mmap(nullptr, fv->size_, PROT_READ, MAP_PRIVATE, fd, 0);
    if (m == MAP_FAILED) {
      ::close(fd);
      return Status::Internal("mmap failed: " + p);
    }
    madvise(m, fv->size_, MADV_SEQUENTIAL);
    fv->data_ = static_cast<const char*>(m);
    fv->mmapped_ = true;
  }
  ::close(fd);
  *out = std::move(fv);
  return Status::OK();
}

FileView::~FileView() {
  if (mmapped_ && data_) munmap(const_cast<char*>(data_), size_);
}

Status ListDir(const std::string& path, std::vector<std::string>* names) {
  names->clear();
  DIR* d = opendir(path.c_str());
  if (!d) return Status::NotFound("cannot list " + path);
  while (struct dirent* e = readdir(d)) {
    std::string n = e->d_name;
    if (n == "." || n == "..") continue;
    names->push_back(n);
  }
  closedir(d);
  std::sort(names->begin(), names->end());
  return Status::OK();
}

bool FileExists(const std::string& path) {
  struct stat st;
  return stat(path.c_str(), &st) == 0;
}

Status WriteFile(const std::string& path, const std::string& content) {
  std::ofstream f(path, std::ios::binary);
  if (!f) return Status::Internal("cannot write " + path);
  f.write(content.data(), content.size());
  return f ? Status::OK() : Status::Internal("write failed " + path);
}

Status MakeDirs(const std::string& path) {
  std::string cur;
  for (auto& part : Split(path, "/")) {
    cur += (cur.empty() && path[0] != '/') ? part : "/" + part;
    if (!FileExists(cur) && mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST)
      return Status::Internal("mkdir failed " + cur);
  }
  return Status::OK();
}

}  // namespace euler

namespace euler {

EngineCounters& EngineCounters::Get() {
  static EngineCounters c;
  return c;
}

void EngineCounters::Reset() {
  for (auto* a : {&queries, &compile_us, &exec_us, &dag_nodes, &remote_calls, &rpc_attempts, &rpc_failures,
                  &rpc_bytes_out, &rpc_bytes_in, &server_requests, &server_us, &local_connections, &tcp_connections,
                  &shm_channels, &shm_bytes})
    a->store(0);
}

namespace {
std::atomic<int> g_op_profile{-1};
std::mutex g_op_prof_mu;
std::map<std::string, std::pair<int64_t, int64_t>> g_op_prof;
}  // namespace

bool OpProfileEnabled() {
  int v = g_op_profile.load(std::memory_order_relaxed);
  if (v < 0) {
    const char* e = getenv("EULER_OP_PROFILE");
    v = (e && atoi(e) != 0) ? 1 : 0;
    g_op_profile.store(v, std::memory_order_relaxed);
  }
  return v == 1;
}
void SetOpProfile(bool on) { g_op_profile.store(on ? 1 : 0, std::memory_order_relaxed); }
void OpProfileAdd(const std::string& op, int64_t us) {
  std::lock_guard<std::mutex> l(g_op_prof_mu);
  auto& e = g_op_prof[op];
  e.first += us;
  e.second += 1;
}
std::map<std::string, std::pair<int64_t, int64_t>> OpProfileSnapshot() {
  std::lock_guard<std::mutex> l(g_op_prof_mu);
  return g_op_prof;
}
void OpProfileReset() {
  std::lock_guard<std::mutex> l(g_op_prof_mu);
  g_op_prof.clear();
}

}  // namespace euler
