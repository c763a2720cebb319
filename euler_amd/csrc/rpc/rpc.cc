#include "rpc/rpc.h"

#include <future>

#include <arpa/inet.h>
#include <errno.h>
#include <netdb.h>
#include <netinet/in.h>
#include <netinet/tcp.h>
#include <sys/epoll.h>
#include <sys/eventfd.h>
#include <sys/mman.h>
#include <sys/syscall.h>
#include <sys/socket.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <sys/un.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <chrono>
#include <deque>
#include <set>
#include <unordered_map>

namespace euler {

namespace {
constexpr uint32_t kMagic = 0x524C5545;  // "EULR"
enum : uint32_t { kPing = 1, kExecute = 2, kMeta = 3, kRegPut = 10, kRegBeat = 11, kRegDel = 12, kRegList = 13,
                  kShmAttach = 20, kReply = 100 };
// Same-host shared-memory payloads: a frame whose kind carries kShmFlag has an 8-byte
// payload = the length of the real payload, which sits at offset 0 of the connection's
// shared region (one request per connection is in flight, so request and reply take turns).
constexpr uint32_t kShmFlag = 0x1000;
constexpr size_t kShmMin = 64 << 10;  // smaller payloads stay in-band
constexpr unsigned int MFD_CLOEXEC_FLAG = 1U;  // MFD_CLOEXEC

size_t ShmCapacity() {
  const char* e = std::getenv("EULER_RPC_SHM_MB");
  const long mb = e ? std::atol(e) : 64;
  return static_cast<size_t>(mb > 0 ? mb : 0) << 20;
}

std::string EncodeLen(uint64_t n) { return std::string(reinterpret_cast<const char*>(&n), 8); }
uint64_t DecodeLen(const std::string& s) {
  uint64_t n = 0;
  if (s.size() == 8) memcpy(&n, s.data(), 8);
  return n;
}

// wall clock (file mtimes of the registry are wall-clock stamps)
double WallSec() {
  return std::chrono::duration<double>(std::chrono::system_clock::now().time_since_epoch()).count();
}

double NowSec() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

bool WriteAll(int fd, const void* p, size_t n) {
  const char* c = static_cast<const char*>(p);
  while (n > 0) {
    ssize_t k = ::send(fd, c, n, MSG_NOSIGNAL);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

bool ReadAll(int fd, void* p, size_t n) {
  char* c = static_cast<char*>(p);
  while (n > 0) {
    ssize_t k = ::recv(fd, c, n, 0);
    if (k < 0 && errno == EINTR) continue;
    if (k <= 0) return false;
    c += k;
    n -= static_cast<size_t>(k);
  }
  return true;
}

bool SendFrame(int fd, uint32_t kind, const std::string& payload) {
  char hdr[16];
  const uint64_t len = payload.size();
  memcpy(hdr, &kMagic, 4);
  memcpy(hdr + 4, &kind, 4);
  memcpy(hdr + 8, &len, 8);
  return WriteAll(fd, hdr, 16) && WriteAll(fd, payload.data(), payload.size());
}

bool RecvFrame(int fd, uint32_t* kind, std::string* payload) {
  char hdr[16];
  if (!ReadAll(fd, hdr, 16)) return false;
  uint32_t magic;
  uint64_t len;
  memcpy(&magic, hdr, 4);
  memcpy(kind, hdr + 4, 4);
  memcpy(&len, hdr + 8, 8);
  if (magic != kMagic || len > (1ULL << 36)) return false;
  payload->resize(len);
  return len == 0 || ReadAll(fd, &(*payload)[0], len);
}

// attach frame: kShmAttach with payload = region size; the memfd travels as SCM_RIGHTS
bool SendAttach(int fd, int memfd, uint64_t size) {
  char hdr[16 + 8];
  const uint32_t kind = kShmAttach;
  const uint64_t len = 8;
  memcpy(hdr, &kMagic, 4);
  memcpy(hdr + 4, &kind, 4);
  memcpy(hdr + 8, &len, 8);
  memcpy(hdr + 16, &size, 8);
  struct iovec iov;
  iov.iov_base = hdr;
  iov.iov_len = sizeof(hdr);
  char ctrl[CMSG_SPACE(sizeof(int))];
  memset(ctrl, 0, sizeof(ctrl));
  struct msghdr msg;
  memset(&msg, 0, sizeof(msg));
  msg.msg_iov = &iov;
  msg.msg_iovlen = 1;
  msg.msg_control = ctrl;
  msg.msg_controllen = sizeof(ctrl);
  struct cmsghdr* cm = CMSG_FIRSTHDR(&msg);
  cm->cmsg_level = SOL_SOCKET;
  cm->cmsg_type = SCM_RIGHTS;
  cm->cmsg_len = CMSG_LEN(sizeof(int));
  memcpy(CMSG_DATA(cm), &memfd, sizeof(int));
  for (;;) {
    const ssize_t k = ::sendmsg(fd, &msg, MSG_NOSIGNAL);
    if (k == static_cast<ssize_t>(sizeof(hdr))) return true;
    if (k < 0 && errno == EINTR) continue;
    return false;  // a short write of 24 bytes on a fresh Unix socket does not happen
  }
}

// Same-host transport: servers also listen on an abstract-namespace Unix socket named after
// their TCP port, so a client on the same host skips the TCP/IP stack ("a
// shared-memory / local transport when client and shards are on one host").  Disabled
// with EULER_RPC_TRANSPORT=tcp.
std::string LocalSocketName(int port) { return std::string("euler_amd_rpc_") + std::to_string(port); }

bool LocalTransportEnabled() {
  const char* t = std::getenv("EULER_RPC_TRANSPORT");
  return t == nullptr || std::string(t) != "tcp";
}

bool IsLocalHost(const std::string& host) {
  if (host == "127.0.0.1" || host == "localhost" || host == "::1") return true;
  char name[256] = {0};
  return gethostname(name, sizeof(name) - 1) == 0 && host == name;
}

socklen_t AbstractAddr(int port, struct sockaddr_un* addr) {
  memset(addr, 0, sizeof(*addr));
  addr->sun_family = AF_UNIX;
  const std::string name = LocalSocketName(port);
  memcpy(addr->sun_path + 1, name.data(), name.size());  // sun_path[0] = 0: abstract namespace
  return static_cast<socklen_t>(offsetof(struct sockaddr_un, sun_path) + 1 + name.size());
}

void SetTimeouts(int fd, int timeout_ms) {
  struct timeval tv;
  tv.tv_sec = timeout_ms / 1000;
  tv.tv_usec = (timeout_ms % 1000) * 1000;
  setsockopt(fd, SOL_SOCKET, SO_RCVTIMEO, &tv, sizeof(tv));
  setsockopt(fd, SOL_SOCKET, SO_SNDTIMEO, &tv, sizeof(tv));
}

int ConnectLocal(const Endpoint& ep, int timeout_ms) {
  int fd = socket(AF_UNIX, SOCK_STREAM, 0);
  if (fd < 0) return -1;
  struct sockaddr_un addr;
  const socklen_t len = AbstractAddr(ep.port, &addr);
  SetTimeouts(fd, timeout_ms);
  if (connect(fd, reinterpret_cast<sockaddr*>(&addr), len) != 0) {
    close(fd);
    return -1;
  }
  return fd;
}

int Connect(const Endpoint& ep, int timeout_ms) {
  if (LocalTransportEnabled() && IsLocalHost(ep.host)) {
    const int fd = ConnectLocal(ep, timeout_ms);
    if (fd >= 0) {
      EngineCounters::Get().local_connections.fetch_add(1, std::memory_order_relaxed);
      return fd;
    }
  }
  struct addrinfo hints, *res = nullptr;
  memset(&hints, 0, sizeof(hints));
  hints.ai_family = AF_INET;
  hints.ai_socktype = SOCK_STREAM;
  if (getaddrinfo(ep.host.c_str(), std::to_string(ep.port).c_str(), &hints, &res) != 0 || !res) return -1;
  int fd = socket(res->ai_family, res->ai_socktype, res->ai_protocol);
  if (fd < 0) {
    freeaddrinfo(res);
    return -1;
  }
  int one = 1;
  setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));
  SetTimeouts(fd, timeout_ms);
  if (connect(fd, res->ai_addr, res->ai_addrlen) != 0) {
    close(fd);
    freeaddrinfo(res);
    return -1;
  }
  freeaddrinfo(res);
  EngineCounters::Get().tcp_connections.fetch_add(1, std::memory_order_relaxed);
  return fd;
}

std::string EncodeExecute(const DAGDef& dag, const std::vector<std::pair<std::string, Tensor>>& inputs,
                          const std::vector<std::string>& outputs) {
  BytesWriter w;
  w.Write(dag.Serialize());
  w.Write<uint32_t>(static_cast<uint32_t>(inputs.size()));
  for (auto& kv : inputs) {
    w.Write(kv.first);
    kv.second.Encode(&w);
  }
  w.Write<uint32_t>(static_cast<uint32_t>(outputs.size()));
  for (auto& o : outputs) w.Write(o);
  return w.str();
}

bool DecodeExecute(const std::string& p, DAGDef* dag, std::vector<std::pair<std::string, Tensor>>* inputs,
                   std::vector<std::string>* outputs) {
  BytesReader r(p.data(), p.size());
  std::string d;
  uint32_t n;
  if (!r.Read(&d) || !DAGDef::Parse(d.data(), d.size(), dag) || !r.Read(&n)) return false;
  inputs->resize(n);
  for (auto& kv : *inputs)
    if (!r.Read(&kv.first) || !Tensor::Decode(&r, &kv.second)) return false;
  if (!r.Read(&n)) return false;
  outputs->resize(n);
  for (auto& o : *outputs)
    if (!r.Read(&o)) return false;
  return true;
}

size_t ReplySize(const Status& st, const std::vector<Tensor>& ts) {
  size_t n = 4 + 4 + st.message().size() + 4;
  for (auto& t : ts) n += t.EncodedSize();
  return n;
}

void EncodeReplyTo(BytesWriter* w, const Status& st, const std::vector<Tensor>& ts) {
  w->Write<int32_t>(static_cast<int32_t>(st.code()));
  w->Write(st.message());
  w->Write<uint32_t>(static_cast<uint32_t>(ts.size()));
  for (auto& t : ts) t.Encode(w);
}

std::string EncodeReply(const Status& st, const std::vector<Tensor>& ts) {
  BytesWriter w;
  w.str().reserve(ReplySize(st, ts));
  EncodeReplyTo(&w, st, ts);
  return std::move(w.str());
}

// false = malformed bytes (a transport failure); *app = the server's own status
bool ParseReply(const char* data, size_t size, Status* app, std::vector<Tensor>* ts) {
  BytesReader r(data, size);
  int32_t code;
  std::string msg;
  uint32_t n;
  if (!r.Read(&code) || !r.Read(&msg) || !r.Read(&n)) return false;
  *app = code != 0 ? Status(static_cast<Code>(code), msg) : Status::OK();
  if (code != 0) return true;
  ts->resize(n);
  for (auto& t : *ts)
    if (!Tensor::Decode(&r, &t)) return false;
  return true;
}

Status DecodeReply(const char* data, size_t size, std::vector<Tensor>* ts) {
  Status app;
  if (!ParseReply(data, size, &app, ts)) return Status::RpcError("malformed reply");
  return app;
}
Status DecodeReply(const std::string& p, std::vector<Tensor>* ts) { return DecodeReply(p.data(), p.size(), ts); }

double FaultRate() {
  static double r = [] {
    const char* e = getenv("EULER_RPC_FAULT_RATE");
    return e ? atof(e) : 0.0;
  }();
  return r;
}
int FaultDelayMs() {
  static int d = [] {
    const char* e = getenv("EULER_RPC_FAULT_DELAY_MS");
    return e ? atoi(e) : 0;
  }();
  return d;
}
}  // namespace

// ============================================================================ execution
Status ExecuteDag(EngineEnv* env, const DAGDef& dag, const std::vector<std::pair<std::string, Tensor>>& inputs,
                  const std::vector<std::string>& outputs, std::vector<Tensor>* results) {
  OpContext ctx(env);
  for (auto& kv : inputs) ctx.Set(kv.first, kv.second);
  Executor ex(dag, &ctx, ThreadPool::Default());
  EULER_RETURN_IF_ERROR(ex.Run());
  results->clear();
  for (auto& o : outputs) {
    Tensor t;
    if (!ctx.TryGet(o, &t)) return Status::NotFound("output '" + o + "' was not produced");
    results->push_back(t);
  }
  return Status::OK();
}

void InProcessShards::Execute(int shard, const DAGDef& dag, std::vector<std::pair<std::string, Tensor>> inputs,
                              std::vector<std::string> outputs, Done done) {
  if (shard < 0 || shard >= num_shards()) {
    done(Status::InvalidArgument("bad shard index"), {});
    return;
  }
  // shards run concurrently on their own pool, like separate servers would
  static ThreadPool* pool = new ThreadPool(16, "euler-inproc-shards");
  EngineEnv* env = envs_[shard];
  auto dagp = std::make_shared<DAGDef>(dag);
  pool->Schedule([env, dagp, inputs, outputs, done] {
    std::vector<Tensor> res;
    Status st;
    try {
      st = ExecuteDag(env, *dagp, inputs, outputs, &res);
    } catch (const std::exception& e) {
      st = Status::Internal(e.what());
    }
    done(st, std::move(res));
  });
}

// ============================================================================ REMOTE kernel
namespace {
class RemoteOp : public OpKernel {
 public:
  bool is_async() const override { return true; }
  void Compute(const NodeDef&, OpContext*) override { EULER_THROW("REMOTE is asynchronous"); }
  void ComputeAsync(const NodeDef& nd, OpContext* ctx, std::function<void(Status)> done) override {
    RemoteClients* rc = ctx->env() ? ctx->env()->clients : nullptr;
    if (!rc) {
      done(Status::Unavailable("REMOTE node but no remote clients configured"));
      return;
    }
    EngineCounters::Get().remote_calls.fetch_add(1, std::memory_order_relaxed);
    // ship every client tensor the sub-DAG references (inputs, attrs, DNF values)
    std::set<std::string> produced;
    for (auto& n : nd.inner)
      for (int k = 0; k < std::max(1, n.output_num); ++k) produced.insert(n.Output(k));
    std::set<std::string> names;
    auto consider = [&](const std::string& s) {
      if (!produced.count(s) && ctx->Has(s)) names.insert(s);
    };
    for (auto& n : nd.inner) {
      for (auto& s : n.inputs) consider(s);
      for (auto& s : n.attrs) consider(s);
      for (auto& conj : n.dnf)
        for (auto& term : Split(conj, ","))
          for (auto& tok : Split(term, " ")) consider(Trim(tok));
    }
    std::vector<std::pair<std::string, Tensor>> inputs;
    for (auto& s : names) inputs.emplace_back(s, ctx->Get(s));
    DAGDef sub;
    sub.nodes = nd.inner;
    const std::string me = nd.name();
    const int on = nd.output_num;
    rc->Execute(nd.shard_idx, sub, std::move(inputs), nd.output_list,
                [ctx, me, on, done](Status st, std::vector<Tensor> res) {
                  if (st.ok()) {
                    for (int k = 0; k < on && k < static_cast<int>(res.size()); ++k)
                      ctx->Set(me + ":" + std::to_string(k), std::move(res[k]));
                  }
                  done(st);
                });
  }
};
}  // namespace
REGISTER_OP_KERNEL("REMOTE", RemoteOp);
void LinkRemoteOp() {}

// ============================================================================ ShardMeta
static std::string HexEncode(const std::string& s) {
  static const char* d = "0123456789abcdef";
  std::string o;
  o.reserve(s.size() * 2);
  for (unsigned char c : s) {
    o.push_back(d[c >> 4]);
    o.push_back(d[c & 15]);
  }
  return o;
}
static std::string HexDecode(const std::string& s) {
  std::string o;
  auto v = [](char c) { return c <= '9' ? c - '0' : c - 'a' + 10; };
  for (size_t i = 0; i + 1 < s.size(); i += 2) o.push_back(static_cast<char>((v(s[i]) << 4) | v(s[i + 1])));
  return o;
}
static std::string JoinD(const std::vector<double>& v) {
  std::vector<std::string> s;
  for (double x : v) {
    std::ostringstream os;
    os.precision(17);
    os << x;
    s.push_back(os.str());
  }
  return Join(s, ",");
}
static std::vector<double> SplitD(const std::string& s) {
  std::vector<double> v;
  for (auto& p : Split(s, ",")) {
    double x = 0;
    ParseDouble(p, &x);
    v.push_back(x);
  }
  return v;
}

std::string ShardMeta::ToString() const {
  std::ostringstream os;
  os << "shard_idx=" << shard_idx << "\nshard_num=" << shard_num << "\nnum_partitions=" << num_partitions
     << "\nnode_sum_weight=" << JoinD(node_weight_sums) << "\nedge_sum_weight=" << JoinD(edge_weight_sums)
     << "\ngraph_label=" << HexEncode(Join(graph_labels, "\x1f")) << "\nindex_info=" << index_info
     << "\ngraph_meta=" << HexEncode(graph_meta) << "\n";
  return os.str();
}

bool ShardMeta::Parse(const std::string& s, ShardMeta* m) {
  for (auto& line : Split(s, "\n")) {
    const size_t eq = line.find('=');
    if (eq == std::string::npos) continue;
    const std::string k = line.substr(0, eq), v = line.substr(eq + 1);
    int64_t x;
    if (k == "shard_idx" && ParseInt64(v, &x)) m->shard_idx = static_cast<int>(x);
    else if (k == "shard_num" && ParseInt64(v, &x)) m->shard_num = static_cast<int>(x);
    else if (k == "num_partitions" && ParseInt64(v, &x)) m->num_partitions = static_cast<uint32_t>(x);
    else if (k == "node_sum_weight") m->node_weight_sums = SplitD(v);
    else if (k == "edge_sum_weight") m->edge_weight_sums = SplitD(v);
    else if (k == "graph_label") m->graph_labels = Split(HexDecode(v), "\x1f");
    else if (k == "index_info") m->index_info = v;
    else if (k == "graph_meta") m->graph_meta = HexDecode(v);
  }
  return true;
}

ShardMeta ShardMeta::FromEnv(const EngineEnv& env, int shard_idx, int shard_num) {
  ShardMeta m;
  m.shard_idx = shard_idx;
  m.shard_num = shard_num;
  if (env.graph) {
    const Graph& g = *env.graph;
    m.num_partitions = std::max<uint32_t>(1, g.meta().partitions_num);
    for (int t = 0; t < g.num_node_types(); ++t) m.node_weight_sums.push_back(g.NodeWeightSum(t));
    for (int t = 0; t < g.num_edge_types(); ++t) m.edge_weight_sums.push_back(g.EdgeWeightSum(t));
    m.graph_labels = g.graph_labels();
    m.graph_meta = g.meta().Serialize();
  }
  if (env.index) m.index_info = env.index->IndexInfo();
  return m;
}

// ============================================================================ Registry
namespace {
class FileRegistry : public Registry {
 public:
  explicit FileRegistry(std::string dir) : dir_(std::move(dir)) { MakeDirs(dir_); }
  Status Register(int shard, const Endpoint& ep, const ShardMeta& meta) override {
    const std::string tmp = JoinPath(dir_, ".tmp." + std::to_string(shard) + "#" + ep.ToString());
    EULER_RETURN_IF_ERROR(WriteFile(tmp, meta.ToString()));
    if (rename(tmp.c_str(), JoinPath(dir_, std::to_string(shard) + "#" + ep.ToString()).c_str()) != 0)
      return Status::Internal("registry rename failed");
    return Status::OK();
  }
  Status Deregister(int shard, const Endpoint& ep) override {
    unlink(JoinPath(dir_, std::to_string(shard) + "#" + ep.ToString()).c_str());
    return Status::OK();
  }
  Status Heartbeat(int shard, const Endpoint& ep) override {
    const std::string path = JoinPath(dir_, std::to_string(shard) + "#" + ep.ToString());
    if (utimensat(AT_FDCWD, path.c_str(), nullptr, 0) != 0)
      return errno == ENOENT ? Status::NotFound("registry entry gone: " + path)
                             : Status::Internal("registry heartbeat failed: " + path);
    return Status::OK();
  }
  Status List(std::map<int, std::vector<std::pair<Endpoint, ShardMeta>>>* out, double ttl) override {
    out->clear();
    std::vector<std::string> names;
    EULER_RETURN_IF_ERROR(ListDir(dir_, &names));
    const double now = WallSec();
    for (auto& n : names) {
      if (n.empty() || n[0] == '.') continue;
      if (ttl > 0) {
        struct stat st;
        if (stat(JoinPath(dir_, n).c_str(), &st) != 0) continue;
        const double mt = st.st_mtim.tv_sec + 1e-9 * st.st_mtim.tv_nsec;
        if (now - mt > ttl) continue;  // no heartbeat within ttl: the server is gone
      }
      const size_t h = n.find('#'), c = n.rfind(':');
      int64_t shard, port;
      if (h == std::string::npos || c == std::string::npos || !ParseInt64(n.substr(0, h), &shard) ||
          !ParseInt64(n.substr(c + 1), &port))
        continue;
      std::unique_ptr<FileView> f;
      if (!FileView::Open(JoinPath(dir_, n), &f).ok()) continue;
      ShardMeta m;
      ShardMeta::Parse(std::string(f->data(), f->size()), &m);
      (*out)[static_cast<int>(shard)].push_back({Endpoint{n.substr(h + 1, c - h - 1), static_cast<int>(port)}, m});
    }
    return Status::OK();
  }

 private:
  std::string dir_;
};

class MemoryRegistry : public Registry {
 public:
  explicit MemoryRegistry(std::string name) : name_(std::move(name)) {}
  static std::mutex& mu() {
    static std::mutex m;
    return m;
  }
  static std::map<std::string, std::map<std::string, std::tuple<int, Endpoint, ShardMeta>>>& store() {
    static std::map<std::string, std::map<std::string, std::tuple<int, Endpoint, ShardMeta>>> s;
    return s;
  }
  Status Register(int shard, const Endpoint& ep, const ShardMeta& meta) override {
    std::lock_guard<std::mutex> l(mu());
    store()[name_][std::to_string(shard) + "#" + ep.ToString()] = std::make_tuple(shard, ep, meta);
    return Status::OK();
  }
  Status Deregister(int shard, const Endpoint& ep) override {
    std::lock_guard<std::mutex> l(mu());
    store()[name_].erase(std::to_string(shard) + "#" + ep.ToString());
    return Status::OK();
  }
  Status Heartbeat(int shard, const Endpoint& ep) override {  // in-process: lives with the server
    std::lock_guard<std::mutex> l(mu());
    return store()[name_].count(std::to_string(shard) + "#" + ep.ToString()) ? Status::OK()
                                                                             : Status::NotFound("gone");
  }
  Status List(std::map<int, std::vector<std::pair<Endpoint, ShardMeta>>>* out, double) override {
    std::lock_guard<std::mutex> l(mu());
    out->clear();
    for (auto& kv : store()[name_]) (*out)[std::get<0>(kv.second)].push_back({std::get<1>(kv.second), std::get<2>(kv.second)});
    return Status::OK();
  }

 private:
  std::string name_;
};

// ---------------------------------------------------------------- TCP registry (client side)
// record separators of the list reply: metas are "k=v\n" text with hex-encoded free-form
// fields, so they never contain these bytes
constexpr char kRecSep = '\x1d', kFieldSep = '\x1e';

class TcpRegistry : public Registry {
 public:
  explicit TcpRegistry(Endpoint ep) : ep_(std::move(ep)) {}
  Status Register(int shard, const Endpoint& ep, const ShardMeta& meta) override {
    return Call(kRegPut, std::to_string(shard) + kFieldSep + ep.ToString() + kFieldSep + meta.ToString(), nullptr);
  }
  Status Deregister(int shard, const Endpoint& ep) override {
    return Call(kRegDel, std::to_string(shard) + kFieldSep + ep.ToString(), nullptr);
  }
  Status Heartbeat(int shard, const Endpoint& ep) override {
    return Call(kRegBeat, std::to_string(shard) + kFieldSep + ep.ToString(), nullptr);
  }
  Status List(std::map<int, std::vector<std::pair<Endpoint, ShardMeta>>>* out, double ttl) override {
    out->clear();
    std::string body;
    EULER_RETURN_IF_ERROR(Call(kRegList, std::to_string(ttl), &body));
    for (auto& rec : Split(body, std::string(1, kRecSep))) {
      auto f = Split(rec, std::string(1, kFieldSep));
      if (f.size() != 3) continue;
      int64_t shard, port;
      const size_t c = f[1].rfind(':');
      if (c == std::string::npos || !ParseInt64(f[0], &shard) || !ParseInt64(f[1].substr(c + 1), &port)) continue;
      ShardMeta m;
      ShardMeta::Parse(f[2], &m);
      (*out)[static_cast<int>(shard)].push_back({Endpoint{f[1].substr(0, c), static_cast<int>(port)}, m});
    }
    return Status::OK();
  }

 private:
  // one request per short connection: "OK" / "NF" (not found) / "ER<msg>" + body
  Status Call(uint32_t kind, const std::string& payload, std::string* body) {
    const int fd = Connect(ep_, 5000);
    if (fd < 0) return Status::Unavailable("registry " + ep_.ToString() + " unreachable");
    uint32_t rk = 0;
    std::string reply;
    const bool ok = SendFrame(fd, kind, payload) && RecvFrame(fd, &rk, &reply) && rk == kReply && reply.size() >= 2;
    close(fd);
    if (!ok) return Status::Unavailable("registry " + ep_.ToString() + " request failed");
    if (StartsWith(reply, "NF")) return Status::NotFound("registry entry gone");
    if (!StartsWith(reply, "OK")) return Status::Internal("registry: " + reply.substr(2));
    if (body) *body = reply.substr(2);
    return Status::OK();
  }
  Endpoint ep_;
};
}  // namespace

// ---------------------------------------------------------------- RegistryServer
RegistryServer::RegistryServer(int port) : port_req_(port) {}
RegistryServer::~RegistryServer() { Stop(); }

Status RegistryServer::Start() {
  fd_ = socket(AF_INET, SOCK_STREAM, 0);
  if (fd_ < 0) return Status::Internal("socket failed");
  int one = 1;
  setsockopt(fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  struct sockaddr_in addr;
  memset(&addr, 0, sizeof(addr));
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_ANY);
  addr.sin_port = htons(static_cast<uint16_t>(port_req_));
  if (bind(fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0)
    return Status::Internal("registry bind failed: " + std::string(strerror(errno)));
  if (listen(fd_, 256) != 0) return Status::Internal("registry listen failed");
  socklen_t len = sizeof(addr);
  getsockname(fd_, reinterpret_cast<sockaddr*>(&addr), &len);
  port_ = ntohs(addr.sin_port);
  running_ = true;
  th_ = std::thread([this] { Loop(); });
  EULER_LOG(Info) << "registry server listening on " << port_;
  return Status::OK();
}

void RegistryServer::Stop() {
  if (!running_.exchange(false)) return;
  shutdown(fd_, SHUT_RDWR);
  close(fd_);
  if (th_.joinable()) th_.join();
}

size_t RegistryServer::size() {
  std::lock_guard<std::mutex> l(mu_);
  return entries_.size();
}

void RegistryServer::Loop() {
  // requests are tiny and connections short: served one at a time on this thread, each
  // socket with a receive timeout so a stalled client cannot block the registry
  while (running_) {
    const int c = accept(fd_, nullptr, nullptr);
    if (c < 0) {
      if (!running_) break;
      continue;
    }
    SetTimeouts(c, 2000);
    uint32_t kind;
    std::string payload;
    if (RecvFrame(c, &kind, &payload)) SendFrame(c, kReply, Handle(kind, payload));
    close(c);
  }
}

std::string RegistryServer::Handle(uint32_t kind, const std::string& payload) {
  auto f = Split(payload, std::string(1, kFieldSep));
  std::lock_guard<std::mutex> l(mu_);
  const double now = WallSec();
  if (kind == kRegList) {
    double ttl = 0;
    ParseDouble(payload, &ttl);
    std::string out = "OK";
    bool first = true;
    for (auto& kv : entries_) {
      if (ttl > 0 && now - kv.second.seen > ttl) continue;
      if (!first) out += kRecSep;
      first = false;
      out += std::to_string(kv.second.shard) + kFieldSep + kv.second.ep.ToString() + kFieldSep + kv.second.meta;
    }
    return out;
  }
  if (f.size() < 2) return "ERmalformed request";
  int64_t shard, port;
  const size_t c = f[1].rfind(':');
  if (!ParseInt64(f[0], &shard) || c == std::string::npos || !ParseInt64(f[1].substr(c + 1), &port))
    return "ERmalformed endpoint";
  const std::string key = f[0] + "#" + f[1];
  if (kind == kRegPut) {
    if (f.size() != 3) return "ERmalformed put";
    entries_[key] = Entry{static_cast<int>(shard), Endpoint{f[1].substr(0, c), static_cast<int>(port)}, f[2], now};
    return "OK";
  }
  if (kind == kRegBeat) {
    auto it = entries_.find(key);
    if (it == entries_.end()) return "NF";
    it->second.seen = now;
    return "OK";
  }
  if (kind == kRegDel) {
    entries_.erase(key);
    return "OK";
  }
  return "ERunknown request";
}

std::unique_ptr<Registry> Registry::Open(const std::string& spec) {
  if (StartsWith(spec, "tcp://")) {
    const std::string hp = spec.substr(6);
    const size_t c = hp.rfind(':');
    int64_t port = 0;
    if (c == std::string::npos || !ParseInt64(hp.substr(c + 1), &port))
      EULER_THROW("registry spec tcp://<host>:<port> expected, got " + spec);
    return std::unique_ptr<Registry>(new TcpRegistry(Endpoint{hp.substr(0, c), static_cast<int>(port)}));
  }
  if (StartsWith(spec, "memory:")) return std::unique_ptr<Registry>(new MemoryRegistry(spec.substr(7)));
  if (StartsWith(spec, "file:")) return std::unique_ptr<Registry>(new FileRegistry(spec.substr(5)));
  if (StartsWith(spec, "zk:") || spec.find("2181") != std::string::npos)
    EULER_THROW("ZooKeeper registries are not built into euler_amd; run euler_amd.tools.registry and use "
                "tcp://<host>:<port>, or a shared directory (file:<dir>)");
  return std::unique_ptr<Registry>(new FileRegistry(spec));
}

// ============================================================================ GraphServer
// Event-driven server: accept threads hand each connection to one of `io_threads` epoll
// loops (non-blocking sockets, level-triggered).  A loop reassembles frames from its
// connections' byte streams, answers ping / meta inline and schedules DAG executions on
// the worker pool; a finished execution is posted back to the connection's loop
// (mutex-protected completion queue + eventfd wake-up), which writes the reply without
// blocking (EPOLLOUT while a reply is partially sent).  Threads do not grow with the
// number of client connections (8 ranks x many workers x S shards), unlike the
// thread-per-connection design it replaces.
struct GraphServer::Conn {
  int fd = -1;
  std::string in;       // received bytes not yet consumed
  size_t in_off = 0;
  std::string out;      // reply bytes not yet written
  size_t out_off = 0;
  bool busy = false;    // an execution of this connection is in flight (one at a time)
  bool closed = false;
  bool want_out = false;
  int pending_fd = -1;  // memfd received with the attach frame
  char* shm = nullptr;  // the client's shared region (same-host connections)
  size_t shm_cap = 0;
  ~Conn() {
    if (shm) munmap(shm, shm_cap);
    if (pending_fd >= 0) close(pending_fd);
  }
};

struct GraphServer::Loop {
  int ep = -1, wake = -1;
  std::thread th;
  std::unordered_map<int, std::shared_ptr<Conn>> conns;  // loop thread only
  std::mutex mu;                                           // guards the queues below
  std::vector<int> incoming;                                // accepted fds to adopt
  std::vector<std::pair<std::shared_ptr<Conn>, std::string>> done;  // finished replies
  void Wake() {
    const uint64_t one = 1;
    ssize_t r = ::write(wake, &one, sizeof(one));
    (void)r;
  }
};

GraphServer::GraphServer(EngineEnv* env, int shard_idx, int shard_num, const ServerOptions& opt)
    : env_(env), shard_idx_(shard_idx), shard_num_(shard_num), opt_(opt) {
  host_ = opt.host.empty() ? "127.0.0.1" : opt.host;
}

GraphServer::~GraphServer() { Stop(); }

Status GraphServer::Start() {
  listen_fd_ = socket(AF_INET, SOCK_STREAM, 0);
  if (listen_fd_ < 0) return Status::Internal("socket failed");
  int one = 1;
  setsockopt(listen_fd_, SOL_SOCKET, SO_REUSEADDR, &one, sizeof(one));
  struct sockaddr_in addr;
  memset(&addr, 0, sizeof(addr));
  addr.sin_family = AF_INET;
  addr.sin_addr.s_addr = htonl(INADDR_ANY);
  addr.sin_port = htons(static_cast<uint16_t>(opt_.port));
  if (bind(listen_fd_, reinterpret_cast<sockaddr*>(&addr), sizeof(addr)) != 0)
    return Status::Internal("bind failed on port " + std::to_string(opt_.port) + ": " + strerror(errno));
  if (listen(listen_fd_, 1024) != 0) return Status::Internal("listen failed");
  socklen_t len = sizeof(addr);
  getsockname(listen_fd_, reinterpret_cast<sockaddr*>(&addr), &len);
  port_ = ntohs(addr.sin_port);
  pool_.reset(new ThreadPool(std::max(1, opt_.num_threads), "euler-server"));
  running_ = true;
  for (int i = 0; i < std::max(1, opt_.io_threads); ++i) {
    std::unique_ptr<Loop> lp(new Loop);
    lp->ep = epoll_create1(EPOLL_CLOEXEC);
    lp->wake = eventfd(0, EFD_NONBLOCK | EFD_CLOEXEC);
    if (lp->ep < 0 || lp->wake < 0) return Status::Internal("epoll/eventfd failed");
    struct epoll_event ev;
    memset(&ev, 0, sizeof(ev));
    ev.events = EPOLLIN;
    ev.data.fd = lp->wake;
    epoll_ctl(lp->ep, EPOLL_CTL_ADD, lp->wake, &ev);
    Loop* raw = lp.get();
    lp->th = std::thread([this, raw] { RunLoop(raw); });
    loops_.push_back(std::move(lp));
  }
  accept_thread_ = std::thread([this] { AcceptLoop(listen_fd_); });
  // same-host listener (abstract Unix socket keyed by the TCP port); best effort
  local_fd_ = socket(AF_UNIX, SOCK_STREAM, 0);
  if (local_fd_ >= 0) {
    struct sockaddr_un ua;
    const socklen_t ulen = AbstractAddr(port_, &ua);
    if (bind(local_fd_, reinterpret_cast<sockaddr*>(&ua), ulen) == 0 && listen(local_fd_, 1024) == 0) {
      local_accept_thread_ = std::thread([this] { AcceptLoop(local_fd_); });
    } else {
      close(local_fd_);
      local_fd_ = -1;
    }
  }
  if (!opt_.registry.empty()) {
    registry_ = Registry::Open(opt_.registry);
    const ShardMeta meta = ShardMeta::FromEnv(*env_, shard_idx_, shard_num_);
    EULER_RETURN_IF_ERROR(registry_->Register(shard_idx_, endpoint(), meta));
    if (opt_.heartbeat_ms > 0) {
      heartbeat_thread_ = std::thread([this, meta] {
        for (;;) {
          {
            std::unique_lock<std::mutex> l(hb_mu_);
            // system_clock deadline: pthread_cond_timedwait (steady-clock waits use
            // pthread_cond_clockwait, which gcc-11's TSAN does not intercept)
            hb_cv_.wait_until(l, std::chrono::system_clock::now() + std::chrono::milliseconds(opt_.heartbeat_ms),
                              [this] { return !running_.load(); });
            if (!running_.load()) return;
          }
          // registry I/O outside the lock
          const Status st = registry_->Heartbeat(shard_idx_, endpoint());
          if (st.code() == Code::NOT_FOUND) registry_->Register(shard_idx_, endpoint(), meta);  // re-register
        }
      });
    }
  }
  EULER_LOG(Info) << "graph server shard " << shard_idx_ << "/" << shard_num_ << " listening on " << port_
                  << " (" << loops_.size() << " epoll loops, " << opt_.num_threads << " workers)";
  return Status::OK();
}

void GraphServer::Stop() {
  if (!running_.exchange(false)) return;
  { std::lock_guard<std::mutex> l(hb_mu_); }  // the heartbeat thread sees running_ == false
  hb_cv_.notify_all();
  if (heartbeat_thread_.joinable()) heartbeat_thread_.join();
  if (registry_) registry_->Deregister(shard_idx_, endpoint());
  shutdown(listen_fd_, SHUT_RDWR);
  close(listen_fd_);
  if (local_fd_ >= 0) {
    shutdown(local_fd_, SHUT_RDWR);
    close(local_fd_);
  }
  if (accept_thread_.joinable()) accept_thread_.join();
  if (local_accept_thread_.joinable()) local_accept_thread_.join();
  // running executions finish first (their completions are then discarded)
  pool_.reset();
  for (auto& lp : loops_) lp->Wake();
  for (auto& lp : loops_) {
    if (lp->th.joinable()) lp->th.join();
    for (auto& kv : lp->conns) close(kv.first);
    {
      std::lock_guard<std::mutex> l(lp->mu);
      for (int fd : lp->incoming) close(fd);
      lp->incoming.clear();
      lp->done.clear();
    }
    close(lp->ep);
    close(lp->wake);
  }
  loops_.clear();
}

void GraphServer::AcceptLoop(int lfd) {
  while (running_) {
    int fd = accept4(lfd, nullptr, nullptr, SOCK_NONBLOCK | SOCK_CLOEXEC);
    if (fd < 0) {
      if (!running_) break;
      continue;
    }
    int one = 1;
    setsockopt(fd, IPPROTO_TCP, TCP_NODELAY, &one, sizeof(one));  // fails harmlessly on Unix sockets
    Loop* lp = loops_[next_loop_.fetch_add(1) % loops_.size()].get();
    {
      std::lock_guard<std::mutex> l(lp->mu);
      lp->incoming.push_back(fd);
    }
    lp->Wake();
  }
}

void GraphServer::RunLoop(Loop* lp) {
  std::vector<struct epoll_event> evs(256);
  while (running_) {
    const int n = epoll_wait(lp->ep, evs.data(), static_cast<int>(evs.size()), 200);
    if (n < 0 && errno != EINTR) break;
    for (int i = 0; i < std::max(n, 0); ++i) {
      const int fd = evs[i].data.fd;
      if (fd == lp->wake) {
        uint64_t v;
        while (::read(lp->wake, &v, sizeof(v)) > 0) {
        }
        continue;
      }
      auto it = lp->conns.find(fd);
      if (it == lp->conns.end()) continue;
      std::shared_ptr<Conn> c = it->second;
      if (evs[i].events & (EPOLLERR | EPOLLHUP)) {
        if (!(evs[i].events & EPOLLIN)) {
          Drop(lp, c);
          continue;
        }
      }
      if (evs[i].events & EPOLLOUT) Flush(lp, c);
      if (!c->closed && (evs[i].events & EPOLLIN)) OnReadable(lp, c);
    }
    // adopt new connections, deliver finished executions
    std::vector<int> inc;
    std::vector<std::pair<std::shared_ptr<Conn>, std::string>> done;
    {
      std::lock_guard<std::mutex> l(lp->mu);
      inc.swap(lp->incoming);
      done.swap(lp->done);
    }
    for (int fd : inc) {
      auto c = std::make_shared<Conn>();
      c->fd = fd;
      struct epoll_event ev;
      memset(&ev, 0, sizeof(ev));
      ev.events = EPOLLIN;
      ev.data.fd = fd;
      if (epoll_ctl(lp->ep, EPOLL_CTL_ADD, fd, &ev) != 0) {
        close(fd);
        continue;
      }
      lp->conns[fd] = c;
    }
    for (auto& d : done) {
      std::shared_ptr<Conn> c = d.first;
      c->busy = false;
      if (c->closed) continue;
      c->out.append(d.second);
      Flush(lp, c);
      if (!c->closed) Dispatch(lp, c);  // a pipelined next request may already be buffered
    }
  }
}

void GraphServer::OnReadable(Loop* lp, const std::shared_ptr<Conn>& c) {
  char buf[1 << 16];
  for (;;) {
    struct iovec iov;
    iov.iov_base = buf;
    iov.iov_len = sizeof(buf);
    char ctrl[CMSG_SPACE(sizeof(int))];
    struct msghdr msg;
    memset(&msg, 0, sizeof(msg));
    msg.msg_iov = &iov;
    msg.msg_iovlen = 1;
    msg.msg_control = ctrl;
    msg.msg_controllen = sizeof(ctrl);
    const ssize_t k = ::recvmsg(c->fd, &msg, MSG_CMSG_CLOEXEC);
    if (k > 0) {
      for (struct cmsghdr* cm = CMSG_FIRSTHDR(&msg); cm; cm = CMSG_NXTHDR(&msg, cm)) {
        if (cm->cmsg_level == SOL_SOCKET && cm->cmsg_type == SCM_RIGHTS) {
          int got;
          memcpy(&got, CMSG_DATA(cm), sizeof(int));
          if (c->pending_fd >= 0) close(c->pending_fd);
          c->pending_fd = got;
        }
      }
    }
    if (k > 0) {
      c->in.append(buf, static_cast<size_t>(k));
      continue;
    }
    if (k < 0 && errno == EINTR) continue;
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) break;
    Drop(lp, c);  // orderly shutdown or error
    return;
  }
  Dispatch(lp, c);
}

void GraphServer::Dispatch(Loop* lp, const std::shared_ptr<Conn>& c) {
  while (!c->busy && !c->closed) {
    const size_t avail = c->in.size() - c->in_off;
    if (avail < 16) break;
    const char* h = c->in.data() + c->in_off;
    uint32_t magic, kind;
    uint64_t len;
    memcpy(&magic, h, 4);
    memcpy(&kind, h + 4, 4);
    memcpy(&len, h + 8, 8);
    if (magic != kMagic || len > (1ULL << 36)) {
      Drop(lp, c);
      return;
    }
    if (avail < 16 + len) break;
    std::string payload(h + 16, static_cast<size_t>(len));
    c->in_off += 16 + len;
    if (c->in_off == c->in.size()) {
      c->in.clear();
      c->in_off = 0;
    } else if (c->in_off > (1u << 20)) {
      c->in.erase(0, c->in_off);
      c->in_off = 0;
    }
    if (kind == kShmAttach) {  // map the client's region (fd arrived with these bytes)
      const uint64_t size = DecodeLen(payload);
      if (c->pending_fd >= 0 && size > 0) {
        void* p = mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_SHARED, c->pending_fd, 0);
        if (p != MAP_FAILED) {
          if (c->shm) munmap(c->shm, c->shm_cap);
          c->shm = static_cast<char*>(p);
          c->shm_cap = size;
          EngineCounters::Get().shm_channels.fetch_add(1, std::memory_order_relaxed);
        }
        close(c->pending_fd);
        c->pending_fd = -1;
      }
      continue;  // no reply
    }
    bool via_shm = false;
    if (kind & kShmFlag) {  // the request payload is in the shared region
      const uint64_t n = DecodeLen(payload);
      if (!c->shm || n > c->shm_cap) {
        Drop(lp, c);
        return;
      }
      payload.assign(c->shm, n);
      EngineCounters::Get().shm_bytes.fetch_add(static_cast<int64_t>(n), std::memory_order_relaxed);
      kind &= ~kShmFlag;
      via_shm = true;
    }
    (void)via_shm;
    requests_++;
    EngineCounters::Get().server_requests.fetch_add(1, std::memory_order_relaxed);
    if (kind != kExecute) {
      std::string reply = Handle(kind, payload);
      char hdr[16];
      const uint64_t rl = reply.size();
      const uint32_t rk = kReply;
      memcpy(hdr, &kMagic, 4);
      memcpy(hdr + 4, &rk, 4);
      memcpy(hdr + 8, &rl, 8);
      c->out.append(hdr, 16);
      c->out.append(reply);
      Flush(lp, c);
      continue;
    }
    c->busy = true;
    std::shared_ptr<Conn> keep = c;
    pool_->Schedule([this, lp, keep, payload = std::move(payload)] {
      Status st;
      std::vector<Tensor> res;
      std::string reply;
      uint32_t rk = kReply;
      {
        ScopedMicros timing(&EngineCounters::Get().server_us);
        HandleExecute(payload, &st, &res);
        const size_t n = ReplySize(st, res);
        if (keep->shm && n >= kShmMin && n <= keep->shm_cap) {
          // the request was consumed (copied out) before this task ran: the region is
          // free, and the reply is encoded straight into it
          BytesWriter w(keep->shm, keep->shm_cap);
          EncodeReplyTo(&w, st, res);
          EngineCounters::Get().shm_bytes.fetch_add(static_cast<int64_t>(n), std::memory_order_relaxed);
          reply = EncodeLen(n);
          rk = kReply | kShmFlag;
        } else {
          reply = EncodeReply(st, res);
        }
      }
      char hdr[16];
      const uint64_t rl = reply.size();
      memcpy(hdr, &kMagic, 4);
      memcpy(hdr + 4, &rk, 4);
      memcpy(hdr + 8, &rl, 8);
      std::string frame(hdr, 16);
      frame.append(reply);
      {
        std::lock_guard<std::mutex> l(lp->mu);
        lp->done.emplace_back(keep, std::move(frame));
      }
      lp->Wake();
    });
  }
}

void GraphServer::Flush(Loop* lp, const std::shared_ptr<Conn>& c) {
  while (c->out_off < c->out.size()) {
    const ssize_t k = ::send(c->fd, c->out.data() + c->out_off, c->out.size() - c->out_off, MSG_NOSIGNAL);
    if (k > 0) {
      c->out_off += static_cast<size_t>(k);
      continue;
    }
    if (k < 0 && errno == EINTR) continue;
    if (k < 0 && (errno == EAGAIN || errno == EWOULDBLOCK)) {
      if (!c->want_out) {
        struct epoll_event ev;
        memset(&ev, 0, sizeof(ev));
        ev.events = EPOLLIN | EPOLLOUT;
        ev.data.fd = c->fd;
        epoll_ctl(lp->ep, EPOLL_CTL_MOD, c->fd, &ev);
        c->want_out = true;
      }
      return;
    }
    Drop(lp, c);
    return;
  }
  c->out.clear();
  c->out_off = 0;
  if (c->want_out) {
    struct epoll_event ev;
    memset(&ev, 0, sizeof(ev));
    ev.events = EPOLLIN;
    ev.data.fd = c->fd;
    epoll_ctl(lp->ep, EPOLL_CTL_MOD, c->fd, &ev);
    c->want_out = false;
  }
}

void GraphServer::Drop(Loop* lp, const std::shared_ptr<Conn>& c) {
  if (c->closed) return;
  c->closed = true;
  epoll_ctl(lp->ep, EPOLL_CTL_DEL, c->fd, nullptr);
  close(c->fd);
  lp->conns.erase(c->fd);
}

std::string GraphServer::Handle(uint32_t kind, const std::string& payload) {
  ScopedMicros timing(&EngineCounters::Get().server_us);
  if (kind == kPing) return EncodeReply(Status::OK(), {});
  if (kind == kMeta)
    return EncodeReply(Status::OK(), {Tensor::Strings({ShardMeta::FromEnv(*env_, shard_idx_, shard_num_).ToString()})});
  if (kind != kExecute) return EncodeReply(Status::Unimplemented("unknown request kind"), {});
  Status st;
  std::vector<Tensor> res;
  HandleExecute(payload, &st, &res);
  return EncodeReply(st, res);
}

void GraphServer::HandleExecute(const std::string& payload, Status* st, std::vector<Tensor>* res) {
  DAGDef dag;
  std::vector<std::pair<std::string, Tensor>> inputs;
  std::vector<std::string> outputs;
  res->clear();
  if (!DecodeExecute(payload, &dag, &inputs, &outputs)) {
    *st = Status::RpcError("malformed execute request");
    return;
  }
  try {
    *st = ExecuteDag(env_, dag, inputs, outputs, res);
  } catch (const std::exception& e) {
    *st = Status::Internal(e.what());
  }
}

// ============================================================================ RpcClients
RpcClients::RpcClients(std::map<int, std::vector<Endpoint>> shards, const ClientOptions& opt) : opt_(opt) {
  int n = 0;
  for (auto& kv : shards) n = std::max(n, kv.first + 1);
  shards_.resize(n);
  rr_ = std::vector<std::atomic<uint64_t>>(n);
  for (auto& kv : shards) {
    auto hl = std::make_shared<HostList>();
    for (auto& ep : kv.second) {
      auto h = std::make_shared<Host>();
      h->ep = ep;
      hl->push_back(std::move(h));
    }
    shards_[kv.first] = std::move(hl);
  }
  for (auto& sp : shards_)
    if (!sp) sp = std::make_shared<HostList>();
  pool_.reset(new ThreadPool(std::max(8, 2 * n), "euler-client"));
}

RpcClients::~RpcClients() {
  pool_.reset();  // in-flight calls finish first; the Host destructors close the pooled channels
}

void RpcClients::UpdateShard(int shard, const std::vector<Endpoint>& eps) {
  if (shard < 0 || shard >= static_cast<int>(shards_.size()) || eps.empty()) return;
  auto cur = std::atomic_load(&shards_[shard]);
  auto next = std::make_shared<HostList>();
  for (const auto& ep : eps) {
    std::shared_ptr<Host> keep;
    for (const auto& h : *cur)
      if (h->ep.host == ep.host && h->ep.port == ep.port) keep = h;
    if (!keep) {
      keep = std::make_shared<Host>();
      keep->ep = ep;
    }
    next->push_back(std::move(keep));
  }
  std::atomic_store(&shards_[shard], std::shared_ptr<const HostList>(std::move(next)));
}

std::map<int, std::vector<std::string>> RpcClients::Endpoints() const {
  std::map<int, std::vector<std::string>> out;
  for (size_t s = 0; s < shards_.size(); ++s)
    for (const auto& h : *std::atomic_load(&shards_[s])) out[static_cast<int>(s)].push_back(h->ep.ToString());
  return out;
}

RpcClients::Chan RpcClients::OpenChan(const Endpoint& ep, int timeout_ms) {
  Chan c;
  c.fd = Connect(ep, timeout_ms);
  if (c.fd < 0) return c;
  struct sockaddr_storage ss;
  socklen_t sl = sizeof(ss);
  const size_t cap = ShmCapacity();
  const char* off = std::getenv("EULER_RPC_SHM");
  if (cap == 0 || (off && std::string(off) == "0") || getsockname(c.fd, reinterpret_cast<sockaddr*>(&ss), &sl) != 0 ||
      ss.ss_family != AF_UNIX)
    return c;
  // same host: a shared region for large payloads, handed to the server with the attach frame
  const int mfd = static_cast<int>(syscall(SYS_memfd_create, "euler_amd_rpc", MFD_CLOEXEC_FLAG));
  if (mfd < 0) return c;
  if (ftruncate(mfd, static_cast<off_t>(cap)) == 0) {
    void* p = mmap(nullptr, cap, PROT_READ | PROT_WRITE, MAP_SHARED, mfd, 0);
    if (p != MAP_FAILED) {
      if (SendAttach(c.fd, mfd, cap)) {
        c.shm = static_cast<char*>(p);
        c.cap = cap;
        EngineCounters::Get().shm_channels.fetch_add(1, std::memory_order_relaxed);
      } else {
        munmap(p, cap);
      }
    }
  }
  close(mfd);  // the mappings keep the region alive
  return c;
}

void RpcClients::CloseChan(Chan* c) {
  if (c->shm) munmap(c->shm, c->cap);
  if (c->fd >= 0) close(c->fd);
  c->shm = nullptr;
  c->fd = -1;
}

Status RpcClients::CallHost(Host* h, uint32_t kind, const std::string& payload, std::string* reply, size_t* in_bytes,
                            std::vector<Tensor>* decoded, Status* app) {
  Chan c;
  {
    std::lock_guard<std::mutex> l(h->mu);
    if (!h->idle.empty()) {
      c = h->idle.back();
      h->idle.pop_back();
    }
  }
  if (c.fd < 0) c = OpenChan(h->ep, opt_.timeout_ms);
  if (c.fd < 0) return Status::Unavailable("connect failed: " + h->ep.ToString());
  uint32_t rk;
  bool ok;
  if (c.shm && payload.size() >= kShmMin && payload.size() <= c.cap) {
    memcpy(c.shm, payload.data(), payload.size());
    EngineCounters::Get().shm_bytes.fetch_add(static_cast<int64_t>(payload.size()), std::memory_order_relaxed);
    ok = SendFrame(c.fd, kind | kShmFlag, EncodeLen(payload.size()));
  } else {
    ok = SendFrame(c.fd, kind, payload);
  }
  ok = ok && RecvFrame(c.fd, &rk, reply);
  // a malformed reply is a transport failure; the server's own status goes to *app
  if (ok && rk == (kReply | kShmFlag) && c.shm) {
    const uint64_t n = DecodeLen(*reply);
    ok = n <= c.cap;
    if (ok) {
      EngineCounters::Get().shm_bytes.fetch_add(static_cast<int64_t>(n), std::memory_order_relaxed);
      *in_bytes = n;
      if (decoded) {  // decode straight out of the region: no staging copy
        reply->clear();
        ok = ParseReply(c.shm, n, app, decoded);
      } else {
        reply->assign(c.shm, n);
      }
    }
  } else {
    ok = ok && rk == kReply;
    *in_bytes = reply->size();
    if (ok && decoded) ok = ParseReply(reply->data(), reply->size(), app, decoded);
  }
  if (!ok) {
    CloseChan(&c);
    return Status::RpcError("rpc to " + h->ep.ToString() + " failed");
  }
  std::lock_guard<std::mutex> l(h->mu);
  if (static_cast<int>(h->idle.size()) < opt_.num_channels_per_host) h->idle.push_back(c);
  else CloseChan(&c);
  return Status::OK();
}

Status RpcClients::Call(int shard, uint32_t kind, const std::string& payload, std::string* reply,
                        std::vector<Tensor>* decoded, Status* app) {
  if (shard < 0 || shard >= static_cast<int>(shards_.size()))
    return Status::Unavailable("no server for shard " + std::to_string(shard));
  const std::shared_ptr<const HostList> snap = std::atomic_load(&shards_[shard]);  // registry watch may swap it
  const HostList& hosts = *snap;
  if (hosts.empty()) return Status::Unavailable("no server for shard " + std::to_string(shard));
  Status last;
  auto& ctr = EngineCounters::Get();
  for (int attempt = 0; attempt <= opt_.num_retries; ++attempt) {
    ctr.rpc_attempts.fetch_add(1, std::memory_order_relaxed);
    if (FaultDelayMs() > 0) std::this_thread::sleep_for(std::chrono::milliseconds(FaultDelayMs()));
    // round-robin over replicas that are not quarantined
    Host* h = nullptr;
    const double now = NowSec();
    for (size_t k = 0; k < hosts.size(); ++k) {
      Host* c = hosts[(rr_[shard].fetch_add(1)) % hosts.size()].get();
      if (c->bad_until <= now) {
        h = c;
        break;
      }
    }
    if (!h) h = hosts[rr_[shard].fetch_add(1) % hosts.size()].get();  // all bad: try anyway
    if (FaultRate() > 0 && ThreadRng().Uniform() < FaultRate()) {
      last = Status::RpcError("injected fault");
    } else {
      size_t in_bytes = 0;
      last = CallHost(h, kind, payload, reply, &in_bytes, decoded, app);
      if (last.ok()) {
        ctr.rpc_bytes_out.fetch_add(static_cast<int64_t>(payload.size()), std::memory_order_relaxed);
        ctr.rpc_bytes_in.fetch_add(static_cast<int64_t>(in_bytes), std::memory_order_relaxed);
        return last;
      }
    }
    ctr.rpc_failures.fetch_add(1, std::memory_order_relaxed);
    failures_++;
    h->bad_until = NowSec() + opt_.bad_host_timeout;  // move to bad host list
    EULER_LOG(Warning) << "rpc shard " << shard << " attempt " << attempt << " failed: " << last.message();
  }
  return last;
}

void RpcClients::Execute(int shard, const DAGDef& dag, std::vector<std::pair<std::string, Tensor>> inputs,
                         std::vector<std::string> outputs, Done done) {
  auto payload = std::make_shared<std::string>(EncodeExecute(dag, inputs, outputs));
  pool_->Schedule([this, shard, payload, done] {
    std::string reply;
    std::vector<Tensor> res;
    Status app;
    Status st = Call(shard, kExecute, *payload, &reply, &res, &app);
    if (st.ok()) st = app;
    done(st, std::move(res));
  });
}

Status RpcClients::Ping(int shard) {
  std::string reply;
  EULER_RETURN_IF_ERROR(Call(shard, kPing, "", &reply));
  std::vector<Tensor> r;
  return DecodeReply(reply, &r);
}

Status RpcClients::FetchMeta(int shard, ShardMeta* meta) {
  std::string reply;
  EULER_RETURN_IF_ERROR(Call(shard, kMeta, "", &reply));
  std::vector<Tensor> r;
  EULER_RETURN_IF_ERROR(DecodeReply(reply, &r));
  if (r.empty()) return Status::RpcError("empty meta reply");
  ShardMeta::Parse(r[0].strings()[0], meta);
  return Status::OK();
}

// ============================================================================ QueryProxy
Status LoadShard(const std::string& data_path, int shard_idx, int shard_num, std::unique_ptr<Graph>* g,
                 std::unique_ptr<IndexManager>* idx, int threads, const LoadOptions& opt) {
  GraphBuilder b;
  b.SetSamplers(opt.node_sampler, opt.edge_sampler);
  EULER_RETURN_IF_ERROR(
      b.LoadReferenceFormat(data_path, shard_idx, shard_num, opt.load_nodes, opt.load_edges, threads));
  *g = b.Finish();
  idx->reset(new IndexManager);
  EULER_RETURN_IF_ERROR((*idx)->Load(JoinPath(data_path, "Index"), shard_idx, shard_num));
  return Status::OK();
}

std::unique_ptr<EngineEnv> QueryProxy::MakeEnv(Graph* g, IndexManager* idx, int shard_num) {
  std::unique_ptr<EngineEnv> e(new EngineEnv);
  e->graph = g;
  e->index = idx;
  e->shard_num = shard_num;
  e->num_partitions = g ? std::max<uint32_t>(1, g->meta().partitions_num) : 1;
  if (g) e->graph_labels = g->graph_labels();
  if (idx) e->index_info = idx->IndexInfo();
  return e;
}

Status QueryProxy::FillWeightTables(const std::vector<ShardMeta>& metas) {
  const int S = static_cast<int>(metas.size());
  size_t nt = 0, et = 0;
  for (auto& m : metas) {
    nt = std::max(nt, m.node_weight_sums.size());
    et = std::max(et, m.edge_weight_sums.size());
  }
  // [type + 1][shard + 1]; last row = all types, last column = all shards
  auto fill = [&](bool node, size_t T, std::vector<std::vector<double>>* tab) {
    tab->assign(T + 1, std::vector<double>(S + 1, 0.0));
    for (int s = 0; s < S; ++s) {
      const auto& v = node ? metas[s].node_weight_sums : metas[s].edge_weight_sums;
      for (size_t t = 0; t < v.size(); ++t) {
        (*tab)[t][s] += v[t];
        (*tab)[t][S] += v[t];
        (*tab)[T][s] += v[t];
        (*tab)[T][S] += v[t];
      }
    }
  };
  fill(true, nt, &env_.node_weight_sums);
  fill(false, et, &env_.edge_weight_sums);
  std::set<std::string> labels;
  for (auto& m : metas)
    for (auto& l : m.graph_labels)
      if (!l.empty()) labels.insert(l);
  env_.graph_labels.assign(labels.begin(), labels.end());
  return Status::OK();
}

static std::string Cfg(const std::map<std::string, std::string>& c, const std::string& k, const std::string& d) {
  auto it = c.find(k);
  return it == c.end() ? d : it->second;
}

Status LoadOptionsFromConfig(const std::map<std::string, std::string>& config, LoadOptions* opt) {
  const std::string data = Cfg(config, "load_data_type", Cfg(config, "data_type", "all"));
  const std::string smp = Cfg(config, "global_sampler_type", Cfg(config, "sampler_type", "all"));
  return LoadOptions::Parse(data, smp, opt);
}

// registry watch (reference ZkServerMonitor child watch, zk_server_monitor.cc:186-200):
// re-list live entries every `period` seconds and swap each shard's replica set, so a
// server that stopped heartbeating is no longer routed to and a new replica is picked up
void QueryProxy::WatchRegistry(std::string spec, double ttl, double period) {
  std::unique_ptr<Registry> r = Registry::Open(spec);
  for (;;) {
    {
      std::unique_lock<std::mutex> l(watch_mu_);
      watch_cv_.wait_until(l, std::chrono::system_clock::now() +
                                  std::chrono::milliseconds(static_cast<int64_t>(period * 1000)),
                           [this] { return watch_stop_; });
      if (watch_stop_) return;
    }
    std::map<int, std::vector<std::pair<Endpoint, ShardMeta>>> listing;
    if (!r->List(&listing, ttl).ok()) continue;
    auto* rc = static_cast<RpcClients*>(clients_.get());
    for (auto& kv : listing) {
      std::vector<Endpoint> eps;
      for (auto& e : kv.second) eps.push_back(e.first);
      rc->UpdateShard(kv.first, eps);  // a shard with no live entry keeps its last replicas
    }
  }
}

Status QueryProxy::SetReplicas(int shard, const std::vector<std::string>& endpoints) {
  if (mode_ != "remote" && mode_ != "graph_partition") return Status::InvalidArgument("not a remote session");
  std::vector<Endpoint> eps;
  for (const auto& e : endpoints) {
    const size_t c = e.rfind(':');
    if (c == std::string::npos) return Status::InvalidArgument("endpoint must be host:port: " + e);
    Endpoint ep;
    ep.host = e.substr(0, c);
    ep.port = std::atoi(e.c_str() + c + 1);
    eps.push_back(ep);
  }
  static_cast<RpcClients*>(clients_.get())->UpdateShard(shard, eps);
  return Status::OK();
}

std::map<int, std::vector<std::string>> QueryProxy::Endpoints() const {
  if (mode_ != "remote" && mode_ != "graph_partition") return {};
  return static_cast<RpcClients*>(clients_.get())->Endpoints();
}

QueryProxy::~QueryProxy() {
  {
    std::lock_guard<std::mutex> l(watch_mu_);
    watch_stop_ = true;
  }
  watch_cv_.notify_all();
  if (watch_thread_.joinable()) watch_thread_.join();
}

Status QueryProxy::Init(const std::map<std::string, std::string>& config) {
  mode_ = Cfg(config, "mode", "local");
  int64_t seed;
  if (ParseInt64(Cfg(config, "seed", ""), &seed)) SetGlobalSeed(static_cast<uint64_t>(seed));
  pool_.reset(new ThreadPool(8, "euler-proxy"));
  LoadOptions lopt;
  EULER_RETURN_IF_ERROR(LoadOptionsFromConfig(config, &lopt));
  if (mode_ == "local") {
    // optional shard_idx / shard_num: this process loads only the partitions p with
    // p % shard_num == shard_idx (reference graph.cc:90-98), e.g. one data-parallel rank's
    // part of a graph row-sharded over the ranks' GPUs (graph/sharded_graph.py)
    int64_t sidx = 0, snum = 1;
    ParseInt64(Cfg(config, "shard_idx", "0"), &sidx);
    ParseInt64(Cfg(config, "shard_num", "1"), &snum);
    if (snum < 1 || sidx < 0 || sidx >= snum) return Status::InvalidArgument("local mode: bad shard_idx / shard_num");
    std::unique_ptr<Graph> g;
    std::unique_ptr<IndexManager> idx;
    EULER_RETURN_IF_ERROR(LoadShard(Cfg(config, "data_path", ""), static_cast<int>(sidx), static_cast<int>(snum), &g,
                                    &idx, 8, lopt));
    return InitWithGraph(std::move(g), std::move(idx));
  }
  int64_t shards = 1;
  if (mode_ == "local_sharded") {
    // S shards of one dataset inside this process, queried through the distribute compiler
    ParseInt64(Cfg(config, "shard_num", "2"), &shards);
    const std::string path = Cfg(config, "data_path", "");
    std::vector<EngineEnv*> envs;
    std::vector<ShardMeta> metas;
    for (int s = 0; s < shards; ++s) {
      std::unique_ptr<Graph> g;
      std::unique_ptr<IndexManager> idx;
      EULER_RETURN_IF_ERROR(LoadShard(path, s, static_cast<int>(shards), &g, &idx, 8, lopt));
      shard_envs_.push_back(MakeEnv(g.get(), idx.get(), static_cast<int>(shards)));
      envs.push_back(shard_envs_.back().get());
      metas.push_back(ShardMeta::FromEnv(*envs.back(), s, static_cast<int>(shards)));
      shard_graphs_.push_back(std::move(g));
      shard_indexes_.push_back(std::move(idx));
    }
    meta_ = shard_graphs_[0]->meta();
    clients_.reset(new InProcessShards(envs));
    env_.shard_num = static_cast<int>(shards);
    env_.num_partitions = std::max<uint32_t>(1, meta_.partitions_num);
    env_.index_info = metas[0].index_info;
    FillWeightTables(metas);
  } else if (mode_ == "remote" || mode_ == "graph_partition") {
    // graph_partition: the same shard cluster, but the shards hold arbitrary partitions
    // (reference query_proxy.cc:35-60 mode names); id-routed ops ask the shards who holds
    // each id first (CompileOptions::graph_partition), hop by hop, so results stay exact
    // (the reference's graph_partition plans run each query partition-locally instead)
    std::string reg = Cfg(config, "registry", Cfg(config, "zk_path", ""));
    if (reg.empty()) return Status::InvalidArgument(mode_ + " mode needs registry=<dir|memory:name>");
    auto r = Registry::Open(reg);
    std::map<int, std::vector<std::pair<Endpoint, ShardMeta>>> listing;
    int64_t want = 0;
    ParseInt64(Cfg(config, "shard_num", "0"), &want);
    double wait = 30, ttl = 10, refresh = 2;
    ParseDouble(Cfg(config, "wait_seconds", "30"), &wait);
    ParseDouble(Cfg(config, "registry_ttl", "10"), &ttl);        // entries not refreshed within ttl are dead
    ParseDouble(Cfg(config, "registry_refresh", "2"), &refresh);  // client re-list period (0: never)
    const double deadline = NowSec() + wait;
    for (;;) {
      EULER_RETURN_IF_ERROR(r->List(&listing, ttl));
      int expect = static_cast<int>(want);
      if (!listing.empty() && expect == 0) expect = listing.begin()->second.front().second.shard_num;
      if (expect > 0 && static_cast<int>(listing.size()) >= expect) break;
      if (NowSec() > deadline) return Status::Unavailable("timed out waiting for graph servers in " + reg);
      std::this_thread::sleep_for(std::chrono::milliseconds(100));
    }
    ClientOptions co;
    int64_t x;
    if (ParseInt64(Cfg(config, "num_retries", "10"), &x)) co.num_retries = static_cast<int>(x);
    if (ParseInt64(Cfg(config, "num_channels_per_host", "4"), &x)) co.num_channels_per_host = static_cast<int>(x);
    ParseDouble(Cfg(config, "bad_host_timeout", "10"), &co.bad_host_timeout);
    std::map<int, std::vector<Endpoint>> eps;
    std::vector<ShardMeta> metas;
    for (auto& kv : listing) {
      for (auto& e : kv.second) eps[kv.first].push_back(e.first);
      metas.push_back(kv.second.front().second);
    }
    clients_.reset(new RpcClients(eps, co));
    if (refresh > 0) watch_thread_ = std::thread([this, reg, ttl, refresh] { WatchRegistry(reg, ttl, refresh); });
    shards = static_cast<int64_t>(listing.size());
    env_.shard_num = static_cast<int>(shards);
    env_.num_partitions = std::max<uint32_t>(1, metas[0].num_partitions);
    env_.index_info = metas[0].index_info;
    meta_.Parse(metas[0].graph_meta.data(), metas[0].graph_meta.size());
    FillWeightTables(metas);
  } else {
    return Status::InvalidArgument("unknown mode " + mode_);
  }
  env_.clients = clients_.get();
  copt_.mode = CompileMode::kDistribute;
  copt_.shard_num = env_.shard_num;
  copt_.graph_partition = mode_ == "graph_partition";
  {
    const char* f = std::getenv("EULER_GQL_FUSE");
    copt_.fuse = !(f && f[0] == '0');
  }
  copt_.neighbor_indexes.clear();
  for (auto& item : Split(env_.index_info, ",")) {
    auto p = Split(item, ":");
    if (p.size() == 2 && p[1] == "hash_range_index") copt_.neighbor_indexes.push_back(p[0]);
  }
  return Status::OK();
}

Status QueryProxy::InitWithGraph(std::unique_ptr<Graph> g, std::unique_ptr<IndexManager> idx) {
  mode_ = "local";
  graph_ = std::move(g);
  index_ = idx ? std::move(idx) : std::unique_ptr<IndexManager>(new IndexManager);
  auto e = MakeEnv(graph_.get(), index_.get(), 1);
  env_ = *e;
  meta_ = graph_->meta();
  ShardMeta m = ShardMeta::FromEnv(env_, 0, 1);
  FillWeightTables({m});
  copt_.mode = CompileMode::kLocal;
  copt_.shard_num = 1;
  return Status::OK();
}

Status QueryProxy::Run(const std::string& gql, const std::vector<std::pair<std::string, Tensor>>& inputs,
                       const std::vector<std::string>& outputs, std::vector<Tensor>* results) {
  auto& ctr = EngineCounters::Get();
  ctr.queries.fetch_add(1, std::memory_order_relaxed);
  std::shared_ptr<const DAGDef> dag;
  {
    ScopedMicros t(&ctr.compile_us);
    EULER_RETURN_IF_ERROR(Compiler::Get().Compile(gql, copt_, &dag));
  }
  ScopedMicros t(&ctr.exec_us);
  return ExecuteDag(&env_, *dag, inputs, outputs, results);
}

Status QueryProxy::RunOp(const std::string& op, const std::vector<std::string>& input_names,
                         const std::vector<std::string>& attrs, int output_num,
                         const std::vector<std::pair<std::string, Tensor>>& inputs, std::vector<Tensor>* results) {
  DAGDef logical;
  NodeDef nd;
  nd.op = op;
  nd.id = 1;
  nd.inputs = input_names;
  nd.attrs = attrs;
  nd.output_num = output_num;
  NodeDef as;
  as.op = "AS";
  as.id = 2;
  as.attrs = {"__result"};
  for (int k = 0; k < output_num; ++k) as.inputs.push_back(nd.Output(k));
  logical.nodes = {nd, as};
  auto& ctr = EngineCounters::Get();
  ctr.queries.fetch_add(1, std::memory_order_relaxed);
  DAGDef phys;
  {
    ScopedMicros t(&ctr.compile_us);
    EULER_RETURN_IF_ERROR(Compiler::Get().Optimize(logical, copt_, &phys));
  }
  std::vector<std::string> outs;
  for (int k = 0; k < output_num; ++k) outs.push_back("__result:" + std::to_string(k));
  ScopedMicros t(&ctr.exec_us);
  return ExecuteDag(&env_, phys, inputs, outs, results);
}

Status QueryProxy::RunOnShard(int shard, const std::string& op, const std::vector<std::string>& attrs,
                              int output_num, std::vector<Tensor>* results) {
  DAGDef dag;
  NodeDef nd;
  nd.op = op;
  nd.id = 1;
  nd.attrs = attrs;
  nd.output_num = output_num;
  dag.nodes = {nd};
  std::vector<std::string> outs;
  for (int k = 0; k < output_num; ++k) outs.push_back(nd.Output(k));
  if (mode_ == "remote") {
    if (!clients_ || shard < 0 || shard >= clients_->num_shards()) return Status::InvalidArgument("no such shard");
    std::promise<std::pair<Status, std::vector<Tensor>>> pr;
    auto fut = pr.get_future();
    clients_->Execute(shard, dag, {}, outs, [&pr](Status st, std::vector<Tensor> t) {
      pr.set_value({st, std::move(t)});
    });
    auto r = fut.get();
    if (!r.first.ok()) return r.first;
    *results = std::move(r.second);
    return Status::OK();
  }
  if (mode_ == "local_sharded") {
    if (shard < 0 || shard >= static_cast<int>(shard_envs_.size())) return Status::InvalidArgument("no such shard");
    return ExecuteDag(shard_envs_[shard].get(), dag, {}, outs, results);
  }
  if (shard != 0 || !graph_) return Status::InvalidArgument("local mode has one shard (0)");
  return ExecuteDag(&env_, dag, {}, outs, results);
}

Status QueryProxy::Explain(const std::string& gql, std::string* out) {
  std::shared_ptr<const DAGDef> dag;
  EULER_RETURN_IF_ERROR(Compiler::Get().Compile(gql, copt_, &dag));
  *out = dag->DebugString();
  return Status::OK();
}

}  // namespace euler
