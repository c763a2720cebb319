// euler_amd engine — graph-plane RPC, service discovery and the query session
// (§5 failure detection).
//
// Transport: length-prefixed binary frames over TCP (no gRPC / protobuf dependency):
//   frame  = u32 magic 'EULR' | u32 kind | u64 payload bytes | payload
//   EXECUTE  payload = DAGDef | u32 n (name, Tensor)* | u32 m output-names*
//            reply   = i32 code | message | u32 m Tensor*
//   PING / META (shard meta as "k=v" lines)
// Server: accept thread + one thread per connection; DAGs run on a compute pool.
// Client: per shard a list of replica endpoints, a small connection pool per
// endpoint, retry on the next replica up to num_retries, bad-host quarantine for
// bad_host_timeout seconds (reference rpc_client.cc:30-57, rpc_manager.cc:57-138).
// Fault injection: EULER_RPC_FAULT_RATE=<p> fails a fraction p of calls before
// sending, EULER_RPC_FAULT_DELAY_MS=<ms> delays every call.
//
// Discovery (replaces ZooKeeper): a registry directory where each server writes
// "<shard>#<host>:<port>" files holding its shard meta, or an in-process memory
// registry for tests.  Servers remove their entry on Stop().
#pragma once

#include <atomic>
#include <condition_variable>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "framework/framework.h"
#include "gql/gql.h"
#include "graph/graph.h"
#include "index/index.h"

namespace euler {

// ============================================================================ remote execution interface
class RemoteClients {
 public:
  virtual ~RemoteClients() = default;
  virtual int num_shards() const = 0;
  using Done = std::function<void(Status, std::vector<Tensor>)>;
  virtual void Execute(int shard, const DAGDef& dag, std::vector<std::pair<std::string, Tensor>> inputs,
                       std::vector<std::string> outputs, Done done) = 0;
};

// Shards living in this process (single-node multi-shard and tests of distribute mode).
class InProcessShards : public RemoteClients {
 public:
  explicit InProcessShards(std::vector<EngineEnv*> shard_envs) : envs_(std::move(shard_envs)) {}
  int num_shards() const override { return static_cast<int>(envs_.size()); }
  void Execute(int shard, const DAGDef& dag, std::vector<std::pair<std::string, Tensor>> inputs,
               std::vector<std::string> outputs, Done done) override;

 private:
  std::vector<EngineEnv*> envs_;
};

// Run a (sub-)DAG against an engine env and fetch named outputs (server side of EXECUTE).
Status ExecuteDag(EngineEnv* env, const DAGDef& dag, const std::vector<std::pair<std::string, Tensor>>& inputs,
                  const std::vector<std::string>& outputs, std::vector<Tensor>* results);

// ============================================================================ shard meta / registry
struct ShardMeta {
  int shard_idx = 0, shard_num = 1;
  uint32_t num_partitions = 1;
  std::vector<double> node_weight_sums, edge_weight_sums;  // per type
  std::vector<std::string> graph_labels;
  std::string index_info;
  std::string graph_meta;  // serialized euler.meta
  std::string ToString() const;
  static bool Parse(const std::string& s, ShardMeta* m);
  static ShardMeta FromEnv(const EngineEnv& env, int shard_idx, int shard_num);
};

struct Endpoint {
  std::string host;
  int port = 0;
  std::string ToString() const { return host + ":" + std::to_string(port); }
};

// Service discovery (reference ZK registry: zk_server_register.cc / zk_server_monitor.cc).
// Liveness replaces ZooKeeper's ephemeral nodes: a server refreshes its entry every
// heartbeat (Heartbeat; NOT_FOUND -> the server registers again, the analog of
// re-registering after a session expiry) and List(ttl) skips entries not refreshed within
// ttl seconds, so a SIGKILLed server drops out of every client's view.
class Registry {
 public:
  virtual ~Registry() = default;
  virtual Status Register(int shard, const Endpoint& ep, const ShardMeta& meta) = 0;
  virtual Status Deregister(int shard, const Endpoint& ep) = 0;
  virtual Status Heartbeat(int shard, const Endpoint& ep) = 0;
  // shard -> live replicas (ttl <= 0: every entry)
  virtual Status List(std::map<int, std::vector<std::pair<Endpoint, ShardMeta>>>* out, double ttl = 0) = 0;
  // "file:<dir>" | "<dir>" | "memory:<name>" | "tcp://<host>:<port>" (RegistryServer)
  static std::unique_ptr<Registry> Open(const std::string& spec);
};

// Network registry service (the reference's ZooKeeper ensemble role, zk_server_register.cc /
// zk_server_monitor.cc) for deployments without a shared filesystem: one small process
// holds the shard -> replica table; servers register and heartbeat over TCP
// (Registry::Open("tcp://host:port")), clients list with a TTL exactly like the file
// registry.  Requests are single frames of the RPC wire format on short connections.
class RegistryServer {
 public:
  explicit RegistryServer(int port = 0);
  ~RegistryServer();
  Status Start();
  void Stop();
  int port() const { return port_; }
  size_t size();

 private:
  void Loop();
  std::string Handle(uint32_t kind, const std::string& payload);
  struct Entry {
    int shard;
    Endpoint ep;
    std::string meta;
    double seen;
  };
  int port_req_, port_ = 0, fd_ = -1;
  std::atomic<bool> running_{false};
  std::thread th_;
  std::mutex mu_;
  std::map<std::string, Entry> entries_;
};

// ============================================================================ server
struct ServerOptions {
  int port = 0;  // 0: ephemeral
  std::string host;  // advertised host (default: 127.0.0.1)
  int num_threads = 32;   // DAG execution workers
  int io_threads = 2;     // epoll event loops (connections are spread over them)
  std::string registry;  // optional
  int heartbeat_ms = 1000;  // registry entry refresh period
};

class GraphServer {
 public:
  GraphServer(EngineEnv* env, int shard_idx, int shard_num, const ServerOptions& opt);
  ~GraphServer();
  Status Start();
  void Stop();
  int port() const { return port_; }
  Endpoint endpoint() const { return {host_, port_}; }
  int64_t requests() const { return requests_.load(); }

 private:
  struct Conn;
  struct Loop;
  void AcceptLoop(int listen_fd);
  void RunLoop(Loop* lp);
  void OnReadable(Loop* lp, const std::shared_ptr<Conn>& c);
  void Dispatch(Loop* lp, const std::shared_ptr<Conn>& c);
  void Flush(Loop* lp, const std::shared_ptr<Conn>& c);
  void Drop(Loop* lp, const std::shared_ptr<Conn>& c);
  std::string Handle(uint32_t kind, const std::string& payload);
  void HandleExecute(const std::string& payload, Status* st, std::vector<Tensor>* res);
  EngineEnv* env_;
  int shard_idx_, shard_num_;
  ServerOptions opt_;
  std::string host_;
  int listen_fd_ = -1, port_ = 0;
  int local_fd_ = -1;  // Unix-domain (abstract namespace) listener for same-host clients
  std::atomic<bool> running_{false};
  std::thread accept_thread_, local_accept_thread_;
  std::vector<std::unique_ptr<Loop>> loops_;
  std::atomic<uint64_t> next_loop_{0};
  std::unique_ptr<ThreadPool> pool_;
  std::unique_ptr<Registry> registry_;
  std::thread heartbeat_thread_;
  std::mutex hb_mu_;
  std::condition_variable hb_cv_;
  std::atomic<int64_t> requests_{0};
};

// ============================================================================ client
struct ClientOptions {
  int num_retries = 10;           // reference kRpcRetryCount
  double bad_host_timeout = 10.0;  // seconds
  int num_channels_per_host = 4;
  int timeout_ms = 60000;
};

class RpcClients : public RemoteClients {
 public:
  RpcClients(std::map<int, std::vector<Endpoint>> shards, const ClientOptions& opt);
  ~RpcClients() override;
  int num_shards() const override { return static_cast<int>(shards_.size()); }
  // replace the replicas of a shard (registry watch); hosts still present keep their pools
  void UpdateShard(int shard, const std::vector<Endpoint>& eps);
  std::map<int, std::vector<std::string>> Endpoints() const;
  void Execute(int shard, const DAGDef& dag, std::vector<std::pair<std::string, Tensor>> inputs,
               std::vector<std::string> outputs, Done done) override;
  Status Ping(int shard);
  Status FetchMeta(int shard, ShardMeta* meta);
  int64_t failures() const { return failures_.load(); }

 private:
  // a pooled connection; same-host (Unix socket) channels also carry a shared-memory
  // region for large payloads
  struct Chan {
    int fd = -1;
    char* shm = nullptr;
    size_t cap = 0;
  };
  // A replica.  Dropped from the routing set by UpdateShard, it lives on while a call
  // holds a snapshot of the old list (that call still returns its channel here), and
  // its destructor closes every pooled channel (socket + shared region).
  struct Host {
    Endpoint ep;
    std::mutex mu;
    std::vector<Chan> idle;  // pooled connected sockets
    double bad_until = 0;
    ~Host() {
      for (auto& c : idle) CloseChan(&c);
    }
  };
  static Chan OpenChan(const Endpoint& ep, int timeout_ms);
  static void CloseChan(Chan* c);
  typedef std::vector<std::shared_ptr<Host>> HostList;
  // transport status; with `decoded`, the reply is decoded in place (straight out of the
  // shared region when it came that way) and the server's status lands in *app
  Status Call(int shard, uint32_t kind, const std::string& payload, std::string* reply,
              std::vector<Tensor>* decoded = nullptr, Status* app = nullptr);
  Status CallHost(Host* h, uint32_t kind, const std::string& payload, std::string* reply, size_t* in_bytes,
                  std::vector<Tensor>* decoded, Status* app);
  // per shard, swapped atomically by UpdateShard (callers work on a snapshot)
  std::vector<std::shared_ptr<const HostList>> shards_;
  std::vector<std::atomic<uint64_t>> rr_;
  ClientOptions opt_;
  std::unique_ptr<ThreadPool> pool_;
  std::atomic<int64_t> failures_{0};
};

// ============================================================================ session (reference QueryProxy)
class QueryProxy {
 public:
  // config keys: mode (local | remote | local_sharded), data_path, shard_num, registry/zk_path,
  // num_retries, bad_host_timeout, num_channels_per_host, seed, load_data_type
  Status Init(const std::map<std::string, std::string>& config);
  // adopt a graph built in-process (Python builder / synthetic generator)
  Status InitWithGraph(std::unique_ptr<Graph> g, std::unique_ptr<IndexManager> idx);
  Status Run(const std::string& gql, const std::vector<std::pair<std::string, Tensor>>& inputs,
             const std::vector<std::string>& outputs, std::vector<Tensor>* results);
  Status Explain(const std::string& gql, std::string* out);
  // one op against ONE shard's own data (no compiler rewrite, no split / merge): local mode
  // runs it on the in-process graph (shard 0), local_sharded on that shard's env, remote
  // mode over that shard's RPC replicas
  Status RunOnShard(int shard, const std::string& op, const std::vector<std::string>& attrs, int output_num,
                    std::vector<Tensor>* results);
  // single-op query (reference Query(op, alias, n_out, inputs, attrs)), sharded like a GQL step
  Status RunOp(const std::string& op, const std::vector<std::string>& input_names,
               const std::vector<std::string>& attrs, int output_num,
               const std::vector<std::pair<std::string, Tensor>>& inputs, std::vector<Tensor>* results);
  const GraphMeta& meta() const { return meta_; }
  Graph* local_graph() const { return graph_.get(); }
  IndexManager* index() const { return index_.get(); }
  EngineEnv* env() { return &env_; }
  const std::string& mode() const { return mode_; }
  int shard_num() const { return env_.shard_num; }
  // run a DAG in-process against a shard env (used by the local fast paths)
  static std::unique_ptr<EngineEnv> MakeEnv(Graph* g, IndexManager* idx, int shard_num);
  // remote mode: current replicas per shard as the client routes to them
  // replace a shard's replica set (what the registry watch does; remote mode only)
  Status SetReplicas(int shard, const std::vector<std::string>& endpoints);
  std::map<int, std::vector<std::string>> Endpoints() const;
  ~QueryProxy();

 private:
  Status FillWeightTables(const std::vector<ShardMeta>& metas);
  void WatchRegistry(std::string spec, double ttl, double period);
  std::thread watch_thread_;
  std::mutex watch_mu_;
  std::condition_variable watch_cv_;
  bool watch_stop_ = false;
  std::string mode_ = "local";
  CompileOptions copt_;
  EngineEnv env_;
  GraphMeta meta_;
  std::unique_ptr<Graph> graph_;
  std::unique_ptr<IndexManager> index_;
  // local_sharded
  std::vector<std::unique_ptr<Graph>> shard_graphs_;
  std::vector<std::unique_ptr<IndexManager>> shard_indexes_;
  std::vector<std::unique_ptr<EngineEnv>> shard_envs_;
  std::unique_ptr<RemoteClients> clients_;
  std::unique_ptr<ThreadPool> pool_;
};

// Load one shard (graph + indexes) from a reference-format directory; opt selects the
// node / edge tables and the global samplers (load_data_type / global_sampler_type).
Status LoadShard(const std::string& data_path, int shard_idx, int shard_num, std::unique_ptr<Graph>* g,
                 std::unique_ptr<IndexManager>* idx, int threads = 8, const LoadOptions& opt = LoadOptions());
// LoadOptions from config keys load_data_type / global_sampler_type (aliases data_type /
// sampler_type, the names initialize_embedded_graph uses)
Status LoadOptionsFromConfig(const std::map<std::string, std::string>& config, LoadOptions* opt);

}  // namespace euler
