// euler_amd engine — GQL (Gremlin-like query language) compiler.
//
//   Parse      hand-written lexer + recursive-descent parser (no flex/bison, no global
//              parser state, errors are returned — the reference exit(1)s on a syntax
//              error, gremlin.y:272-276) producing a chain of steps;
//   Translate  steps -> logical DAG of API_* ops + AS alias nodes + client-side
//              POST_PROCESS / API_GET_NB_FILTER (reference translator.cc);
//   Optimize   local mode: as is.  distribute mode: every shardable API op becomes
//              split -> REMOTE x shard_num -> merge following the reference's rule table
//              (compiler.cc:37-573): ID_SPLIT / BROAD_CAST_SPLIT / SAMPLE_*_SPLIT,
//              APPEND / IDX+DATA / REGULAR_DATA / MULTI_TYPE merges, ID_UNIQUE + gathers
//              before neighbor / feature RPCs, then CSE of identical splits.
//   Compile    cached by (query, mode) behind a mutex; DAGs are immutable once cached.
#pragma once

#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

#include "framework/framework.h"

namespace euler {

struct GqlStep {
  std::string op;                       // v e sampleN sampleNWithTypes sampleE outV inV outE sampleNB sampleLNB
                                        // values label select v_select udf
  std::vector<std::string> params;
  std::vector<std::string> udf_params;  // [..] numeric list for udfs
  std::vector<std::string> dnf;         // conjunction strings "f op v,f op v"
  std::vector<std::string> post;        // "order_by id asc", "limit 2"
  std::string alias;
};

Status ParseGql(const std::string& query, std::vector<GqlStep>* steps);

enum class CompileMode { kLocal = 0, kDistribute = 1 };

struct CompileOptions {
  CompileMode mode = CompileMode::kLocal;
  int shard_num = 1;
  // names of neighbor (hash_range) indexes: conditions on them stay on the shard
  std::vector<std::string> neighbor_indexes;
  // fuse independent REMOTE nodes of a shard into one RPC (reference FusionAndShardRule,
  // compiler.cc:92-162 / DAGDef::FusionNodes, dag_def.cc:128-203); EULER_GQL_FUSE=0 disables
  bool fuse = true;
  // graph_partition mode: shards hold arbitrary partitions (e.g. a min-cut partitioner's),
  // not id-hash ones; id-routed ops first ask every shard which ids it holds
  // (API_GET_NODE_T != -1) and route each id to its owner (GP_ID_SPLIT)
  bool graph_partition = false;
};

// REMOTE fusion pass of the distribute-mode optimizer (exposed for tests)
void FuseRemoteNodes(DAGDef* dag);

class Compiler {
 public:
  static Compiler& Get();
  Status Compile(const std::string& query, const CompileOptions& opt, std::shared_ptr<const DAGDef>* dag);
  // logical translation only (exposed for tests / explain)
  Status Translate(const std::vector<GqlStep>& steps, const CompileOptions& opt, DAGDef* dag);
  Status Optimize(const DAGDef& logical, const CompileOptions& opt, DAGDef* physical);
  void ClearCache();

 private:
  std::mutex mu_;
  std::map<std::string, std::shared_ptr<const DAGDef>> cache_;
};

}  // namespace euler
