// Native remote console: an interactive client against a live graph (remote shards through
// the registry, or an embedded graph directory), built on the same QueryProxy as the
// Python API.  Reference: euler/tools/remote_console/remote_console.cc:27-157 (query_nb,
// query_sp_fea, query_dense_fea over QueryProxy; ZooKeeper address read from stdin).
//
//   remote_console --registry=/shared/reg --shard_num=2        (remote shards)
//   remote_console --data_path=/data/euler                      (embedded graph)
//
// Commands (one per line):
//   query_nb <id> <edge_type>            full out-neighbours: ids, weights, types
//   sample_nb <id> <edge_type> <count>   weighted neighbour sampling
//   query_sp_fea <id> <feature>          sparse feature values
//   query_dense_fea <id> <feature>       dense feature values
//   query_bin_fea <id> <feature>         binary feature bytes
//   gql <query> [-- name=v1,v2 ...]      any GQL query; inputs are uint64 lists
//   explain <query>                      the compiled physical DAG
//   meta | help | quit
#include <unistd.h>

#include <cstdio>
#include <iostream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "framework/framework.h"
#include "rpc/rpc.h"

using euler::QueryProxy;
using euler::Status;
using euler::Tensor;

namespace {

const char* kHelp =
    "query_nb <id> <edge_type> | sample_nb <id> <edge_type> <count> | query_sp_fea <id> <feature> |\n"
    "query_dense_fea <id> <feature> | query_bin_fea <id> <feature> | gql <query> [-- name=v1,v2 ...] |\n"
    "explain <query> | meta | help | quit\n";

std::vector<std::string> Split(const std::string& s) {
  std::istringstream in(s);
  std::vector<std::string> out;
  std::string w;
  while (in >> w) out.push_back(w);
  return out;
}

void Print(const std::string& label, const Tensor& t) {
  std::printf("%s:", label.c_str());
  if (!t.defined()) {
    std::printf(" <none>\n");
    return;
  }
  if (t.dtype() == euler::DType::kString) {
    for (const auto& s : t.strings()) std::printf(" %s", s.c_str());
  } else if (t.dtype() == euler::DType::kFloat || t.dtype() == euler::DType::kDouble) {
    for (int64_t i = 0; i < t.numel(); ++i) std::printf(" %g", t.AsDouble(i));
  } else if (t.dtype() == euler::DType::kUInt64) {
    for (uint64_t v : t.ToUInt64()) std::printf(" %llu", static_cast<unsigned long long>(v));
  } else {
    for (int64_t i = 0; i < t.numel(); ++i) std::printf(" %lld", static_cast<long long>(t.AsInt(i)));
  }
  std::printf("\n");
}

int EdgeType(const QueryProxy& qp, const std::string& s) {
  const int id = qp.meta().EdgeTypeId(s);
  if (id >= 0) return id;
  return std::atoi(s.c_str());
}

bool Run(QueryProxy* qp, const std::string& gql, const std::vector<std::pair<std::string, Tensor>>& inputs,
         const std::vector<std::string>& outputs, const std::vector<std::string>& labels) {
  std::vector<Tensor> res;
  const Status s = qp->Run(gql, inputs, outputs, &res);
  if (!s.ok()) {
    std::printf("error: %s\n", s.ToString().c_str());
    return false;
  }
  for (size_t i = 0; i < res.size() && i < labels.size(); ++i) Print(labels[i], res[i]);
  return true;
}

Tensor Ids(const std::string& s) { return Tensor::FromVector<uint64_t>({std::strtoull(s.c_str(), nullptr, 10)}); }

// one command; false on quit
bool Handle(QueryProxy* qp, const std::string& line) {
  const std::vector<std::string> a = Split(line);
  if (a.empty()) return true;
  const std::string& cmd = a[0];
  if (cmd == "quit" || cmd == "exit") return false;
  if (cmd == "help") {
    std::printf("%s", kHelp);
  } else if (cmd == "meta") {
    std::printf("%s\n", qp->meta().ToString().c_str());
  } else if ((cmd == "query_nb" && a.size() == 3) || (cmd == "sample_nb" && a.size() == 4)) {
    std::vector<std::pair<std::string, Tensor>> in = {
        {"nodes", Ids(a[1])}, {"edge_types", Tensor::FromVector<int32_t>({EdgeType(*qp, a[2])})}};
    std::string q = "v(nodes).outV(edge_types).as(nb)";
    if (cmd == "sample_nb") {
      in.emplace_back("nb_count", Tensor::FromVector<int64_t>({std::atoll(a[3].c_str())}));
      q = "v(nodes).sampleNB(edge_types, nb_count, -1).as(nb)";
    }
    Run(qp, q, in, {"nb:1", "nb:2", "nb:3"}, {"nb", "weights", "types"});
  } else if ((cmd == "query_sp_fea" || cmd == "query_dense_fea" || cmd == "query_bin_fea") && a.size() == 3) {
    const std::string prefix = cmd == "query_sp_fea" ? "sparse_" : (cmd == "query_dense_fea" ? "dense_" : "binary_");
    Run(qp, "v(nodes).values(__f0).as(fea)", {{"nodes", Ids(a[1])}, {"__f0", Tensor::Strings({prefix + a[2]})}},
        {"fea:1"}, {"feature"});
  } else if (cmd == "explain" && a.size() >= 2) {
    std::string out;
    const Status s = qp->Explain(line.substr(line.find(a[1])), &out);
    std::printf("%s\n", s.ok() ? out.c_str() : ("error: " + s.ToString()).c_str());
  } else if (cmd == "gql" && a.size() >= 2) {
    // gql <query> [-- name=v1,v2 ...]; outputs: every slot of every alias is printed
    const size_t sep = line.find(" -- ");
    const std::string q = line.substr(line.find(a[1]), sep == std::string::npos ? std::string::npos
                                                                                  : sep - line.find(a[1]));
    std::vector<std::pair<std::string, Tensor>> in;
    if (sep != std::string::npos) {
      for (const std::string& kv : Split(line.substr(sep + 4))) {
        const size_t eq = kv.find('=');
        if (eq == std::string::npos) continue;
        std::vector<uint64_t> vals;
        std::stringstream vs(kv.substr(eq + 1));
        std::string item;
        while (std::getline(vs, item, ',')) vals.push_back(std::strtoull(item.c_str(), nullptr, 10));
        in.emplace_back(kv.substr(0, eq), Tensor::FromVector<uint64_t>(vals));
      }
    }
    // aliases: every ".as(x)" in the query; print slots 0..3 of each until one is missing
    std::vector<std::string> outs, labels;
    for (size_t p = q.find(".as("); p != std::string::npos; p = q.find(".as(", p + 1)) {
      const std::string alias = q.substr(p + 4, q.find(')', p) - p - 4);
      for (int k = 0; k < 4; ++k) {
        outs.push_back(alias + ":" + std::to_string(k));
        labels.push_back(alias + ":" + std::to_string(k));
      }
    }
    std::vector<Tensor> res;
    const Status s = qp->Run(q, in, outs, &res);
    if (!s.ok()) {
      // fewer slots than 4 for some alias: retry with slots 0..1
      outs.clear();
      labels.clear();
      for (size_t p = q.find(".as("); p != std::string::npos; p = q.find(".as(", p + 1)) {
        const std::string alias = q.substr(p + 4, q.find(')', p) - p - 4);
        for (int k = 0; k < 2; ++k) outs.push_back(alias + ":" + std::to_string(k));
      }
      labels = outs;
      Run(qp, q, in, outs, labels);
    } else {
      for (size_t i = 0; i < res.size(); ++i) Print(labels[i], res[i]);
    }
  } else {
    std::printf("unknown or malformed command; %s", kHelp);
  }
  std::fflush(stdout);
  return true;
}

}  // namespace

int main(int argc, char** argv) {
  euler::LinkGraphOps();
  euler::LinkDistOps();
  euler::LinkRemoteOp();
  std::map<std::string, std::string> cfg;
  for (int i = 1; i < argc; ++i) {
    std::string arg = argv[i];
    if (arg.rfind("--", 0) != 0) continue;
    arg = arg.substr(2);
    const size_t eq = arg.find('=');
    if (eq != std::string::npos) {
      cfg[arg.substr(0, eq)] = arg.substr(eq + 1);
    } else if (i + 1 < argc) {
      cfg[arg] = argv[++i];
    }
  }
  if (!cfg.count("mode")) cfg["mode"] = cfg.count("registry") || cfg.count("zk_path") ? "remote" : "local";
  QueryProxy qp;
  const Status s = qp.Init(cfg);
  if (!s.ok()) {
    std::fprintf(stderr, "remote_console: init failed: %s\n", s.ToString().c_str());
    return 1;
  }
  const bool tty = isatty(0);
  std::string line;
  while (true) {
    if (tty) {
      std::printf("euler> ");
      std::fflush(stdout);
    }
    if (!std::getline(std::cin, line)) break;
    if (!Handle(&qp, line)) break;
  }
  return 0;
}
