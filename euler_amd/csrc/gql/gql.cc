#include "gql/gql.h"

#include <algorithm>
#include <functional>
#include <set>
#include <unordered_map>

namespace euler {

// ============================================================================ lexer
// Separators: whitespace ( ) . , ; — '[' and ']' are kept as tokens (udf numeric
// parameter lists).  This mirrors the reference lexer (gremlin.l:13-53) where the
// structure comes from keywords, not from punctuation.
static std::vector<std::string> Lex(const std::string& q) {
  std::vector<std::string> toks;
  std::string cur;
  auto flush = [&] {
    if (!cur.empty()) toks.push_back(cur);
    cur.clear();
  };
  for (size_t i = 0; i < q.size(); ++i) {
    const char c = q[i];
    if (isspace(static_cast<unsigned char>(c)) || c == '(' || c == ')' || c == ',' || c == ';') {
      flush();
    } else if (c == '.') {
      // '.' separates steps, except inside a number (e.g. 1.5) or a negative literal
      const bool in_number = !cur.empty() && (isdigit(static_cast<unsigned char>(cur.back()))) &&
                             i + 1 < q.size() && isdigit(static_cast<unsigned char>(q[i + 1])) &&
                             std::all_of(cur.begin(), cur.end(), [](char x) { return isdigit(static_cast<unsigned char>(x)) || x == '-'; });
      if (in_number) cur.push_back(c);
      else flush();
    } else if (c == '[' || c == ']') {
      flush();
      toks.push_back(std::string(1, c));
    } else {
      cur.push_back(c);
    }
  }
  flush();
  return toks;
}

static const std::set<std::string>& StepKeywords() {
  static const std::set<std::string> k = {"v", "e", "sampleN", "sampleNWithTypes", "sampleE", "select", "v_select",
                                          "outV", "inV", "outE", "sampleNB", "sampleLNB", "values", "label",
                                          "sampleNodeAt"};
  return k;
}

static bool IsUdf(const std::string& t) {
  return StartsWith(t, "udf_") || t == "mean" || t == "min" || t == "max";
}

static bool IsKeyword(const std::string& t) {
  static const std::set<std::string> k = {"has", "hasKey", "hasLabel", "and", "or", "order_by", "limit", "as",
                                          "[", "]"};
  return StepKeywords().count(t) || k.count(t) || IsUdf(t);
}

Status ParseGql(const std::string& query, std::vector<GqlStep>* steps) {
  steps->clear();
  auto toks = Lex(query);
  size_t i = 0;
  const size_t n = toks.size();
  auto err = [&](const std::string& m) {
    return Status::InvalidArgument("GQL syntax error near token " + std::to_string(i) + " ('" +
                                   (i < n ? toks[i] : std::string("<end>")) + "'): " + m + " in: " + query);
  };
  std::vector<std::string> conj;  // terms of the conjunction being built
  auto cur = [&]() -> GqlStep* { return steps->empty() ? nullptr : &steps->back(); };
  auto close_conj = [&] {
    if (!conj.empty() && cur()) cur()->dnf.push_back(Join(conj, ","));
    conj.clear();
  };
  while (i < n) {
    const std::string& t = toks[i];
    if (StepKeywords().count(t)) {
      close_conj();
      GqlStep s;
      s.op = t;
      ++i;
      while (i < n && !IsKeyword(toks[i])) s.params.push_back(toks[i++]);
      steps->push_back(s);
      continue;
    }
    if (!cur()) return err("query must start with a root step (v, e, sampleN, sampleNWithTypes, sampleE)");
    if (t == "has") {
      if (i + 3 >= n) return err("has() needs <field> <op> <value>");
      conj.push_back(toks[i + 1] + " " + toks[i + 2] + " " + toks[i + 3]);
      i += 4;
    } else if (t == "hasLabel") {
      if (i + 1 >= n) return err("hasLabel() needs a label");
      conj.push_back("node_type eq " + toks[i + 1]);
      i += 2;
    } else if (t == "hasKey") {
      if (i + 1 >= n) return err("hasKey() needs a key");
      conj.push_back(toks[i + 1] + " not_in __euler_none__");
      i += 2;
    } else if (t == "and") {
      ++i;
    } else if (t == "or") {
      close_conj();
      ++i;
    } else if (t == "order_by") {
      close_conj();
      if (i + 1 >= n) return err("order_by needs a field");
      std::string dir = "asc";
      size_t k = i + 2;
      if (k < n && (toks[k] == "asc" || toks[k] == "desc")) {
        dir = toks[k];
        ++k;
      }
      cur()->post.push_back("order_by " + toks[i + 1] + " " + dir);
      i = k;
    } else if (t == "limit") {
      close_conj();
      if (i + 1 >= n) return err("limit needs a count");
      cur()->post.push_back("limit " + toks[i + 1]);
      i += 2;
    } else if (t == "as") {
      close_conj();
      if (i + 1 >= n) return err("as() needs an alias");
      cur()->alias = toks[i + 1];
      i += 2;
    } else if (IsUdf(t)) {
      close_conj();
      if (cur()->op != "values") return err("a udf must follow values()");
      GqlStep u;
      u.op = "udf";
      u.params.push_back(StartsWith(t, "udf_") ? t : "udf_" + t);
      ++i;
      while (i < n && !IsKeyword(toks[i])) u.params.push_back(toks[i++]);
      if (i < n && toks[i] == "[") {
        ++i;
        while (i < n && toks[i] != "]") u.udf_params.push_back(toks[i++]);
        if (i >= n) return err("unterminated udf parameter list");
        ++i;
      }
      // attach to the values step
      GqlStep& vs = *cur();
      vs.udf_params = u.udf_params;
      vs.params.push_back("__udf__=" + u.params[0]);
      for (size_t k = 1; k < u.params.size(); ++k) vs.params.push_back("__udfarg__=" + u.params[k]);
    } else {
      return err("unexpected token");
    }
  }
  close_conj();
  if (steps->empty()) return err("empty query");
  const std::string& root = steps->front().op;
  if (root != "v" && root != "e" && root != "sampleN" && root != "sampleNWithTypes" && root != "sampleE")
    return Status::InvalidArgument("GQL: query must start with v/e/sampleN/sampleNWithTypes/sampleE: " + query);
  return Status::OK();
}

// ============================================================================ translator
namespace {

struct Cursor {
  std::string ids;  // input reference of the current id set
  bool edges = false;
};

class Translator {
 public:
  // nodes are referenced while later ones are appended: keep the storage stable
  Translator(const CompileOptions& opt, DAGDef* dag) : opt_(opt), dag_(dag) {}

  NodeDef& Add(const std::string& op) {
    NodeDef nd;
    nd.op = op;
    nd.id = next_id_++;
    dag_->nodes.push_back(nd);
    return dag_->nodes.back();
  }

  void Alias(const std::string& alias, const std::vector<std::string>& outs, const Cursor& c) {
    if (alias.empty()) return;
    NodeDef& as = Add("AS");
    as.inputs = outs;
    as.attrs = {alias};
    as.output_num = static_cast<int>(outs.size());
    aliases_[alias] = c;
  }

  bool NeighborOnly(const std::vector<std::string>& dnf) const {
    for (auto& conj : dnf)
      for (auto& term : Split(conj, ",")) {
        auto parts = Split(Trim(term), " ");
        if (parts.empty()) continue;
        if (std::find(opt_.neighbor_indexes.begin(), opt_.neighbor_indexes.end(), parts[0]) ==
            opt_.neighbor_indexes.end())
          return false;
      }
    return true;
  }

  Status Run(const std::vector<GqlStep>& steps) {
    // node references are held while later nodes are appended: keep storage stable
    dag_->nodes.reserve(steps.size() * 8 + 8);
    Cursor c;
    for (size_t si = 0; si < steps.size(); ++si) {
      const GqlStep& s = steps[si];
      const std::string& op = s.op;
      if (op == "v" || op == "e") {
        const bool edges = op == "e";
        if (s.dnf.empty() && s.post.empty() && !s.params.empty()) {
          c = {s.params[0], edges};
          Alias(s.alias, {s.params[0]}, c);
        } else {
          NodeDef& nd = Add(edges ? "API_GET_EDGE" : "API_GET_NODE");
          if (!s.params.empty()) nd.inputs = {s.params[0]};
          nd.dnf = s.dnf;
          nd.post_process = s.post;
          c = {nd.Output(0), edges};
          Alias(s.alias, {nd.Output(0)}, c);
        }
      } else if (op == "sampleN" || op == "sampleE") {
        if (s.params.size() < 2) return Status::InvalidArgument(op + " needs (type, count)");
        NodeDef& nd = Add(op == "sampleN" ? "API_SAMPLE_NODE" : "API_SAMPLE_EDGE");
        nd.attrs = {s.params[0], s.params[1]};
        nd.dnf = s.dnf;
        c = {nd.Output(0), op == "sampleE"};
        Alias(s.alias, {nd.Output(0)}, c);
        if (!s.post.empty()) {
          NodeDef& pp = Add("POST_PROCESS");
          pp.inputs = {c.ids};
          pp.post_process = s.post;
          c.ids = pp.Output(0);
        }
      } else if (op == "sampleNWithTypes") {
        if (s.params.size() < 2) return Status::InvalidArgument("sampleNWithTypes needs (types, counts)");
        NodeDef& nd = Add("API_SAMPLE_N_WITH_TYPES");
        nd.attrs = {s.params[0], s.params[1]};
        nd.output_num = 2;
        c = {nd.Output(1), false};
        Alias(s.alias, {nd.Output(0), nd.Output(1)}, c);
      } else if (op == "select" || op == "v_select") {
        if (s.params.empty()) return Status::InvalidArgument(op + " needs an alias");
        auto it = aliases_.find(s.params[0]);
        if (it == aliases_.end()) return Status::InvalidArgument("unknown alias in " + op + ": " + s.params[0]);
        c = it->second;
      } else if (op == "outV" || op == "inV" || op == "sampleNB") {
        const bool sample = op == "sampleNB";
        std::string nb_op = sample ? "API_SAMPLE_NB" : (op == "outV" ? "API_GET_NB_NODE" : "API_GET_RNB_NODE");
        const bool split_filter = !sample && !s.dnf.empty() && opt_.mode == CompileMode::kDistribute &&
                                  !NeighborOnly(s.dnf);
        NodeDef& nd = Add(nb_op);
        nd.inputs = {c.ids};
        nd.output_num = 4;
        if (sample) {
          if (s.params.size() < 3) return Status::InvalidArgument("sampleNB needs (edge_types, count, default)");
          nd.attrs = {s.params[0], s.params[1], s.params[2]};
          if (s.params.size() > 3) nd.attrs.push_back(s.params[3]);  // keyed draws
        } else {
          nd.attrs = {s.params.empty() ? std::string("-1") : s.params[0]};
        }
        std::vector<std::string> outs = {nd.Output(0), nd.Output(1), nd.Output(2), nd.Output(3)};
        if (split_filter) {
          // attribute-index condition in distribute mode (reference translator.cc:253-322):
          // unconditioned neighbors (remote) -> filtered node set (remote) -> client filter
          const std::string nb_name = nd.name();
          NodeDef& gn = Add("API_GET_NODE");
          gn.inputs = {nb_name + ":1"};
          gn.dnf = s.dnf;
          NodeDef& f = Add("API_GET_NB_FILTER");
          f.inputs = {nb_name + ":0", nb_name + ":1", nb_name + ":2", nb_name + ":3", gn.Output(0)};
          f.post_process = s.post;
          f.output_num = 4;
          outs = {f.Output(0), f.Output(1), f.Output(2), f.Output(3)};
        } else {
          nd.dnf = s.dnf;
          nd.post_process = s.post;
        }
        c = {outs[1], false};
        Alias(s.alias, outs, c);
      } else if (op == "sampleNodeAt") {
        // keyed root draws (graph.h KeyedBuckets): the cursor holds codes pos * buckets + bucket
        if (s.params.size() < 3) return Status::InvalidArgument("sampleNodeAt needs (node_type, buckets, key, [default])");
        NodeDef& nd = Add("API_SAMPLE_NODE_AT");
        nd.inputs = {c.ids};
        nd.attrs = s.params;
        c = {nd.Output(0), false};
        Alias(s.alias, {nd.Output(0)}, c);
      } else if (op == "outE") {
        NodeDef& nd = Add("API_GET_NB_EDGE");
        nd.inputs = {c.ids};
        nd.attrs = {s.params.empty() ? std::string("-1") : s.params[0]};
        nd.dnf = s.dnf;
        nd.output_num = 3;
        std::vector<std::string> outs = {nd.Output(0), nd.Output(1), nd.Output(2)};
        c = {nd.Output(1), true};
        Alias(s.alias, outs, c);
      } else if (op == "sampleLNB") {
        // (edge_types, n, m, [weight_func,] default) — reference translator.cc:339-532
        if (s.params.size() < 4) return Status::InvalidArgument("sampleLNB needs (edge_types, n, m, [sqrt,] default)");
        const std::string et = s.params[0], bn = s.params[1], m = s.params[2];
        const bool wf = s.params.size() >= 5;
        const std::string def = s.params.back();
        std::string layer;
        if (!wf) {
          NodeDef& w = Add("API_GET_EDGE_SUM_WEIGHT");
          w.inputs = {c.ids};
          w.attrs = {et};
          NodeDef& r = Add("API_SAMPLE_ROOT");
          r.inputs = {c.ids, w.Output(0)};
          r.attrs = {bn, m, def};
          NodeDef& l = Add("API_SAMPLE_L");
          l.inputs = {r.Output(0)};
          l.attrs = {et, def};
          layer = l.Output(0);
        } else {
          NodeDef& nb = Add("API_GET_NB_NODE");
          nb.inputs = {c.ids};
          nb.attrs = {et};
          nb.output_num = 4;
          NodeDef& l = Add("API_LOCAL_SAMPLE_L");
          l.inputs = {nb.Output(0), nb.Output(1), nb.Output(2), nb.Output(3)};
          l.attrs = {bn, m, s.params[3], def};
          layer = l.Output(0);
        }
        NodeDef& adj = Add("API_SPARSE_GET_ADJ");
        adj.inputs = {c.ids, layer};
        adj.attrs = {et, bn, m};
        adj.output_num = 2;
        std::vector<std::string> outs = {adj.Output(0), adj.Output(1), layer};
        c = {layer, false};
        Alias(s.alias, outs, c);
      } else if (op == "values") {
        NodeDef& nd = Add("API_GET_P");
        nd.inputs = {c.ids};
        for (auto& p : s.params) {
          if (StartsWith(p, "__udf__=")) nd.udf_name = p.substr(8);
          else if (StartsWith(p, "__udfarg__=")) nd.udf_str_params.push_back(p.substr(11));
          else nd.attrs.push_back(p);
        }
        for (auto& x : s.udf_params) {
          double v = 0;
          ParseDouble(x, &v);
          nd.udf_num_params.push_back(static_cast<float>(v));
        }
        nd.output_num = 2 * static_cast<int>(nd.attrs.size());
        std::vector<std::string> outs;
        for (int k = 0; k < nd.output_num; ++k) outs.push_back(nd.Output(k));
        Alias(s.alias, outs, c);
      } else if (op == "label") {
        NodeDef& nd = Add("API_GET_NODE_T");
        nd.inputs = {c.ids};
        Alias(s.alias, {nd.Output(0)}, c);
      } else {
        return Status::InvalidArgument("unsupported GQL step " + op);
      }
    }
    return Status::OK();
  }

 private:
  const CompileOptions& opt_;
  DAGDef* dag_;
  int next_id_ = 1;
  std::map<std::string, Cursor> aliases_;
};

// ---------------------------------------------------------------- optimizer helpers
enum class SplitKind { kId, kBroadcast, kAllShards, kSampleNode, kSampleEdge, kSampleNTypes };
enum class MergeKind { kIdxData, kRegular, kAppend, kMultiType };

struct Rule {
  SplitKind split;
  MergeKind merge;
  bool unique;
  // groups for kIdxData: (idx slot, data slots...)
  std::function<std::vector<std::vector<int>>(const NodeDef&)> groups;
};

std::vector<std::vector<int>> NbGroups(const NodeDef&) { return {{0, 1, 2, 3}}; }
std::vector<std::vector<int>> EdgeGroups(const NodeDef&) { return {{0, 1, 2}}; }
std::vector<std::vector<int>> PairGroups(const NodeDef& nd) {
  std::vector<std::vector<int>> g;
  for (int i = 0; i + 1 < nd.output_num; i += 2) g.push_back({i, i + 1});
  return g;
}

const std::map<std::string, Rule>& Rules() {
  static const std::map<std::string, Rule> r = {
      {"API_GET_NB_NODE", {SplitKind::kId, MergeKind::kIdxData, true, NbGroups}},
      {"API_GET_RNB_NODE", {SplitKind::kId, MergeKind::kIdxData, true, NbGroups}},
      {"API_SAMPLE_NB", {SplitKind::kId, MergeKind::kIdxData, false, NbGroups}},
      {"API_GET_NB_EDGE", {SplitKind::kId, MergeKind::kIdxData, false, EdgeGroups}},
      {"API_GET_P", {SplitKind::kId, MergeKind::kIdxData, true, PairGroups}},
      {"API_SPARSE_GET_ADJ", {SplitKind::kId, MergeKind::kIdxData, false, [](const NodeDef&) {
                                return std::vector<std::vector<int>>{{0, 1}};
                              }}},
      {"API_GET_NODE_T", {SplitKind::kId, MergeKind::kRegular, false, nullptr}},
      {"API_GET_EDGE_SUM_WEIGHT", {SplitKind::kId, MergeKind::kRegular, false, nullptr}},
      {"API_SAMPLE_L", {SplitKind::kId, MergeKind::kRegular, false, nullptr}},
      // codes pos * buckets + bucket route like ids: buckets is a multiple of the partitions
      {"API_SAMPLE_NODE_AT", {SplitKind::kId, MergeKind::kRegular, false, nullptr}},
      {"API_NODE_BUCKET_WEIGHT", {SplitKind::kAllShards, MergeKind::kAppend, false, nullptr}},
      {"API_GET_NODE", {SplitKind::kId, MergeKind::kAppend, false, nullptr}},
      {"API_GET_EDGE", {SplitKind::kId, MergeKind::kAppend, false, nullptr}},
      {"API_SAMPLE_NODE", {SplitKind::kSampleNode, MergeKind::kAppend, false, nullptr}},
      {"API_SAMPLE_EDGE", {SplitKind::kSampleEdge, MergeKind::kAppend, false, nullptr}},
      {"API_SAMPLE_N_WITH_TYPES", {SplitKind::kSampleNTypes, MergeKind::kMultiType, false, nullptr}},
      {"API_GET_GRAPH_BY_LABEL", {SplitKind::kBroadcast, MergeKind::kMultiType, false, nullptr}},
  };
  return r;
}

class Optimizer {
 public:
  Optimizer(const CompileOptions& opt, DAGDef* out) : opt_(opt), out_(out) {}

  NodeDef& Add(const std::string& op) {
    NodeDef nd;
    nd.op = op;
    nd.id = next_id_++;
    out_->nodes.push_back(nd);
    return out_->nodes.back();
  }

  std::string Map(const std::string& ref) const {
    auto it = rename_.find(ref);
    return it == rename_.end() ? ref : it->second;
  }

  void Run(const DAGDef& logical) {
    // node references are held while more nodes are appended: reserve an upper bound
    out_->nodes.reserve(logical.nodes.size() * (16 + 8 * static_cast<size_t>(std::max(1, opt_.shard_num))) + 16);
    for (auto& n : logical.nodes) next_id_ = std::max(next_id_, n.id + 1);
    for (const NodeDef& orig : logical.nodes) {
      NodeDef nd = orig;
      for (auto& in : nd.inputs) in = Map(in);
      for (auto& a : nd.attrs) a = Map(a);
      auto it = Rules().find(nd.op);
      if (it == Rules().end()) {
        // client-side op (AS, POST_PROCESS, API_GET_NB_FILTER, API_SAMPLE_ROOT, ...)
        out_->nodes.push_back(nd);
        continue;
      }
      EmitSharded(orig, nd, it->second);
    }
    Cse();
    if (opt_.fuse) FuseRemoteNodes(out_);
  }

 private:
  // inner op executed on shard s with input 0 replaced by `in0` (and attr overrides)
  std::string Remote(const NodeDef& op, int s, const std::vector<std::string>& inputs,
                     const std::vector<std::string>& attrs, std::vector<std::string>* outs) {
    NodeDef inner = op;
    inner.inputs = inputs;
    inner.attrs = attrs;
    NodeDef& r = Add("REMOTE");
    r.shard_idx = s;
    r.inner = {inner};
    // client-side tensors the shard needs: inputs + attrs that are node outputs or external names
    r.inputs = inputs;
    for (auto& a : attrs)
      if (a.find(',') != std::string::npos && a.find(':') != std::string::npos) r.inputs.push_back(a);
    r.output_num = op.output_num;
    for (int k = 0; k < op.output_num; ++k) r.output_list.push_back(inner.Output(k));
    outs->clear();
    for (int k = 0; k < op.output_num; ++k) outs->push_back(r.Output(k));
    return r.name();
  }

  void EmitSharded(const NodeDef& orig, NodeDef nd, const Rule& rule) {
    const int S = std::max(1, opt_.shard_num);
    const bool has_input = !nd.inputs.empty();
    std::string gather_idx, unique_src;
    // optional de-duplication of the ids before the RPC (reference compiler.cc:37-90)
    if (rule.unique && has_input) {
      NodeDef& u = Add("ID_UNIQUE");
      u.inputs = {nd.inputs[0]};
      u.output_num = 2;
      gather_idx = u.Output(1);
      nd.inputs[0] = u.Output(0);
    }
    std::vector<std::vector<std::string>> shard_outs(S);
    std::vector<std::string> merge_idx(S);
    SplitKind split = rule.split;
    if (split == SplitKind::kId && !has_input) split = SplitKind::kAllShards;
    if (split == SplitKind::kId) {
      std::string spn;
      // bucket codes (API_SAMPLE_NODE_AT) are not ids: they keep the hash route
      if (opt_.graph_partition && S > 1 && nd.op != "API_SAMPLE_NODE_AT") {
        spn = GpSplit(nd.inputs[0], S);
      } else {
        NodeDef& sp = Add("ID_SPLIT");
        sp.inputs = {nd.inputs[0]};
        sp.output_num = 2 * S;
        spn = sp.name();
      }
      for (int s = 0; s < S; ++s) {
        std::vector<std::string> ins = nd.inputs;
        ins[0] = spn + ":" + std::to_string(2 * s);
        merge_idx[s] = spn + ":" + std::to_string(2 * s + 1);
        if (nd.op == "API_SPARSE_GET_ADJ") {
          // candidates are broadcast; original row positions travel so batches stay aligned
          ins.resize(2);
          ins.push_back(merge_idx[s]);
        }
        Remote(nd, s, ins, nd.attrs, &shard_outs[s]);
      }
    } else if (split == SplitKind::kBroadcast || split == SplitKind::kAllShards) {
      for (int s = 0; s < S; ++s) Remote(nd, s, nd.inputs, nd.attrs, &shard_outs[s]);
    } else {
      const char* sop = split == SplitKind::kSampleNode   ? "SAMPLE_NODE_SPLIT"
                        : split == SplitKind::kSampleEdge ? "SAMPLE_EDGE_SPLIT"
                                                          : "SAMPLE_N_WITH_TYPES_SPLIT";
      NodeDef& sp = Add(sop);
      sp.attrs = {nd.attrs.at(0), nd.attrs.at(1)};
      sp.output_num = S;
      const std::string spn = sp.name();
      for (int s = 0; s < S; ++s) {
        std::vector<std::string> attrs = nd.attrs;
        attrs[1] = spn + ":" + std::to_string(s);
        Remote(nd, s, nd.inputs, attrs, &shard_outs[s]);
      }
    }
    // merges -> final output names for each original slot
    std::vector<std::string> final_out(nd.output_num);
    if (rule.merge == MergeKind::kIdxData) {
      for (auto& g : rule.groups(nd)) {
        NodeDef& im = Add("IDX_MERGE");
        for (int s = 0; s < S; ++s) {
          im.inputs.push_back(shard_outs[s][g[0]]);
          im.inputs.push_back(merge_idx[s]);
        }
        final_out[g[0]] = im.Output(0);
        for (size_t k = 1; k < g.size(); ++k) {
          NodeDef& dm = Add("DATA_MERGE");
          for (int s = 0; s < S; ++s) {
            dm.inputs.push_back(shard_outs[s][g[k]]);
            dm.inputs.push_back(shard_outs[s][g[0]]);
            dm.inputs.push_back(merge_idx[s]);
          }
          final_out[g[k]] = dm.Output(0);
        }
        if (!gather_idx.empty()) {
          NodeDef& ig = Add("IDX_GATHER");
          ig.inputs = {final_out[g[0]], gather_idx};
          const std::string merged_idx = final_out[g[0]];
          for (size_t k = 1; k < g.size(); ++k) {
            NodeDef& dg = Add("DATA_GATHER");
            dg.inputs = {final_out[g[k]], merged_idx, gather_idx};
            final_out[g[k]] = dg.Output(0);
          }
          final_out[g[0]] = ig.Output(0);
        }
      }
    } else if (rule.merge == MergeKind::kRegular) {
      for (int k = 0; k < nd.output_num; ++k) {
        NodeDef& rm = Add("REGULAR_DATA_MERGE");
        for (int s = 0; s < S; ++s) {
          rm.inputs.push_back(shard_outs[s][k]);
          rm.inputs.push_back(merge_idx[s]);
        }
        final_out[k] = rm.Output(0);
      }
    } else if (rule.merge == MergeKind::kAppend) {
      NodeDef& am = Add("APPEND_MERGE");
      for (int s = 0; s < S; ++s) am.inputs.push_back(shard_outs[s][0]);
      final_out[0] = am.Output(0);
      if (!nd.post_process.empty()) {
        NodeDef& pp = Add("POST_PROCESS");
        pp.inputs = {final_out[0]};
        pp.post_process = nd.post_process;
        final_out[0] = pp.Output(0);
      }
    } else {  // multi-type / row append: slot 0 idx, slot 1 data
      NodeDef& im = Add("MULTI_TYPE_IDX_MERGE");
      for (int s = 0; s < S; ++s) im.inputs.push_back(shard_outs[s][0]);
      NodeDef& dm = Add("MULTI_TYPE_DATA_MERGE");
      for (int s = 0; s < S; ++s) {
        dm.inputs.push_back(shard_outs[s][1]);
        dm.inputs.push_back(shard_outs[s][0]);
      }
      final_out[0] = im.Output(0);
      if (nd.output_num > 1) final_out[1] = dm.Output(0);
    }
    for (int k = 0; k < nd.output_num; ++k) rename_[orig.Output(k)] = final_out[k];
  }

  // graph_partition routing of the ids (or edges, by source) in `ids`: every shard reports
  // the type of each id (-1: not held there), GP_ID_SPLIT sends each row to its first holder;
  // one ownership round per distinct input of the query
  std::string GpSplit(const std::string& ids, int S) {
    auto it = gp_split_.find(ids);
    if (it != gp_split_.end()) return it->second;
    NodeDef& src = Add("ID_SRC");
    src.inputs = {ids};
    const std::string src_out = src.Output(0);
    std::vector<std::string> types;
    for (int s = 0; s < S; ++s) {
      NodeDef q;
      q.op = "API_GET_NODE_T";
      q.id = next_id_++;
      q.output_num = 1;
      std::vector<std::string> outs;
      Remote(q, s, {src_out}, {}, &outs);
      types.push_back(outs[0]);
    }
    NodeDef& sp = Add("GP_ID_SPLIT");
    sp.inputs = {ids};
    sp.inputs.insert(sp.inputs.end(), types.begin(), types.end());
    sp.output_num = 2 * S;
    gp_split_[ids] = sp.name();
    return sp.name();
  }

  // common-subexpression elimination of identical split / unique nodes (reference optimizer.cc:167-201)
  void Cse() {
    std::map<std::string, std::string> seen;  // signature -> node name
    std::unordered_map<std::string, std::string> repl;
    std::vector<NodeDef> kept;
    for (auto& n : out_->nodes) {
      NodeDef m = n;
      auto fix = [&](std::string& ref) {
        const std::string node = InputNode(ref);
        auto it = repl.find(node);
        if (it != repl.end()) ref = it->second + ref.substr(node.size());
      };
      for (auto& in : m.inputs) fix(in);
      for (auto& a : m.attrs) fix(a);
      for (auto& inner : m.inner) {
        for (auto& in : inner.inputs) fix(in);
        for (auto& a : inner.attrs) fix(a);
      }
      if (m.op == "ID_SPLIT" || m.op == "ID_UNIQUE") {
        const std::string sig = m.op + "|" + Join(m.inputs, ";");
        auto it = seen.find(sig);
        if (it != seen.end()) {
          repl[m.name()] = it->second;
          continue;
        }
        seen[sig] = m.name();
      }
      kept.push_back(m);
    }
    out_->nodes.swap(kept);
  }

  const CompileOptions& opt_;
  DAGDef* out_;
  std::map<std::string, std::string> gp_split_;  // ids input -> its GP_ID_SPLIT node
  int next_id_ = 1;
  std::unordered_map<std::string, std::string> rename_;
};

}  // namespace

// Fuse the REMOTE nodes of each shard that do not depend on each other into one REMOTE
// with a multi-node inner sub-DAG: one RPC per shard per dependency level instead of one
// per op (e.g. a hop's sampleNB and the frontier's values()).  Greedy in topological
// order: a REMOTE joins the first group of its shard that is not among its ancestor
// groups.  Ancestry is evaluated at join time as the transitive closure through the
// groups' CURRENT dependencies (a group gains dependencies as members join, and every
// node downstream of it inherits them), so a join can never close a cycle.  Output slots
// of a fused member are renumbered behind the group's first node.  If the fused list
// cannot be ordered topologically (a bug), the unfused DAG is kept.
void FuseRemoteNodes(DAGDef* dag) {
  std::vector<NodeDef>& nodes = dag->nodes;
  const size_t N = nodes.size();
  std::unordered_map<std::string, size_t> by_name;
  for (size_t i = 0; i < N; ++i) by_name[nodes[i].name()] = i;
  std::vector<int> group(N, -1);
  std::vector<std::set<int>> dep(N);   // nearest groups each node depends on (direct or via non-REMOTE nodes)
  std::vector<std::set<int>> gdep;     // union of the members' dep sets, per group (grows as members join)
  std::vector<std::vector<size_t>> members;
  std::vector<int> gshard;
  auto refs = [](const NodeDef& n) {
    std::vector<std::string> r = n.inputs;
    for (auto& a : n.attrs)
      if (a.find(':') != std::string::npos) r.push_back(a);
    return r;
  };
  auto closure = [&](const std::set<int>& seed) {
    std::set<int> out(seed);
    std::vector<int> stack(seed.begin(), seed.end());
    while (!stack.empty()) {
      const int g = stack.back();
      stack.pop_back();
      for (int h : gdep[g])
        if (out.insert(h).second) stack.push_back(h);
    }
    return out;
  };
  for (size_t i = 0; i < N; ++i) {
    std::set<int> d;
    for (auto& ref : refs(nodes[i])) {
      auto it = by_name.find(InputNode(ref));
      if (it == by_name.end() || it->second >= i) continue;
      const size_t p = it->second;
      if (group[p] >= 0) d.insert(group[p]);
      else d.insert(dep[p].begin(), dep[p].end());
    }
    dep[i] = d;
    if (nodes[i].op != "REMOTE") continue;
    const std::set<int> anc = closure(d);
    int g = -1;
    for (size_t k = 0; k < members.size(); ++k)
      if (gshard[k] == nodes[i].shard_idx && !anc.count(static_cast<int>(k))) {
        g = static_cast<int>(k);
        break;
      }
    if (g < 0) {
      g = static_cast<int>(members.size());
      members.push_back({});
      gdep.push_back({});
      gshard.push_back(nodes[i].shard_idx);
    }
    members[g].push_back(i);
    gdep[g].insert(d.begin(), d.end());
    group[i] = g;
  }
  // merge: the first member absorbs the others' inner nodes, inputs and output slots
  std::unordered_map<std::string, std::string> ren;  // "REMOTE,<b>:<k>" -> "REMOTE,<a>:<off + k>"
  std::vector<bool> drop(N, false);
  std::vector<NodeDef> original;
  for (auto& mem : members) {
    if (mem.size() < 2) continue;
    if (original.empty()) original = nodes;
    NodeDef& head = nodes[mem[0]];
    const std::string hn = head.name();
    std::set<std::string> ins(head.inputs.begin(), head.inputs.end());
    for (size_t k = 1; k < mem.size(); ++k) {
      NodeDef& m = nodes[mem[k]];
      for (int o = 0; o < m.output_num; ++o) ren[m.Output(o)] = hn + ":" + std::to_string(head.output_num + o);
      head.output_num += m.output_num;
      head.output_list.insert(head.output_list.end(), m.output_list.begin(), m.output_list.end());
      head.inner.insert(head.inner.end(), m.inner.begin(), m.inner.end());
      for (auto& x : m.inputs)
        if (ins.insert(x).second) head.inputs.push_back(x);
      drop[mem[k]] = true;
    }
  }
  if (ren.empty()) return;
  std::vector<NodeDef> kept;
  kept.reserve(N);
  for (size_t i = 0; i < N; ++i) {
    if (drop[i]) continue;
    NodeDef m = nodes[i];
    for (auto& x : m.inputs) {
      auto it = ren.find(x);
      if (it != ren.end()) x = it->second;
    }
    for (auto& x : m.attrs) {
      auto it = ren.find(x);
      if (it != ren.end()) x = it->second;
    }
    kept.push_back(std::move(m));
  }
  // the fused node sits where its first member was: restore a topological order
  std::unordered_map<std::string, size_t> pos;
  for (size_t i = 0; i < kept.size(); ++i) pos[kept[i].name()] = i;
  std::vector<int> indeg(kept.size(), 0);
  std::vector<std::vector<size_t>> succ(kept.size());
  for (size_t i = 0; i < kept.size(); ++i)
    for (auto& ref : refs(kept[i])) {
      auto it = pos.find(InputNode(ref));
      if (it == pos.end() || it->second == i) continue;
      succ[it->second].push_back(i);
      ++indeg[i];
    }
  std::vector<NodeDef> order;
  order.reserve(kept.size());
  std::vector<size_t> ready;
  for (size_t i = 0; i < kept.size(); ++i)
    if (indeg[i] == 0) ready.push_back(i);
  for (size_t r = 0; r < ready.size(); ++r) {
    order.push_back(kept[ready[r]]);
    for (size_t j : succ[ready[r]])
      if (--indeg[j] == 0) ready.push_back(j);
  }
  if (order.size() == kept.size()) {
    nodes.swap(order);
  } else {
    EULER_LOG(Error) << "FuseRemoteNodes: fused DAG is cyclic; keeping the unfused plan";
    nodes.swap(original);
  }
}

Compiler& Compiler::Get() {
  static Compiler c;
  return c;
}

Status Compiler::Translate(const std::vector<GqlStep>& steps, const CompileOptions& opt, DAGDef* dag) {
  dag->nodes.clear();
  Translator t(opt, dag);
  return t.Run(steps);
}

Status Compiler::Optimize(const DAGDef& logical, const CompileOptions& opt, DAGDef* physical) {
  physical->nodes.clear();
  if (opt.mode == CompileMode::kLocal) {
    *physical = logical;
    return Status::OK();
  }
  Optimizer o(opt, physical);
  o.Run(logical);
  return Status::OK();
}

Status Compiler::Compile(const std::string& query, const CompileOptions& opt, std::shared_ptr<const DAGDef>* dag) {
  const std::string key = std::to_string(static_cast<int>(opt.mode)) + (opt.fuse ? "f" : "u") +
                          (opt.graph_partition ? "g" : "h") + "|" +
                          std::to_string(opt.shard_num) + "|" +
                          Join(opt.neighbor_indexes, ",") + "|" + query;
  {
    std::lock_guard<std::mutex> l(mu_);
    auto it = cache_.find(key);
    if (it != cache_.end()) {
      *dag = it->second;
      return Status::OK();
    }
  }
  std::vector<GqlStep> steps;
  EULER_RETURN_IF_ERROR(ParseGql(query, &steps));
  DAGDef logical;
  EULER_RETURN_IF_ERROR(Translate(steps, opt, &logical));
  auto phys = std::make_shared<DAGDef>();
  EULER_RETURN_IF_ERROR(Optimize(logical, opt, phys.get()));
  std::lock_guard<std::mutex> l(mu_);
  cache_[key] = phys;
  *dag = phys;
  return Status::OK();
}

void Compiler::ClearCache() {
  std::lock_guard<std::mutex> l(mu_);
  cache_.clear();
}

}  // namespace euler
