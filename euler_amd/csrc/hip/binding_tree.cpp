// torch binding of the fused GraphSAGE tree step (sage_tree.hip).
//
// A TreePlan is built once per trainer from a dict of device tensors and sizes: every
// operand is validated here (dtype, device, contiguity and the exact element count the
// kernels' grids assume), the kernel argument blocks are filled once, and the per-step
// methods only launch on torch's current stream (hipGraph-capturable, no allocation,
// no host sync, no per-call Python marshalling).
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "hip/tree_args.h"

namespace py = pybind11;
using namespace euler_hip;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

// EULER_AMD_TREE_SYNC=1: synchronise after every launch and name the kernel that failed
// (debugging aid; never set it for timing or graph capture)
bool sync_debug() {
  static const bool on = [] {
    const char* e = std::getenv("EULER_AMD_TREE_SYNC");
    return e && e[0] == '1';
  }();
  return on;
}

void ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "euler_amd tree kernel '", what, "' failed: ", hipGetErrorString(e));
  if (sync_debug()) {
    const hipError_t s = hipStreamSynchronize(c10::hip::getCurrentHIPStream().stream());
    TORCH_CHECK(s == hipSuccess, "euler_amd tree kernel '", what, "' faulted: ", hipGetErrorString(s));
    fprintf(stderr, "[tree-sync] %s ok\n", what);
  }
}

class TreePlan {
 public:
  explicit TreePlan(py::dict d) : d_(d) {
    L_ = geti("L");
    B_ = geti("B");
    TORCH_CHECK(L_ >= 1 && L_ <= 3, "TreePlan: 1..3 hops");
    TORCH_CHECK(B_ > 0 && B_ % 32 == 0, "TreePlan: batch must be a positive multiple of 32");
    F_ = getv("F");
    logP_ = getv("logP");  // logP[k] for levels k = 1..L-1 (index 0 unused)
    masks_ = getv("masks");
    dims_ = getv("H");     // padded conv widths H_0..H_{L-1}
    TORCH_CHECK((int)F_.size() == L_ + 1 && (int)masks_.size() == L_ + 1 && (int)logP_.size() >= L_ &&
                    (int)dims_.size() == L_,
                "TreePlan: F/masks need L+1 entries (index 0 unused), logP L, H L");
    D_ = geti("D");
    E_ = geti("E");
    C_ = geti("C");
    C_real_ = geti("C_real");
    self_ = geti("include_self");
    dev_ = T("rng").device();
    TORCH_CHECK(dev_.is_cuda(), "TreePlan: tensors must be on the GPU");
    for (int k = 1; k < L_; ++k) TORCH_CHECK(logP_[k] >= 4 && (1 << logP_[k]) > F_[k], "TreePlan: slot group too small");
    for (int k = 0; k < L_; ++k) TORCH_CHECK(dims_[k] % 64 == 0, "TreePlan: conv widths must be padded to 64");
    TORCH_CHECK(D_ % 16 == 0 && E_ % 32 == 0 && C_ % 32 == 0 && C_real_ <= C_, "TreePlan: padded dims");
    // level sizes M[k] = B * P1 * ... * Pk
    M_.assign(L_, 0);
    M_[0] = B_;
    for (int k = 1; k < L_; ++k) M_[k] = M_[k - 1] << logP_[k];
    if (has("dw_route_impl")) route_impl_ = static_cast<int>(geti("dw_route_impl"));
    build_graph();
    build_fwd();
    build_comb();
    build_head();
    build_dw();
    build_opt();
  }

  void sample() {
    const c10::DeviceGuard g(dev_);
    ok(eh_tr_sample(&sample_, stream()), "tr_sample");
  }

  // gemm_only (pipelined step): layer 0 from the A rows the previous optimizer launch's
  // gather blocks wrote (opt(..., with_gather=True))
  void fwd(c10::optional<torch::Tensor> prof, bool gemm_only) {
    const c10::DeviceGuard g(dev_);
    TORCH_CHECK(!gemm_only || pipeline_ok(), "TreePlan: no pipelined forward for this plan");
    TrFwdArgs a0 = fwd0_;
    if (prof.has_value()) {
      need(*prof, torch::kInt64, (fwd0_.M / (gemm_only ? 64 : bm0_)) * 8, "prof");
      a0.prof = reinterpret_cast<long long*>(prof->data_ptr<int64_t>());
    }
    ok(eh_tr_fwd(&a0, gemm_only ? 3 : (L_ == 1 ? 1 : 0), feat_fp32_, bm0_, stream()), "tr_fwd");
    if (L_ == 3) ok(eh_tr_fwd(&fwd1_, 2, 0, bm1_, stream()), "tr_fwd(inner)");
  }

  // with_sample: extra blocks of the launch draw the next step's batch
  void head(c10::optional<torch::Tensor> prof, bool with_sample) {
    const c10::DeviceGuard g(dev_);
    TrHeadArgs a = head_;
    if (with_sample) {
      a.smp = sample_;
      a.nsample = static_cast<int32_t>((sample_.M + kTrHeadSampleRows - 1) / kTrHeadSampleRows);
    }
    if (prof.has_value()) {
      need(*prof, torch::kInt64, (B_ / kTrHeadRows) * 8, "prof");
      a.prof = reinterpret_cast<long long*>(prof->data_ptr<int64_t>());
    }
    ok(eh_tr_head(&a, B_, stream()), "tr_head");
  }

  void bwd() {
    if (L_ != 3) return;
    const c10::DeviceGuard g(dev_);
    ok(eh_tr_bwd(&bwd1_, stream()), "tr_bwd");
  }

  // dW of the given problems, one launch: routed problems first, the others grouped
  void dw(std::vector<int64_t> which, c10::optional<torch::Tensor> prof) {
    const c10::DeviceGuard g(dev_);
    TrDwLaunch L{};
    L.route_impl = route_impl_;
    if (prof.has_value()) {
      TORCH_CHECK(prof->dtype() == torch::kInt64 && prof->is_cuda() && prof->is_contiguous(), "dw: prof");
      L.prof = reinterpret_cast<long long*>(prof->data_ptr<int64_t>());
    }
    for (int64_t i : which) {
      TORCH_CHECK(i >= 0 && i < (int64_t)probs_.size(), "dw: problem index out of range");
      if (probs_[i].route) {
        TORCH_CHECK(L.nroute < 2, "dw: at most two routed problems per launch");
        L.route[L.nroute++] = probs_[i];
      } else {
        TORCH_CHECK(L.plain.n < kTrMaxProbs, "dw: too many problems");
        L.plain.p[L.plain.n++] = probs_[i];
      }
    }
    if (L.nroute == 0 && L.plain.n == 0) return;
    ok(eh_tr_dw(&L, stream()), "tr_dw");
  }

  std::vector<int64_t> problems(bool route) const {
    std::vector<int64_t> out;
    for (size_t i = 0; i < probs_.size(); ++i)
      if (static_cast<bool>(probs_[i].route) == route) out.push_back(static_cast<int64_t>(i));
    return out;
  }

  // mode 0 reduce, 1 optimizer, 2 fused, 3 shadows only
  // with_sample: modes 1/2 also draw the next step's batch (extra blocks of the launch)
  // with_gather: extra blocks gather the NEXT step's layer-0 inputs (the tree the head's
  // sampler drew) into A0_kt and A0_rows, so that step's forward is GEMM-only
  void opt(int64_t mode, double grad_scale, bool with_sample, bool with_gather) {
    const c10::DeviceGuard g(dev_);
    TORCH_CHECK(!with_gather || pipeline_ok(), "TreePlan: no pipelined gather for this plan");
    TrOptArgs a = opt_;
    a.grad_scale = static_cast<float>(grad_scale);
    if (!with_sample) a.nsample = 0;
    if (with_gather) {
      a.gat = fwd0_;
      a.ngather = static_cast<int32_t>(fwd0_.M / 32);
      a.gat_fp32 = feat_fp32_;
      static const int first = [] {
        const char* e = std::getenv("EULER_AMD_GATHER_FIRST");
        return e ? std::atoi(e) : 1;
      }();
      a.gather_first = first;
      static const int tpb = [] {
        const char* e = std::getenv("EULER_AMD_OPT_TPB");
        return e ? std::atoi(e) : 4;
      }();
      a.opt_tpb = tpb;
    }
    ok(eh_tr_opt(&a, static_cast<int>(mode), stream()), "tr_opt");
  }

  // the pipelined step applies: 2 hops, the 64-row layer-0 kernel, A0_rows given, sibling
  // groups of at most 32 rows (one gather tile)
  bool pipeline_ok() const {
    return L_ == 2 && fwd0_.a_rows != nullptr && !cached_ && bm0_ <= 64 && logP_[1] <= 5 && D_ % 64 == 0 &&
           fwd0_.M % 64 == 0 && dims_[0] <= 256 &&
           eh_tr_gather32_lds(static_cast<int>(D_), static_cast<int>(fwd0_.FL)) <= 64 * 1024;
  }

  // split-K reduce (mode 0) of a subset of the flat segments (data-parallel buckets);
  // head_stats: this launch also reduces the head's loss / F1 partials
  void opt_segments(int64_t mode, std::vector<int64_t> segs, bool head_stats) {
    TORCH_CHECK(mode == 0, "opt_segments: only the reduce (mode 0) runs on a segment subset");
    TORCH_CHECK(!segs.empty() && (int64_t)segs.size() <= opt_.nseg, "opt_segments: bad segment list");
    const c10::DeviceGuard g(dev_);
    TrOptArgs a = opt_;
    int blk = 0, n = 0;
    for (int64_t k : segs) {
      TORCH_CHECK(k >= 0 && k < opt_.nseg, "opt_segments: segment index out of range");
      TrSeg s = opt_.seg[k];
      s.blk0 = blk;
      blk += tr_seg_prepare(s);
      a.seg[n++] = s;
    }
    a.nseg = n;
    a.nblk = blk;
    a.nsample = 0;
    if (!head_stats) a.nhead = 0;
    ok(eh_tr_opt(&a, 0, stream()), "tr_opt(segments)");
  }

  int64_t fwd_blocks() const { return fwd0_.M / bm0_; }
  void set_lr(double lr) { opt_.lr = static_cast<float>(lr); }
  // bf16 gradient buffer for the data-parallel hand-off (None: fp32 grad)
  // the flat fp32 gradient the reduce launch writes and the optimizer reads (e.g. a view of
  // the xGMI all-reduce's IPC input region, so the all-reduce runs in place there)
  void set_grad(torch::Tensor g) {
    TORCH_CHECK(g.is_cuda() && g.scalar_type() == torch::kFloat32 && g.is_contiguous() && g.numel() == opt_.n,
                "grad must be a contiguous fp32 GPU tensor of the flat parameter size");
    grad_ = g;
    opt_.g = g.data_ptr<float>();
  }
  void set_grad16(c10::optional<torch::Tensor> g16) {
    if (!g16.has_value()) {
      opt_.g16 = nullptr;
      g16_ = torch::Tensor();
      return;
    }
    TORCH_CHECK(g16->is_cuda() && g16->scalar_type() == torch::kBFloat16 && g16->is_contiguous() &&
                    g16->numel() == opt_.n,
                "grad16 must be a contiguous bf16 GPU tensor of the flat parameter size");
    g16_ = *g16;
    opt_.g16 = reinterpret_cast<uint16_t*>(g16_.data_ptr());
  }
  int64_t num_problems() const { return (int64_t)probs_.size(); }
  // blocks of the routed problem i in a dw launch (the prof rows it stamps)
  int64_t route_blocks(int64_t i) const {
    const TrDwProb& p = probs_.at(i);
    return p.route ? (int64_t)(p.P / 64) * ((p.Q + 127) / 128) * p.S : 0;
  }
  std::vector<int64_t> splits() const {
    std::vector<int64_t> s;
    for (const auto& p : probs_) s.push_back(p.S);
    return s;
  }

 private:
  py::dict d_;
  int L_, B_, D_, E_, C_, C_real_, self_;
  int feat_fp32_ = 0, bm0_ = 32, bm1_ = 32;
  int route_impl_ = 0;  // EULER_AMD_DW_ROUTE_IMPL / plan key dw_route_impl
  bool cached_ = false;
  std::vector<int64_t> F_, logP_, masks_, dims_, M_;
  c10::Device dev_{c10::kCPU};
  TrGraph graph_{};
  TrTree tree_{};
  TrSampleArgs sample_{};
  TrFwdArgs fwd0_{}, fwd1_{};
  TrHeadArgs head_{};
  TrBwdArgs bwd1_{};
  std::vector<TrDwProb> probs_;
  std::vector<torch::Tensor> owned_;
  torch::Tensor roots_cur_;  // the forward's copy of the batch's roots (read by the head)
  TrOptArgs opt_{};
  torch::Tensor g16_, grad_;

  bool has(const char* k) const { return d_.contains(k) && !d_[k].is_none(); }
  int64_t geti(const char* k) const {
    TORCH_CHECK(d_.contains(k), "TreePlan: missing '", k, "'");
    return d_[k].cast<int64_t>();
  }
  double getf(const char* k) const { return d_[k].cast<double>(); }
  std::vector<int64_t> getv(const char* k) const {
    TORCH_CHECK(d_.contains(k), "TreePlan: missing '", k, "'");
    return d_[k].cast<std::vector<int64_t>>();
  }
  torch::Tensor T(const char* k) const {
    TORCH_CHECK(has(k), "TreePlan: missing tensor '", k, "'");
    return d_[k].cast<torch::Tensor>();
  }
  torch::Tensor Tk(const std::string& k) const { return T(k.c_str()); }
  void need(const torch::Tensor& t, c10::ScalarType st, int64_t numel, const std::string& name) const {
    TORCH_CHECK(t.is_cuda() && t.device() == dev_, name, " must be on the trainer's GPU");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    TORCH_CHECK(t.scalar_type() == st, name, " has the wrong dtype");
    if (numel >= 0) TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
  }
  template <typename P>
  P* ptr(const std::string& k, c10::ScalarType st, int64_t numel) {
    torch::Tensor t = Tk(k);
    need(t, st, numel, k);
    return reinterpret_cast<P*>(t.data_ptr());
  }
  uint16_t* bf(const std::string& k, int64_t numel) { return ptr<uint16_t>(k, torch::kBFloat16, numel); }
  float* f32(const std::string& k, int64_t numel) { return ptr<float>(k, torch::kFloat32, numel); }
  int32_t* i32(const std::string& k, int64_t numel) { return ptr<int32_t>(k, torch::kInt32, numel); }

  int64_t Hin(int k) const { return k == 0 ? D_ : dims_[k - 1]; }

  void build_graph() {
    torch::Tensor indptr = T("indptr"), rng = T("rng");
    need(indptr, torch::kInt64, -1, "indptr");
    need(rng, torch::kInt64, 2, "rng");
    const int64_t T_ = geti("num_types");
    TORCH_CHECK(T_ >= 1 && T_ <= 32 && (indptr.numel() - 1) % T_ == 0, "TreePlan: indptr must be [N*T+1]");
    graph_.indptr = indptr.data_ptr<int64_t>();
    graph_.num_types = static_cast<int32_t>(T_);
    graph_.num_rows = (indptr.numel() - 1) / T_;
    torch::Tensor nbr = T("nbr"), cumw = T("cumw");
    need(nbr, torch::kInt32, -1, "nbr");
    need(cumw, torch::kFloat32, nbr.numel(), "cumw");
    graph_.nbr = nbr.data_ptr<int32_t>();
    graph_.cumw = cumw.data_ptr<float>();
    torch::Tensor prob = T("node_prob");
    need(prob, torch::kFloat32, -1, "node_prob");
    graph_.pop = prob.numel();
    TORCH_CHECK(graph_.pop > 0, "TreePlan: empty root population");
    graph_.prob = prob.data_ptr<float>();
    graph_.alias = i32("node_alias", graph_.pop);
    graph_.root_rows = has("root_rows") ? i32("root_rows", graph_.pop) : nullptr;
    tree_.rng = rng.data_ptr<int64_t>();
    tree_.F1 = L_ > 1 ? static_cast<int32_t>(F_[1]) : 0;
    tree_.F2 = L_ > 2 ? static_cast<int32_t>(F_[2]) : 0;
    tree_.logP1 = L_ > 1 ? static_cast<int32_t>(logP_[1]) : 0;
    tree_.logP2 = L_ > 2 ? static_cast<int32_t>(logP_[2]) : 0;
    tree_.m1 = static_cast<uint32_t>(masks_[1]);
    tree_.m2 = L_ > 2 ? static_cast<uint32_t>(masks_[2]) : 0u;
  }

  void build_fwd() {
    // "fwd_features" (+ "fwd_nodes" / "fwd_leaf" cache positions): the forward gathers from
    // a feature cache filled by the sharded-feature exchange instead of the whole table
    const bool cached = has("fwd_features");
    torch::Tensor x = cached ? T("fwd_features") : T("features");
    TORCH_CHECK(x.dim() == 2 && x.size(1) == D_, "features must be [N, D] with D padded to 16");
    TORCH_CHECK(cached || x.size(0) == graph_.num_rows, "features must have one row per graph row");
    TORCH_CHECK(x.scalar_type() == torch::kBFloat16 || x.scalar_type() == torch::kFloat32,
                "features must be bf16 or fp32");
    need(x, x.scalar_type(), -1, "features");
    feat_fp32_ = x.scalar_type() == torch::kFloat32;
    const int lv = L_ - 1;           // level of layer 0's target rows
    const int64_t M = M_[lv];
    TrSampleArgs& sm = sample_;
    sm.g = graph_;
    sm.tr = tree_;
    sm.M = M;
    sm.lv = lv;
    sm.FL = static_cast<int32_t>(F_[L_]);
    sm.mL = static_cast<uint32_t>(masks_[L_]);
    sm.hopL = L_;
    sm.roots = i32("roots", B_);
    sm.nodes = i32("nodes", M);
    sm.leaf = i32("leaf", M * sm.FL);
    TrFwdArgs& a = fwd0_;
    a.x = x.data_ptr();
    a.D = D_;
    a.M = M;
    a.FL = sm.FL;
    a.include_self = self_;
    a.inv_leaf = 1.f / static_cast<float>(a.FL + self_);
    cached_ = cached;
    a.nodes = cached ? i32("fwd_nodes", M) : sm.nodes;
    a.leaf = cached ? i32("fwd_leaf", M * sm.FL) : sm.leaf;
    a.roots_in = sm.roots;
    roots_cur_ = torch::zeros({B_}, torch::TensorOptions().dtype(torch::kInt32).device(dev_));
    a.roots_cur = roots_cur_.data_ptr<int32_t>();
    a.B = B_;
    a.step = ptr<int64_t>("step", torch::kInt64, 1);
    a.rng = ptr<int64_t>("rng", torch::kInt64, 2);
    if (L_ == 1) {
      a.a_next = bf("A0", B_ * 2 * D_);  // the head's input rows [B][2D]
      bm0_ = 32;
      return;
    }
    a.W = bf("W0_sh", dims_[0] * 2 * D_);
    a.H = static_cast<int32_t>(dims_[0]);
    a.a_kt = bf("A0_kt", M * 2 * D_);
    a.mask = i32_as_u32("mask0", (M / 32) * dims_[0]);
    a.logPg = static_cast<int32_t>(logP_[lv]);
    a.Fg = static_cast<int32_t>(F_[lv]);
    a.inv_grp = 1.f / static_cast<float>(a.Fg + self_);
    a.a_next = bf("A1", M_[lv - 1] * 2 * dims_[0]);
    a.a_rows = has("A0_rows") ? bf("A0_rows", M * 2 * D_) : nullptr;
    bm0_ = (1 << a.logPg) > 32 ? (1 << a.logPg) : 32;
    if (has("fwd_bm")) bm0_ = std::max<int>(bm0_, static_cast<int>(geti("fwd_bm")));
    TORCH_CHECK(bm0_ == 32 || bm0_ == 64 || bm0_ == 128, "TreePlan: fwd rows per block must be 32, 64 or 128");
    TORCH_CHECK(M % bm0_ == 0, "TreePlan: target rows must be a multiple of the fwd block rows");
    if (L_ == 3) {
      TrFwdArgs& b = fwd1_;
      b.x = Tk("A1").data_ptr();
      b.D = static_cast<int32_t>(dims_[0]);
      b.M = M_[1];
      b.include_self = self_;
      b.W = bf("W1_sh", dims_[1] * 2 * dims_[0]);
      b.H = static_cast<int32_t>(dims_[1]);
      b.a_kt = bf("A1_kt", M_[1] * 2 * dims_[0]);
      b.mask = i32_as_u32("mask1", (M_[1] / 32) * dims_[1]);
      b.logPg = static_cast<int32_t>(logP_[1]);
      b.Fg = static_cast<int32_t>(F_[1]);
      b.inv_grp = 1.f / static_cast<float>(b.Fg + self_);
      b.a_next = bf("A2", B_ * 2 * dims_[1]);
      bm1_ = (1 << b.logPg) > 32 ? (1 << b.logPg) : 32;
    }
  }

  // fc and out_fc combined for the head (TrCombArgs): rebuilt every step by extra blocks
  // of the first forward launch from the fp32 masters in the flat buffer
  void build_comb() {
    torch::Tensor flat = T("flat");
    need(flat, torch::kFloat32, -1, "flat");
    std::vector<int64_t> off = getv("offsets");  // L convs, fc W, fc b, out W, end
    TORCH_CHECK((int)off.size() == L_ + 4 && off.back() == flat.numel(), "TreePlan: offsets must cover the flat buffer");
    const int64_t H = dims_[L_ - 1];
    TORCH_CHECK(off[L_ + 1] - off[L_] == (int64_t)E_ * H && off[L_ + 3] - off[L_ + 2] == (int64_t)C_ * E_,
                "TreePlan: fc / out_fc segments do not match E, H, C");
    TORCH_CHECK(C_ % 16 == 0 && H % 16 == 0 && E_ % 32 == 0, "TreePlan: combination tiles need C % 16, H % 16, E % 32");
    float* base = flat.data_ptr<float>();
    TrCombArgs& c = fwd0_.comb;
    c.bfc = base + off[L_ + 1];
    c.wout = base + off[L_ + 2];
    c.wout_sh = bf("Wout_sh", (int64_t)C_ * E_);
    c.wfcT_sh = bf("Wfc_shT", (int64_t)E_ * H);
    c.C = C_;
    c.E = E_;
    c.H = static_cast<int32_t>(H);
    c.Wc = owned_bf16((int64_t)C_ * H);
    c.WcT = owned_bf16((int64_t)C_ * H);
    c.bc = owned(C_);
    fwd0_.ncomb = 1;
  }

  uint16_t* owned_bf16(int64_t n) {
    torch::Tensor t = torch::zeros({n}, torch::TensorOptions().dtype(torch::kBFloat16).device(dev_));
    owned_.push_back(t);
    return reinterpret_cast<uint16_t*>(t.data_ptr());
  }

  float* owned(int64_t n) {  // plan-owned fp32 scratch
    torch::Tensor t = torch::zeros({n}, torch::TensorOptions().dtype(torch::kFloat32).device(dev_));
    owned_.push_back(t);
    return t.data_ptr<float>();
  }

  uint32_t* i32_as_u32(const std::string& k, int64_t numel) { return reinterpret_cast<uint32_t*>(i32(k, numel)); }

  void build_head() {
    const int last = L_ - 1;
    const int64_t Hin2 = 2 * Hin(last), H = dims_[last];
    TrHeadArgs& a = head_;
    a.A = bf("A" + std::to_string(last), B_ * Hin2);
    a.Hin2 = static_cast<int32_t>(Hin2);
    a.H = static_cast<int32_t>(H);
    a.E = E_;
    a.C = C_;
    a.C_real = C_real_;
    a.W = bf("W" + std::to_string(last) + "_sh", H * Hin2);
    a.WT = L_ > 1 ? bf("W" + std::to_string(last) + "_shT", H * Hin2) : nullptr;
    a.Wfc = bf("Wfc_sh", (int64_t)E_ * H);
    a.WfcT = bf("Wfc_shT", (int64_t)E_ * H);
    a.Wout = bf("Wout_sh", (int64_t)C_ * E_);
    a.WoutT = bf("Wout_shT", (int64_t)C_ * E_);
    a.bfc = f32("bfc", E_);
    a.Wc = fwd0_.comb.Wc;
    a.WcT = fwd0_.comb.WcT;
    a.bc = fwd0_.comb.bc;
    a.roots = fwd0_.roots_cur;
    const int mode = static_cast<int>(geti("label_mode"));
    torch::Tensor lab = T("labels");
    TORCH_CHECK(lab.is_cuda() && lab.is_contiguous() && lab.device() == dev_, "labels must be contiguous on the GPU");
    TORCH_CHECK(mode >= 0 && mode <= 2, "label_mode must be 0, 1 or 2");
    // "label_rows": a label table over other rows than the graph's (the row-sharded trainer
    // hands the head a [B] table of the batch's labels with roots = 0 .. B-1)
    const int64_t lrows = has("label_rows") ? geti("label_rows") : graph_.num_rows;
    if (mode == 0) {
      TORCH_CHECK(lab.scalar_type() == torch::kInt16 && lab.numel() == lrows, "labels int16 [N]");
    } else if (mode == 1) {
      TORCH_CHECK(lab.scalar_type() == torch::kInt32 && lab.numel() == lrows, "labels int32 [N]");
    } else {
      TORCH_CHECK(lab.scalar_type() == torch::kBFloat16 && lab.numel() == lrows * C_, "labels bf16 [N, C]");
    }
    a.labels = lab.data_ptr();
    a.label_mode = mode;
    a.inv_scale = 1.f / static_cast<float>(B_ * C_real_);
    a.A_kt = bf("A" + std::to_string(last) + "_kt", B_ * Hin2);
    a.h_kt = bf("h_kt", B_ * H);
    a.emb_kt = bf("emb_kt", (int64_t)B_ * E_);
    a.dlog_kt = bf("dlog_kt", (int64_t)B_ * C_);
    a.demb_kt = bf("demb_kt", (int64_t)B_ * E_);
    a.g_kt = bf("g_kt", B_ * H);
    a.dA = L_ > 1 ? f32("dA" + std::to_string(last), B_ * Hin2) : nullptr;
    const int64_t nblk = B_ / kTrHeadRows;
    a.dbfc_part = owned(nblk * E_);
    a.head_part = owned(nblk * 4);
    a.prof = nullptr;
    const size_t lds = eh_tr_head_lds(a.Hin2, a.H, a.E, a.C, mode);
    TORCH_CHECK(lds <= 160 * 1024 - 64, "TreePlan: head tile does not fit in LDS (", lds, " bytes)");
    if (L_ == 3) {
      TrBwdArgs& b = bwd1_;
      b.dA = f32("dA2", B_ * 2 * dims_[1]);
      b.mask = i32_as_u32("mask1", (M_[1] / 32) * dims_[1]);
      b.WT = bf("W1_shT", dims_[1] * 2 * dims_[0]);
      b.Hk = static_cast<int32_t>(dims_[1]);
      b.K2out = static_cast<int32_t>(2 * dims_[0]);
      b.M = M_[1];
      b.logPg = static_cast<int32_t>(logP_[1]);
      b.Fg = static_cast<int32_t>(F_[1]);
      b.include_self = self_;
      b.inv = 1.f / static_cast<float>(b.Fg + self_);
      b.dA_out = f32("dA1", M_[1] * 2 * dims_[0]);
    }
  }

  // split-K plan.  Stored-G problems: ~target workgroups of 64x64 tiles, at least min_kps
  // 32-row k-blocks per split.  Routed problems: 64x128 tiles, S a multiple of 8 (XCD
  // mapping) near route_target workgroups.
  void plan_splits(TrDwProb& p, bool route) const {
    const int64_t MB = p.MB;
    if (route) {
      const int64_t tiles = (p.P / 64) * ((p.Q + 127) / 128);
      const int64_t target = has("dw_route_wg") ? geti("dw_route_wg") : 256;
      int64_t S = (target + tiles - 1) / tiles;
      S = (S + 7) / 8 * 8;
      if (S > (MB + 7) / 8 * 8) S = (MB + 7) / 8 * 8;
      p.kps = static_cast<int32_t>((MB + S - 1) / S);
      p.S = static_cast<int32_t>(S);  // >= ceil(MB / kps); trailing splits may be empty
      return;
    }
    const int64_t tiles = ((p.P + 63) / 64) * ((p.Q + 63) / 64);
    const int64_t target = has("dw_target_wg") ? geti("dw_target_wg") : 512;
    const int64_t minkps = has("dw_min_kps") ? geti("dw_min_kps") : 4;
    int64_t kps = (MB * tiles + target - 1) / target;
    if (kps < minkps) kps = minkps;
    if (kps > MB) kps = MB;
    p.kps = static_cast<int32_t>(kps);
    p.S = static_cast<int32_t>((MB + kps - 1) / kps);
  }

  void add_prob(const std::string& /*name*/, int64_t P, int64_t Q, int64_t M, const uint16_t* G, const uint16_t* X,
                const float* dA, const uint32_t* mask, int logPg, int Fg) {
    TrDwProb p{};
    p.P = static_cast<int32_t>(P);
    p.Q = static_cast<int32_t>(Q);
    p.MB = static_cast<int32_t>(M / 32);
    plan_splits(p, dA != nullptr);
    const int64_t S = p.S;
    // split-K partials are owned by the plan (their size follows its split plan)
    torch::Tensor t = torch::empty({S * P * Q}, torch::TensorOptions().dtype(torch::kFloat32).device(dev_));
    owned_.push_back(t);
    p.part = t.data_ptr<float>();
    p.G = G;
    p.X = X;
    if (dA) {
      TORCH_CHECK(P % 64 == 0, "TreePlan: routed dW needs P % 64 == 0");
      p.route = 1;
      p.dA = dA;
      p.mask = mask;
      p.logPg = logPg;
      p.Fg = Fg;
      p.include_self = self_;
      p.inv = 1.f / static_cast<float>(Fg + self_);
    }
    probs_.push_back(p);
  }

  void build_dw() {
    // conv layers 0..L-1, then fc and out_fc
    for (int k = 0; k < L_; ++k) {
      const int64_t P = dims_[k], Q = 2 * Hin(k);
      const std::string ks = std::to_string(k);
      if (k < L_ - 1) {
        const int lvl = L_ - 1 - k;  // target level of layer k
        add_prob("part" + ks, P, Q, M_[lvl], nullptr, bf("A" + ks + "_kt", M_[lvl] * Q),
                 f32("dA" + std::to_string(k + 1), M_[lvl - 1] * 2 * P), i32_as_u32("mask" + ks, (M_[lvl] / 32) * P),
                 static_cast<int>(logP_[lvl]), static_cast<int>(F_[lvl]));
      } else {
        add_prob("part" + ks, P, Q, B_, bf("g_kt", B_ * P), bf("A" + ks + "_kt", B_ * Q), nullptr, nullptr, 0, 0);
      }
    }
    const int64_t H = dims_[L_ - 1];
    add_prob("part_fc", E_, H, B_, bf("demb_kt", (int64_t)B_ * E_), bf("h_kt", B_ * H), nullptr, nullptr, 0, 0);
    add_prob("part_out", C_, E_, B_, bf("dlog_kt", (int64_t)B_ * C_), bf("emb_kt", (int64_t)B_ * E_), nullptr,
             nullptr, 0, 0);
  }

  void build_opt() {
    torch::Tensor flat = T("flat");
    const int64_t n = flat.numel();
    TrOptArgs& a = opt_;
    a.p = f32("flat", n);
    a.g = f32("grad", n);
    a.m = f32("m", n);
    a.v = f32("v", n);
    a.n = n;
    std::vector<int64_t> off = getv("offsets");  // L convs, fc W, fc b, out W, end
    TORCH_CHECK((int)off.size() == L_ + 4 && off.back() == n, "TreePlan: offsets must cover the flat buffer");
    // segments: conv weights [H_k][2 Hin_k] (+ transposed shadows where a backward GEMM
    // reads them), fc W [E][H], fc bias [E] (vector), out W [C][E]
    const int64_t H = dims_[L_ - 1];
    int seg = 0, blk = 0;
    for (int k = 0; k < L_ + 3; ++k) {
      TrSeg& s = a.seg[seg++];
      s.off = off[k];
      s.n = off[k + 1] - off[k];
      s.blk0 = blk;
      const bool bias = k == L_ + 1;
      if (bias) {  // the head's per-block fc-bias sums
        s.part = head_.dbfc_part;
        s.S = static_cast<int32_t>(B_ / kTrHeadRows);
        s.rows = 1;
        s.cols = 0;
        blk += tr_seg_prepare(s);
        continue;
      }
      const int pi = k < L_ ? k : (k == L_ ? L_ : L_ + 1);
      const TrDwProb& p = probs_[pi];
      TORCH_CHECK(s.n == (int64_t)p.P * p.Q, "TreePlan: flat segment ", k, " does not match its dW problem");
      s.part = p.part;
      s.S = p.S;
      s.rows = p.P;
      s.cols = p.Q;
      TORCH_CHECK(s.rows % 8 == 0 && s.cols % 32 == 0, "TreePlan: weight segments need rows % 8, cols % 32");
      if (k < L_) {
        const std::string ks = std::to_string(k);
        s.sh = bf("W" + ks + "_sh", s.n);
        s.shT = k >= 1 ? bf("W" + ks + "_shT", s.n) : nullptr;
      } else if (k == L_) {
        s.sh = bf("Wfc_sh", (int64_t)E_ * H);
        s.shT = bf("Wfc_shT", (int64_t)E_ * H);
      } else {
        s.sh = bf("Wout_sh", (int64_t)C_ * E_);
        s.shT = bf("Wout_shT", (int64_t)C_ * E_);
      }
      blk += tr_seg_prepare(s);
    }
    a.nseg = seg;
    a.nblk = blk;
    a.smp = sample_;
    a.nsample = static_cast<int32_t>((sample_.M + 63) / 64);
    a.step = ptr<int64_t>("step", torch::kInt64, 1);
    a.lr = static_cast<float>(getf("lr"));
    a.b1 = static_cast<float>(getf("beta1"));
    a.b2 = static_cast<float>(getf("beta2"));
    a.eps = static_cast<float>(getf("eps"));
    a.wd = static_cast<float>(getf("weight_decay"));
    a.grad_scale = 1.f;
    a.kind = static_cast<int32_t>(geti("opt_kind"));
    a.head_part = head_.head_part;
    a.nhead = static_cast<int32_t>(B_ / kTrHeadRows);
    a.loss_acc = f32("loss_acc", 1);
    a.counts = i32_as_u32("counts", 3);
    a.loss_out = f32("loss_out", 1);
  }
};

// Layer 0 of a 2-hop SAGE tower over GIVEN roots (pair / unsupervised models, where the
// roots are a node's sampled positive and negatives): the tree sampler draws hop 1 and the
// leaves from the roots in `roots_in`, tr_fwd (mode 0) gathers the leaf rows, runs the
// layer-0 GEMM + ReLU and the tree mean of hop 1, producing the last conv's input rows
// A1 = [h0(root) | mean h0(hop-1 nbrs)] [R][2H0] bf16.  The backward takes dA1 (fp32),
// routes it through the tree and the ReLU bits inside the split-K dW kernel and reduces
// the partials into the fp32 gradient of W0.  The rest of the tower (last conv, fc, loss)
// is ordinary torch on [R][2H0] rows (euler_amd/models/sage_tower.py).
class TowerPlan {
 public:
  explicit TowerPlan(py::dict d) : d_(d) {
    R_ = geti("R");
    F1_ = geti("F1");
    F2_ = geti("F2");
    logP_ = geti("logP");
    D_ = geti("D");
    H_ = geti("H");
    self_ = geti("include_self");
    dev_ = T("rng").device();
    TORCH_CHECK(dev_.is_cuda(), "TowerPlan: tensors must be on the GPU");
    TORCH_CHECK(R_ > 0 && R_ % 32 == 0, "TowerPlan: roots must be a positive multiple of 32");
    TORCH_CHECK(logP_ >= 4 && (1 << logP_) > F1_ && F1_ >= 1 && F2_ >= 1, "TowerPlan: slot group too small");
    TORCH_CHECK(D_ % 16 == 0 && H_ % 64 == 0, "TowerPlan: padded dims (D % 16, H % 64)");
    M_ = R_ << logP_;
    // graph + tree
    torch::Tensor indptr = T("indptr"), rng = T("rng"), nbr = T("nbr"), cumw = T("cumw"), prob = T("node_prob");
    need(indptr, torch::kInt64, -1, "indptr");
    need(rng, torch::kInt64, 2, "rng");
    const int64_t nt = geti("num_types");
    TORCH_CHECK(nt >= 1 && nt <= 32 && (indptr.numel() - 1) % nt == 0, "TowerPlan: indptr must be [N*T+1]");
    g_.indptr = indptr.data_ptr<int64_t>();
    g_.num_types = static_cast<int32_t>(nt);
    g_.num_rows = (indptr.numel() - 1) / nt;
    need(nbr, torch::kInt32, -1, "nbr");
    need(cumw, torch::kFloat32, nbr.numel(), "cumw");
    g_.nbr = nbr.data_ptr<int32_t>();
    g_.cumw = cumw.data_ptr<float>();
    need(prob, torch::kFloat32, -1, "node_prob");
    g_.pop = prob.numel();
    g_.prob = prob.data_ptr<float>();
    g_.alias = ptr<int32_t>("node_alias", torch::kInt32, g_.pop);
    // candidate -> row map of the root sampler (node-type subset); used when the roots are
    // drawn in the sampler (PairPlan), not when they are given
    g_.root_rows = has("root_rows") ? ptr<int32_t>("root_rows", torch::kInt32, g_.pop) : nullptr;
    tree_.rng = rng.data_ptr<int64_t>();
    tree_.root_in = ptr<int32_t>("roots_in", torch::kInt32, R_);
    tree_.F1 = static_cast<int32_t>(F1_);
    tree_.F2 = 0;
    tree_.logP1 = static_cast<int32_t>(logP_);
    tree_.logP2 = 0;
    tree_.m1 = static_cast<uint32_t>(geti("mask1"));
    tree_.m2 = 0u;
    // sampler: level-1 slots (hop 1 of each root) and their F2 leaves
    sample_.g = g_;
    sample_.tr = tree_;
    sample_.M = M_;
    sample_.lv = 1;
    sample_.FL = static_cast<int32_t>(F2_);
    sample_.mL = static_cast<uint32_t>(geti("mask2"));
    sample_.hopL = 2;
    sample_.roots = has("roots_out") ? ptr<int32_t>("roots_out", torch::kInt32, R_) : owned_i32(R_);
    sample_.nodes = ptr<int32_t>("nodes", torch::kInt32, M_);
    sample_.leaf = ptr<int32_t>("leaf", torch::kInt32, M_ * F2_);
    // layer 0 (mode 0)
    torch::Tensor x = T("features");
    TORCH_CHECK(x.dim() == 2 && x.size(1) == D_ && x.size(0) == g_.num_rows, "features must be [N, D]");
    TORCH_CHECK(x.scalar_type() == torch::kBFloat16 || x.scalar_type() == torch::kFloat32, "features bf16 / fp32");
    need(x, x.scalar_type(), -1, "features");
    feat_fp32_ = x.scalar_type() == torch::kFloat32;
    TrFwdArgs& a = fwd_;
    a.x = x.data_ptr();
    a.D = static_cast<int32_t>(D_);
    a.M = M_;
    a.FL = static_cast<int32_t>(F2_);
    a.include_self = static_cast<int32_t>(self_);
    a.inv_leaf = 1.f / static_cast<float>(F2_ + self_);
    a.nodes = sample_.nodes;
    a.leaf = sample_.leaf;
    a.roots_in = sample_.roots;
    a.roots_cur = owned_i32(R_);
    a.B = static_cast<int32_t>(R_);
    a.step = nullptr;
    a.rng = rng.data_ptr<int64_t>();
    a.W = ptr<uint16_t>("W0_sh", torch::kBFloat16, H_ * 2 * D_);
    a.H = static_cast<int32_t>(H_);
    a.a_kt = ptr<uint16_t>("A0_kt", torch::kBFloat16, M_ * 2 * D_);
    a.mask = reinterpret_cast<uint32_t*>(ptr<int32_t>("mask0", torch::kInt32, (M_ / 32) * H_));
    a.logPg = static_cast<int32_t>(logP_);
    a.Fg = static_cast<int32_t>(F1_);
    a.inv_grp = 1.f / static_cast<float>(F1_ + self_);
    a.a_next = ptr<uint16_t>("A1", torch::kBFloat16, R_ * 2 * H_);
    a.ncomb = 0;
    bm_ = (1 << logP_) > 32 ? (1 << logP_) : 32;
    TORCH_CHECK(bm_ <= 128 && M_ % bm_ == 0, "TowerPlan: sibling groups of at most 128 rows");
    // routed dW of W0 (G routed from dA1 through the tree and the ReLU bits)
    TrDwProb& p = prob_;
    p.P = static_cast<int32_t>(H_);
    p.Q = static_cast<int32_t>(2 * D_);
    p.MB = static_cast<int32_t>(M_ / 32);
    const int64_t tiles = (p.P / 64) * ((p.Q + 127) / 128);
    const int64_t target = has("dw_route_wg") ? geti("dw_route_wg") : 256;
    int64_t S = (target + tiles - 1) / tiles;
    S = (S + 7) / 8 * 8;
    if (S > (p.MB + 7) / 8 * 8) S = (p.MB + 7) / 8 * 8;
    p.kps = static_cast<int32_t>((p.MB + S - 1) / S);
    p.S = static_cast<int32_t>(S);
    part_ = torch::empty({S * p.P * p.Q}, torch::TensorOptions().dtype(torch::kFloat32).device(dev_));
    p.part = part_.data_ptr<float>();
    p.G = nullptr;
    p.X = a.a_kt;
    p.route = 1;
    p.dA = ptr<float>("dA1", torch::kFloat32, R_ * 2 * H_);
    p.mask = a.mask;
    p.logPg = static_cast<int32_t>(logP_);
    p.Fg = static_cast<int32_t>(F1_);
    p.include_self = static_cast<int32_t>(self_);
    p.inv = 1.f / static_cast<float>(F1_ + self_);
    // reduce into the fp32 gradient / bf16 shadow of the fp32 master (one weight segment)
    TrOptArgs& o = opt_;
    float* w = ptr<float>("W0", torch::kFloat32, H_ * 2 * D_);
    o.p = o.m = o.v = w;
    o.g = ptr<float>("gW0", torch::kFloat32, H_ * 2 * D_);
    o.n = H_ * 2 * D_;
    TrSeg& sg = o.seg[0];
    sg.off = 0;
    sg.n = o.n;
    sg.part = p.part;
    sg.S = p.S;
    sg.rows = static_cast<int32_t>(H_);
    sg.cols = static_cast<int32_t>(2 * D_);
    sg.blk0 = 0;
    sg.sh = const_cast<uint16_t*>(a.W);
    sg.shT = nullptr;
    o.nseg = 1;
    o.nblk = tr_seg_prepare(sg);
    dummy_ = torch::zeros({8}, torch::TensorOptions().dtype(torch::kFloat32).device(dev_));
    step_ = torch::zeros({1}, torch::TensorOptions().dtype(torch::kInt64).device(dev_));
    o.step = step_.data_ptr<int64_t>();
    o.head_part = o.loss_acc = o.loss_out = dummy_.data_ptr<float>();
    o.nhead = 0;
    o.counts = nullptr;
    o.nsample = 0;
    o.kind = 2;
  }

  // refresh the bf16 fm shadow of W0 from the fp32 master (call after each update)
  void shadow() {
    const c10::DeviceGuard g(dev_);
    ok(eh_tr_opt(&opt_, 3, stream()), "tower shadow");
  }
  void sample() {
    const c10::DeviceGuard g(dev_);
    ok(eh_tr_sample(&sample_, stream()), "tower sample");
  }
  void fwd() {
    const c10::DeviceGuard g(dev_);
    ok(eh_tr_fwd(&fwd_, 0, feat_fp32_, bm_, stream()), "tower fwd");
  }
  // internals for PairPlan (the fused pair step reuses this tower's sampler / forward /
  // routed dW description)
  const TrSampleArgs& sample_args() const { return sample_; }
  const TrFwdArgs& fwd_args() const { return fwd_; }
  const TrDwProb& prob() const { return prob_; }
  int feat_fp32() const { return feat_fp32_; }
  int bm() const { return bm_; }
  int64_t R() const { return R_; }
  int64_t H() const { return H_; }
  int64_t D() const { return D_; }
  c10::Device device() const { return dev_; }

  // dA1 (the plan's buffer) -> gW0 (the plan's buffer)
  void bwd() {
    const c10::DeviceGuard g(dev_);
    TrDwLaunch L{};
    L.route[0] = prob_;
    L.nroute = 1;
    ok(eh_tr_dw(&L, stream()), "tower dw");
    ok(eh_tr_opt(&opt_, 0, stream()), "tower reduce");
  }

 private:
  py::dict d_;
  int64_t R_, F1_, F2_, logP_, D_, H_, self_, M_;
  int feat_fp32_ = 0, bm_ = 32;
  c10::Device dev_{c10::kCPU};
  TrGraph g_{};
  TrTree tree_{};
  TrSampleArgs sample_{};
  TrFwdArgs fwd_{};
  TrDwProb prob_{};
  TrOptArgs opt_{};
  torch::Tensor part_, dummy_, step_;
  std::vector<torch::Tensor> owned_;

  bool has(const char* k) const { return d_.contains(k) && !d_[k].is_none(); }
  int64_t geti(const char* k) const {
    TORCH_CHECK(d_.contains(k), "TowerPlan: missing '", k, "'");
    return d_[k].cast<int64_t>();
  }
  torch::Tensor T(const char* k) const {
    TORCH_CHECK(has(k), "TowerPlan: missing tensor '", k, "'");
    return d_[k].cast<torch::Tensor>();
  }
  void need(const torch::Tensor& t, c10::ScalarType st, int64_t numel, const std::string& name) const {
    TORCH_CHECK(t.is_cuda() && t.device() == dev_, name, " must be on the tower's GPU");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    TORCH_CHECK(t.scalar_type() == st, name, " has the wrong dtype");
    if (numel >= 0) TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
  }
  template <typename P>
  P* ptr(const char* k, c10::ScalarType st, int64_t numel) {
    torch::Tensor t = T(k);
    need(t, st, numel, k);
    return reinterpret_cast<P*>(t.data_ptr());
  }
  int32_t* owned_i32(int64_t n) {
    torch::Tensor t = torch::full({n}, -1, torch::TensorOptions().dtype(torch::kInt32).device(dev_));
    owned_.push_back(t);
    return t.data_ptr<int32_t>();
  }
};

// The fused unsupervised GraphSAGE step (models/sage_tower.py, fused mode): both towers'
// layer 0 (their TowerPlan samplers + forwards; the roots are drawn inside the samplers:
// source roots from the alias table, the context tower's positives as one out-neighbour of
// the recomputed source root and its negatives from a stream of their own), the pair head
// (tr_pair_head: last conv + fc of both towers, pair loss, backward to dA1), ONE dW launch
// (both routed W0 problems + W1 / Wfc of both towers) and ONE optimizer launch over the
// flat parameters (split-K reduce, Adam / Adagrad / SGD / momentum, bf16 shadows, loss and
// reciprocal-rank hand-off): 7 launches per step.
class PairPlan {
 public:
  PairPlan(const TowerPlan& s, const TowerPlan& c, py::dict d) : d_(d), dev_(s.device()) {
    B_ = geti("B");
    K_ = geti("K");
    H0_ = s.H();
    H1_ = geti("H1");
    E_ = geti("E");
    TORCH_CHECK(c.R() == B_ * (1 + K_) && s.R() == B_, "PairPlan: tower roots must be B and B (1 + K)");
    TORCH_CHECK(c.H() == H0_ && c.D() == s.D(), "PairPlan: towers must have the same layer-0 shape");
    TORCH_CHECK(B_ % 32 == 0 && K_ >= 1 && K_ <= 15, "PairPlan: B % 32 == 0 and 1 <= K <= 15");
    TORCH_CHECK(H1_ % 64 == 0 && E_ % 32 == 0, "PairPlan: padded dims (H1 % 64, E % 32)");
    TORCH_CHECK(eh_tr_pair_head_lds(static_cast<int>(K_), static_cast<int>(2 * H0_), static_cast<int>(H1_),
                                    static_cast<int>(E_)) <= 160 * 1024 - 256,
                "PairPlan: the pair head does not fit in LDS (K / widths too large)");
    fpx_ = s.feat_fp32();
    bm_s_ = s.bm();
    bm_c_ = c.bm();
    // samplers: roots drawn in the kernels
    ss_ = s.sample_args();
    sc_ = c.sample_args();
    ss_.tr.root_in = nullptr;
    ss_.tr.root_mode = 0;
    ss_.tr.stream_off = 0;
    sc_.tr.root_in = nullptr;
    sc_.tr.root_mode = 1;
    sc_.tr.pair_B = static_cast<int32_t>(B_);
    sc_.tr.pair_mask = static_cast<uint32_t>(geti("pos_mask"));
    sc_.tr.stream_off = 8;
    // forwards: the source tower's block 0 advances the Adam step and the RNG counter
    step_ = T("step");
    need(step_, torch::kInt64, 1, "step");
    fs_ = s.fwd_args();
    fc_ = c.fwd_args();
    fs_.roots_in = ss_.roots;  // roots_cur: the roots the samplers drew
    fc_.roots_in = sc_.roots;
    fs_.step = step_.data_ptr<int64_t>();
    fc_.step = nullptr;
    rng_dummy_ = torch::zeros({2}, torch::TensorOptions().dtype(torch::kInt64).device(dev_));
    fc_.rng = rng_dummy_.data_ptr<int64_t>();
    // head
    nblk_ = B_ / 16;
    TrPairHeadArgs& h = head_;
    h.B = static_cast<int32_t>(B_);
    h.K = static_cast<int32_t>(K_);
    h.H0x2 = static_cast<int32_t>(2 * H0_);
    h.H1 = static_cast<int32_t>(H1_);
    h.E = static_cast<int32_t>(E_);
    h.inv_n = 1.f / static_cast<float>(B_ * (1 + K_));
    h.head_part = owned(nblk_ * 4);
    tower(h.s, s, "s");
    tower(h.c, c, "c");
    // dW: routed W0 of both towers + W1 / Wfc of both towers
    L_.route[0] = s.prob();
    L_.route[1] = c.prob();
    L_.nroute = 2;
    L_.plain.n = 0;
    const char* tn[2] = {"s", "c"};
    const int64_t R[2] = {B_, B_ * (1 + K_)};
    const TrPairTower* tw[2] = {&h.s, &h.c};
    for (int t = 0; t < 2; ++t) {
      plain_[2 * t] = add_plain(H1_, 2 * H0_, R[t], tw[t]->g_kt, tw[t]->A1_kt);   // dW1 = g^T A1
      plain_[2 * t + 1] = add_plain(E_, H1_, R[t], tw[t]->de_kt, tw[t]->h_kt);   // dWfc = de^T h1
    }
    (void)tn;
    // optimizer over the flat buffer: per tower W0, W1, Wfc, bfc
    TrOptArgs& o = opt_;
    torch::Tensor flat = T("flat");
    need(flat, torch::kFloat32, -1, "flat");
    std::vector<int64_t> off = d_["offsets"].cast<std::vector<int64_t>>();
    // the flat buffers may end in padding (parallel/flat.py pads to a multiple of 8)
    TORCH_CHECK(off.size() == 9 && off.back() <= flat.numel(), "PairPlan: offsets = 8 segments + end");
    o.n = off.back();
    const int64_t nbuf = flat.numel();
    o.p = flat.data_ptr<float>();
    o.g = ptr<float>("grad", torch::kFloat32, nbuf);
    o.m = ptr<float>("m", torch::kFloat32, nbuf);
    o.v = ptr<float>("v", torch::kFloat32, nbuf);
    int blk = 0, seg = 0;
    const TowerPlan* tp[2] = {&s, &c};
    for (int t = 0; t < 2; ++t) {
      const TrPairTower& T_ = *tw[t];
      const TrDwProb& W0 = tp[t]->prob();
      add_seg(seg++, blk, off[4 * t], W0.part, W0.S, W0.P, W0.Q, const_cast<uint16_t*>(tp[t]->fwd_args().W), nullptr);
      const TrDwProb& W1 = L_.plain.p[plain_[2 * t]];
      add_seg(seg++, blk, off[4 * t + 1], W1.part, W1.S, W1.P, W1.Q, const_cast<uint16_t*>(T_.W1),
              const_cast<uint16_t*>(T_.W1T));
      const TrDwProb& Wf = L_.plain.p[plain_[2 * t + 1]];
      add_seg(seg++, blk, off[4 * t + 2], Wf.part, Wf.S, Wf.P, Wf.Q, const_cast<uint16_t*>(T_.Wfc),
              const_cast<uint16_t*>(T_.WfcT));
      add_seg(seg++, blk, off[4 * t + 3], T_.dbfc_part, static_cast<int32_t>(nblk_), 1, 0, nullptr, nullptr);
      TORCH_CHECK(off[4 * t + 4] - off[4 * t + 3] == E_, "PairPlan: bias segment must be E long");
    }
    o.nseg = seg;
    o.nblk = blk;
    o.step = step_.data_ptr<int64_t>();
    o.lr = static_cast<float>(getf("lr"));
    o.b1 = static_cast<float>(getf("beta1"));
    o.b2 = static_cast<float>(getf("beta2"));
    o.eps = static_cast<float>(getf("eps"));
    o.wd = static_cast<float>(getf("weight_decay"));
    o.grad_scale = 1.f;
    o.kind = static_cast<int32_t>(geti("opt_kind"));
    o.head_part = h.head_part;
    o.nhead = static_cast<int32_t>(nblk_);
    o.loss_acc = ptr<float>("loss_acc", torch::kFloat32, 1);
    o.loss_out = ptr<float>("loss_out", torch::kFloat32, 1);
    o.stat_f = ptr<float>("mrr_sum", torch::kFloat32, 1);
    o.counts = nullptr;
    o.nsample = 0;
  }

  void sample() {
    const c10::DeviceGuard g(dev_);
    ok(eh_tr_sample(&ss_, stream()), "pair sample (source)");
    ok(eh_tr_sample(&sc_, stream()), "pair sample (context)");
  }
  void fwd() {
    const c10::DeviceGuard g(dev_);
    ok(eh_tr_fwd(&fs_, 0, fpx_, bm_s_, stream()), "pair fwd (source)");
    ok(eh_tr_fwd(&fc_, 0, fpx_, bm_c_, stream()), "pair fwd (context)");
  }
  void head() {
    const c10::DeviceGuard g(dev_);
    ok(eh_tr_pair_head(&head_, stream()), "pair head");
  }
  void dw() {
    const c10::DeviceGuard g(dev_);
    TrDwLaunch L = L_;
    ok(eh_tr_dw(&L, stream()), "pair dw");
  }
  // 0: split-K reduce into the flat gradient; 1: optimizer from it (scaled); 2: both; 3: shadows
  void opt(int mode, double grad_scale) {
    const c10::DeviceGuard g(dev_);
    TrOptArgs a = opt_;
    a.grad_scale = static_cast<float>(grad_scale);
    ok(eh_tr_opt(&a, mode, stream()), "pair opt");
  }
  void set_lr(double lr) { opt_.lr = static_cast<float>(lr); }
  void set_grad(torch::Tensor g) {
    need(g, torch::kFloat32, -1, "grad");
    TORCH_CHECK(g.numel() >= opt_.n, "grad has ", g.numel(), " elements, fewer than the ", opt_.n, " parameters");
    grad_keep_ = g;
    opt_.g = g.data_ptr<float>();
  }

 private:
  py::dict d_;
  c10::Device dev_;
  int64_t B_, K_, H0_, H1_, E_, nblk_;
  int fpx_ = 0, bm_s_ = 32, bm_c_ = 32;
  TrSampleArgs ss_{}, sc_{};
  TrFwdArgs fs_{}, fc_{};
  TrPairHeadArgs head_{};
  TrDwLaunch L_{};
  int plain_[4] = {0, 0, 0, 0};
  TrOptArgs opt_{};
  torch::Tensor step_, rng_dummy_, grad_keep_;
  std::vector<torch::Tensor> owned_;

  void tower(TrPairTower& t, const TowerPlan& tp, const std::string& x) {
    const int64_t R = tp.R();
    t.A1 = tp.fwd_args().a_next;
    t.W1 = bf(("W1_sh_" + x).c_str(), H1_ * 2 * H0_);
    t.W1T = bf(("W1_shT_" + x).c_str(), H1_ * 2 * H0_);
    t.Wfc = bf(("Wfc_sh_" + x).c_str(), E_ * H1_);
    t.WfcT = bf(("Wfc_shT_" + x).c_str(), E_ * H1_);
    t.bfc = ptr<float>(("bfc_" + x).c_str(), torch::kFloat32, E_);
    t.A1_kt = owned_bf16(R * 2 * H0_);
    t.h_kt = owned_bf16(R * H1_);
    t.de_kt = owned_bf16(R * E_);
    t.g_kt = owned_bf16(R * H1_);
    t.dA1 = const_cast<float*>(tp.prob().dA);
    t.dbfc_part = owned(nblk_ * E_);
  }

  // stored-G dW problem: ~512 workgroups of 64 x 64 tiles, >= 4 k-blocks per split
  int add_plain(int64_t P, int64_t Q, int64_t M, const uint16_t* G, const uint16_t* X) {
    TORCH_CHECK(M % 32 == 0 && P % 32 == 0 && Q % 32 == 0, "PairPlan: dW problem shapes");
    TrDwProb p{};
    p.P = static_cast<int32_t>(P);
    p.Q = static_cast<int32_t>(Q);
    p.MB = static_cast<int32_t>(M / 32);
    const int64_t tiles = ((P + 63) / 64) * ((Q + 63) / 64);
    const int64_t target = has("dw_target_wg") ? geti("dw_target_wg") : 512;
    int64_t kps = (p.MB * tiles + target - 1) / target;
    kps = std::max<int64_t>(kps, 4);
    kps = std::min<int64_t>(kps, p.MB);
    p.kps = static_cast<int32_t>(kps);
    p.S = static_cast<int32_t>((p.MB + kps - 1) / kps);
    p.part = owned(static_cast<int64_t>(p.S) * P * Q);
    p.G = G;
    p.X = X;
    TORCH_CHECK(L_.plain.n < kTrMaxProbs, "PairPlan: too many dW problems");
    L_.plain.p[L_.plain.n] = p;
    return L_.plain.n++;
  }

  void add_seg(int seg, int& blk, int64_t off, const float* part, int32_t S, int64_t rows, int64_t cols, uint16_t* sh,
               uint16_t* shT) {
    TORCH_CHECK(seg < kTrMaxSegs, "PairPlan: too many optimizer segments");
    TrSeg& g = opt_.seg[seg];
    g.off = off;
    g.n = cols > 0 ? rows * cols : E_;
    g.part = part;
    g.S = S;
    g.rows = static_cast<int32_t>(rows);
    g.cols = static_cast<int32_t>(cols);
    g.blk0 = blk;
    g.sh = sh;
    g.shT = shT;
    if (cols > 0)
      TORCH_CHECK(rows % 8 == 0 && cols % 32 == 0, "PairPlan: weight segments need rows % 8, cols % 32");
    blk += tr_seg_prepare(g);
  }

  bool has(const char* k) const { return d_.contains(k) && !d_[k].is_none(); }
  int64_t geti(const char* k) const {
    TORCH_CHECK(d_.contains(k), "PairPlan: missing '", k, "'");
    return d_[k].cast<int64_t>();
  }
  double getf(const char* k) const { return d_[k].cast<double>(); }
  torch::Tensor T(const char* k) const {
    TORCH_CHECK(has(k), "PairPlan: missing tensor '", k, "'");
    return d_[k].cast<torch::Tensor>();
  }
  void need(const torch::Tensor& t, c10::ScalarType st, int64_t numel, const std::string& name) const {
    TORCH_CHECK(t.is_cuda() && t.device() == dev_, name, " must be on the plan's GPU");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    TORCH_CHECK(t.scalar_type() == st, name, " has the wrong dtype");
    if (numel >= 0) TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
  }
  template <typename P>
  P* ptr(const char* k, c10::ScalarType st, int64_t numel) {
    torch::Tensor t = T(k);
    need(t, st, numel, k);
    return reinterpret_cast<P*>(t.data_ptr());
  }
  uint16_t* bf(const char* k, int64_t numel) { return ptr<uint16_t>(k, torch::kBFloat16, numel); }
  float* owned(int64_t n) {
    torch::Tensor t = torch::zeros({n}, torch::TensorOptions().dtype(torch::kFloat32).device(dev_));
    owned_.push_back(t);
    return t.data_ptr<float>();
  }
  uint16_t* owned_bf16(int64_t n) {
    torch::Tensor t = torch::zeros({n}, torch::TensorOptions().dtype(torch::kBFloat16).device(dev_));
    owned_.push_back(t);
    return reinterpret_cast<uint16_t*>(t.data_ptr());
  }
};

}  // namespace

void register_tree_ops(py::module& m) {
  static_assert(kTrHeadSampleRows == 256, "head sampler blocks: 1024 threads, 256 rows");
  py::class_<TreePlan>(m, "TreePlan")
      .def(py::init<py::dict>())
      .def("sample", &TreePlan::sample)
      .def("fwd", &TreePlan::fwd, py::arg("prof") = py::none(), py::arg("gemm_only") = false)
      .def("fwd_blocks", [](const TreePlan& t) { return t.fwd_blocks(); })
      .def("head", &TreePlan::head, py::arg("prof") = py::none(), py::arg("with_sample") = false)
      .def("bwd", &TreePlan::bwd)
      .def("dw", &TreePlan::dw, py::arg("which"), py::arg("prof") = py::none())
      .def("route_blocks", &TreePlan::route_blocks)
      .def("opt", &TreePlan::opt, py::arg("mode"), py::arg("grad_scale") = 1.0, py::arg("with_sample") = false,
           py::arg("with_gather") = false)
      .def("pipeline_ok", &TreePlan::pipeline_ok)
      .def("opt_segments", &TreePlan::opt_segments, py::arg("mode"), py::arg("segs"), py::arg("head_stats"))
      .def("set_lr", &TreePlan::set_lr)
      .def("set_grad16", &TreePlan::set_grad16, py::arg("g16"))
      .def("set_grad", &TreePlan::set_grad, py::arg("g"))
      .def("num_problems", &TreePlan::num_problems)
      .def("splits", &TreePlan::splits)
      .def("problems", &TreePlan::problems, py::arg("route"));
  m.attr("tree_head_rows") = kTrHeadRows;
  py::class_<TowerPlan>(m, "TowerPlan")
      .def(py::init<py::dict>())
      .def("shadow", &TowerPlan::shadow)
      .def("sample", &TowerPlan::sample)
      .def("fwd", &TowerPlan::fwd)
      .def("bwd", &TowerPlan::bwd);
  py::class_<PairPlan>(m, "PairPlan")
      .def(py::init<const TowerPlan&, const TowerPlan&, py::dict>(), py::keep_alive<1, 2>(), py::keep_alive<1, 3>())
      .def("sample", &PairPlan::sample)
      .def("fwd", &PairPlan::fwd)
      .def("head", &PairPlan::head)
      .def("dw", &PairPlan::dw)
      .def("opt", &PairPlan::opt, py::arg("mode"), py::arg("grad_scale") = 1.0)
      .def("set_lr", &PairPlan::set_lr)
      .def("set_grad", &PairPlan::set_grad);
}
