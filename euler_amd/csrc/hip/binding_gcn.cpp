// torch binding of the fused GCN training step (gcn.hip, gcn_args.h).
//
// A GcnPlan is built once per trainer (and again when the flow's capacities grow) from a
// dict of device tensors and sizes; every operand is validated here, the argument blocks
// are filled once and step() only launches, on torch's current stream: the root draw, three
// launches per hop, the outer layer (L = 2), the head, d(W0) (L = 2) and the reduce into the
// flat gradient — hipGraph-capturable (no allocation, no host sync).  The flat optimizer
// runs after it (parallel/flat.py), with the data-parallel all-reduce in between.
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>

#include <string>
#include <vector>

#include "hip/gcn_args.h"
#include "hip/launchers.h"

namespace py = pybind11;
using namespace euler_hip;

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "euler_amd GCN kernel '", what, "' failed: ", hipGetErrorString(e));
}

int64_t round_up(int64_t x, int64_t m) { return (x + m - 1) / m * m; }

// LDS / staged image stride of a width (gcn.hip img_ld; kWide = 144 for fc / label widths)
int64_t img_ld(int64_t w) { return w <= 64 ? 80 : 144; }

class GcnPlan {
 public:
  explicit GcnPlan(py::dict d) : d_(d) {
    L_ = geti("L");
    B_ = geti("B");
    self_ = static_cast<int32_t>(geti("self_loops"));
    TORCH_CHECK(L_ == 1 || L_ == 2, "GcnPlan: 1 or 2 GCN layers");
    TORCH_CHECK(B_ > 0, "GcnPlan: batch must be positive");
    torch::Tensor indptr = T("indptr"), nbr = T("nbr");
    need(indptr, torch::kInt64, -1, "indptr");
    need(nbr, torch::kInt32, -1, "nbr");
    dev_ = indptr.device();
    const int64_t types = geti("num_types");
    TORCH_CHECK(types >= 1 && types <= 32 && (indptr.numel() - 1) % types == 0, "GcnPlan: indptr must be [N*T+1]");
    g_.indptr = indptr.data_ptr<int64_t>();
    g_.nbr = nbr.data_ptr<int32_t>();
    g_.cumw = nullptr;
    if (has("cumw")) {  // the layer-wise (AdaptiveGCN) draw's weighted neighbour picks
      torch::Tensor cw = T("cumw");
      need(cw, torch::kFloat32, nbr.numel(), "cumw");
      g_.cumw = cw.data_ptr<float>();
    }
    g_.num_types = static_cast<int32_t>(types);
    g_.num_rows = (indptr.numel() - 1) / types;
    N_ = g_.num_rows;
    TORCH_CHECK(N_ < (int64_t{1} << 31), "GcnPlan: < 2^31 rows");
    masks_ = getv("masks");
    cap_e_ = getv("cap_e");
    cap_n_ = getv("cap_n");
    TORCH_CHECK((int)masks_.size() == L_ && (int)cap_e_.size() == L_ && (int)cap_n_.size() == L_,
                "GcnPlan: one mask / edge cap / set cap per hop");
    // root sampler (alias table) and the graph's Philox state; the reduce launch advances it
    prob_ = T("node_prob");
    need(prob_, torch::kFloat32, -1, "node_prob");
    alias_ = T("node_alias");
    need(alias_, torch::kInt32, prob_.numel(), "node_alias");
    if (has("root_rows")) {
      root_rows_ = T("root_rows");
      need(root_rows_, torch::kInt32, prob_.numel(), "root_rows");
    }
    rng_ = T("rng");
    need(rng_, torch::kInt64, 2, "rng");
    build_tables();
    build_hops();
    build_layer_draws();
    build_model();
  }

  // one training step up to the flat gradient (loss_out, counts, overflow updated on the device)
  // fused_opt: the reduce launch also applies the flat optimizer (set_optimizer)
  void step(bool fused_opt) {
    const c10::DeviceGuard guard(dev_);
    step_until_head();
    hipStream_t s = stream();
    TORCH_CHECK(!fused_opt || red_opt_.fuse_opt, "GcnPlan: set_optimizer first");
    GcnHeadArgs ha = head_;
    if (fused_opt) ha.ostep_inc = opt_step_;  // the optimizer's step, read by the reduce below
    ok(eh_gcn_head(&ha, s), "gcn_head");
    if (L_ == 2) ok(eh_gcn_dw(&dw_, dw_blocks_, s), "gcn_dw");
    if (fused_opt) {
      ok(eh_gcn_reduce(&red_opt_, s), "gcn_reduce(opt)");
    } else {
      ok(eh_gcn_reduce(&red_, s), "gcn_reduce");
    }
  }

  // the flat optimizer the fused step applies: d = {flat, grad, m, v, step, kind,
  // lr, b1, b2, eps, wd, grad_scale}; every reduce segment is a view of `grad`, and the
  // segments must cover the whole flat buffer.  Returns False (nothing set) otherwise.
  bool set_optimizer(py::dict d) {
    auto t = [&](const char* k) { return d[k].cast<torch::Tensor>(); };
    torch::Tensor flat = t("flat"), grad = t("grad"), m = t("m"), v = t("v"), stp = t("step");
    need(flat, torch::kFloat32, -1, "flat");
    need(grad, torch::kFloat32, flat.numel(), "grad");
    need(m, torch::kFloat32, flat.numel(), "m");
    need(v, torch::kFloat32, flat.numel(), "v");
    need(stp, torch::kInt64, 1, "step");
    GcnReduceArgs r = red_;
    int64_t covered = 0;
    const float* g0 = grad.data_ptr<float>();
    for (int k = 0; k < r.nseg; ++k) {
      GcnRedSeg& q = r.seg[k];
      const int64_t off = q.grad - g0;
      const int64_t n = static_cast<int64_t>(q.rows) * q.cols;
      if (off < 0 || off + n > flat.numel()) return false;
      q.p = flat.data_ptr<float>() + off;
      q.m = m.data_ptr<float>() + off;
      q.v = v.data_ptr<float>() + off;
      covered += n;
    }
    const int64_t used = d.contains("used") ? d["used"].cast<int64_t>() : flat.numel();
    if (covered != used) return false;  // every parameter element (the tail is padding)
    r.fuse_opt = 1;
    r.okind = d["kind"].cast<int>();
    r.ostep = stp.data_ptr<int64_t>();
    opt_step_ = stp.data_ptr<int64_t>();
    r.lr = d["lr"].cast<float>();
    r.b1 = d["b1"].cast<float>();
    r.b2 = d["b2"].cast<float>();
    r.eps = d["eps"].cast<float>();
    r.wd = d["wd"].cast<float>();
    r.grad_scale = d["grad_scale"].cast<float>();
    red_opt_ = r;
    opt_refs_ = {flat, grad, m, v, stp};
    return true;
  }

  void step_until_head() {
    hipStream_t s = stream();
    for (int h = 0; h < L_; ++h) {  // hop 0's expand also draws the roots
      if (hops_[h].lflag) ok(eh_gcn_layer_draw(&draws_[h], s), "gcn_layer_draw");
      ok(eh_gcn_expand(&hops_[h], s), "gcn_expand");
      ok(eh_gcn_mark(&hops_[h], s), "gcn_mark");
      ok(eh_gcn_place(&hops_[h], s), "gcn_place");
    }
    if (L_ == 2) ok(eh_gcn_layer(&layer_, s), "gcn_layer");
  }

  // per-phase wall-clock stamps of the head launch (one eager step; diagnostics)
  torch::Tensor head_profile() {
    const c10::DeviceGuard guard(dev_);
    const int64_t nblk = (B_ + 15) / 16;
    torch::Tensor prof = torch::zeros({nblk, 16}, torch::TensorOptions().dtype(torch::kInt64).device(dev_));
    GcnHeadArgs a = head_;
    a.prof = reinterpret_cast<long long*>(prof.data_ptr<int64_t>());
    step_until_head();
    ok(eh_gcn_head(&a, stream()), "gcn_head(prof)");
    if (L_ == 2) ok(eh_gcn_dw(&dw_, dw_blocks_, stream()), "gcn_dw");
    ok(eh_gcn_reduce(&red_, stream()), "gcn_reduce");
    return prof;
  }

  // after a discarded step (overflow / look-back timeout) a node counter may be left
  // non-zero: the trainer clears them with the overflow word
  void reset_counters() {
    const c10::DeviceGuard guard(dev_);
    cntw_.zero_();
  }

  // one eager step with the head's fp32 root aggregates written out [B][KP] (diagnostics)
  torch::Tensor head_aggregates() {
    const c10::DeviceGuard guard(dev_);
    torch::Tensor out = torch::zeros({B_, head_.lin.inp}, torch::TensorOptions().dtype(torch::kFloat32).device(dev_));
    GcnHeadArgs a = head_;
    a.dbg_agg = out.data_ptr<float>();
    step_until_head();
    ok(eh_gcn_head(&a, stream()), "gcn_head(dbg)");
    if (L_ == 2) ok(eh_gcn_dw(&dw_, dw_blocks_, stream()), "gcn_dw");
    ok(eh_gcn_reduce(&red_, stream()), "gcn_reduce");
    return out;
  }

  // the last step's flow (for tests): roots, node set, per-hop counts, edges and offsets
  py::dict flow() const {
    py::dict o;
    o["roots"] = roots_;
    o["set"] = set_;
    o["cnt"] = cnt_;
    o["rself"] = rself_;
    py::list hops;
    for (int h = 0; h < L_; ++h) {
      py::dict x;
      x["off"] = off_[h];
      x["enode"] = enode_[h];
      x["etgt"] = etgt_[h];
      x["esrc"] = esrc_[h];
      x["deg_s"] = degs_[h];
      hops.append(x);
    }
    o["hops"] = hops;
    if (L_ == 2) {
      o["h1"] = h1_;
      o["agg1"] = agg1_;
    }
    return o;
  }
  int64_t launches() const { return 1 + 3 * L_ + (L_ == 2 ? 2 : 0) + 1 + ndraws_; }

 private:
  py::dict d_;
  int L_ = 0;
  int32_t self_ = 1;
  int64_t B_ = 0, N_ = 0;
  c10::Device dev_{c10::kCPU};
  GcnGraph g_{};
  std::vector<int64_t> masks_, cap_e_, cap_n_, cap_t_;
  torch::Tensor prob_, alias_, root_rows_, rng_;
  torch::Tensor roots_, set_, cnt_, rself_, first_, cntw_, tag_, pos_, stamp_, overflow_, err_;
  std::vector<torch::Tensor> off_, enode_, etgt_, esrc_, eflag_, degs_, scan_deg_, scan_flag_;
  torch::Tensor h1_, agg1_, feat_, part_w_, part_fc_, part_bfc_, part_out_, part_stat_, part_w0_;
  std::vector<torch::Tensor> imgs_;
  GcnHop hops_[kGcnMaxHops]{};
  GcnLayerDraw draws_[kGcnMaxHops]{};
  int ndraws_ = 0;
  torch::Tensor lflag_;
  std::vector<torch::Tensor> draw_refs_;
  GcnLayerArgs layer_{};
  GcnHeadArgs head_{};
  GcnDwArgs dw_{};
  GcnReduceArgs red_opt_{};
  int64_t* opt_step_ = nullptr;
  std::vector<torch::Tensor> opt_refs_;
  torch::Tensor dagg_;
  GcnReduceArgs red_{};
  int64_t dw_blocks_ = 0;

  bool has(const char* k) const { return d_.contains(k) && !d_[k].is_none(); }
  int64_t geti(const char* k) const {
    TORCH_CHECK(d_.contains(k), "GcnPlan: missing '", k, "'");
    return d_[k].cast<int64_t>();
  }
  std::vector<int64_t> getv(const char* k) const {
    TORCH_CHECK(d_.contains(k), "GcnPlan: missing '", k, "'");
    return d_[k].cast<std::vector<int64_t>>();
  }
  torch::Tensor T(const char* k) const {
    TORCH_CHECK(has(k), "GcnPlan: missing tensor '", k, "'");
    return d_[k].cast<torch::Tensor>();
  }
  void need(const torch::Tensor& t, c10::ScalarType st, int64_t numel, const std::string& name) const {
    TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
    if (dev_.is_cuda()) TORCH_CHECK(t.device() == dev_, name, " must be on the plan's GPU");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
    if (numel >= 0) TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
  }
  torch::Tensor zeros(int64_t n, c10::ScalarType st) const {
    return torch::zeros({n}, torch::TensorOptions().dtype(st).device(dev_));
  }
  torch::Tensor full(int64_t n, int64_t v, c10::ScalarType st) const {
    return torch::full({n}, v, torch::TensorOptions().dtype(st).device(dev_));
  }

  void build_tables() {
    // per-node tables: never cleared (every entry is keyed by the step epoch)
    first_ = full(N_, -1, torch::kInt64);  // all ones = the largest 64-bit key
    cntw_ = zeros(N_, torch::kInt32);      // zero between hops (claimers reset their node's)
    tag_ = full(N_, -1, torch::kInt32);
    pos_ = zeros(N_, torch::kInt32);
    // the plan's epoch continues across re-plans (capacity growth) of one trainer
    stamp_ = has("stamp") ? T("stamp") : zeros(1, torch::kInt32);
    need(stamp_, torch::kInt32, 1, "stamp");
    overflow_ = T("overflow");
    need(overflow_, torch::kInt32, 1, "overflow");
    err_ = overflow_;  // look-back timeouts are reported through the same word (bit 1)
    roots_ = zeros(B_, torch::kInt32);
    cnt_ = zeros(kGcnMaxHops + 1, torch::kInt32);
    rself_ = zeros(B_, torch::kInt32);
  }

  void build_hops() {
    cap_t_.assign(L_, 0);
    int64_t set_cap = 0;
    for (int h = 0; h < L_; ++h) {
      cap_t_[h] = round_up(h == 0 ? B_ : cap_n_[h - 1], 256);
      TORCH_CHECK(cap_e_[h] > 0 && cap_n_[h] > 0, "GcnPlan: capacities must be positive");
      set_cap = std::max(set_cap, cap_n_[h]);
    }
    // the cumulative set is read as targets up to cap_t of the next hop
    set_ = full(round_up(set_cap, 256) + 256, -1, torch::kInt32);
    {
      // cnt[0] = B (a constant): written once here
      auto c = torch::tensor({static_cast<int32_t>(B_), 0, 0}, torch::TensorOptions().dtype(torch::kInt32));
      cnt_.copy_(c);
    }
    for (int h = 0; h < L_; ++h) {
      off_.push_back(zeros(cap_t_[h] + 1, torch::kInt32));
      enode_.push_back(full(cap_e_[h], -1, torch::kInt32));
      etgt_.push_back(zeros(cap_e_[h], torch::kInt32));
      esrc_.push_back(full(cap_e_[h], -1, torch::kInt32));
      eflag_.push_back(zeros(cap_e_[h], torch::kUInt8));
      degs_.push_back(zeros(round_up(cap_n_[h], 256), torch::kInt32));
      GcnHop& a = hops_[h];
      a.g = g_;
      a.mask = static_cast<uint32_t>(masks_[h]);
      a.h = h;
      a.self_loops = self_;
      a.roots = h == 0 ? roots_.data_ptr<int32_t>() : nullptr;
      if (h == 0) {
        a.prob = prob_.data_ptr<float>();
        a.alias = alias_.data_ptr<int32_t>();
        a.root_rows = root_rows_.defined() ? root_rows_.data_ptr<int32_t>() : nullptr;
        a.pop = prob_.numel();
        a.rng = rng_.data_ptr<int64_t>();
      }
      a.B = static_cast<int32_t>(B_);
      a.set = set_.data_ptr<int32_t>();
      a.cnt = cnt_.data_ptr<int32_t>();
      a.cap_t = cap_t_[h];
      a.cap_e = cap_e_[h];
      a.cap_n = cap_n_[h];
      a.off = off_[h].data_ptr<int32_t>();
      a.enode = enode_[h].data_ptr<int32_t>();
      a.etgt = etgt_[h].data_ptr<int32_t>();
      a.esrc = esrc_[h].data_ptr<int32_t>();
      a.deg_s = degs_[h].data_ptr<int32_t>();
      a.rself = rself_.data_ptr<int32_t>();
      a.first = reinterpret_cast<uint64_t*>(first_.data_ptr<int64_t>());
      a.cntw = cntw_.data_ptr<int32_t>();
      a.eflag = eflag_[h].data_ptr<uint8_t>();
      a.tag = tag_.data_ptr<int32_t>();
      a.pos = pos_.data_ptr<int32_t>();
      scan_deg_.push_back(zeros(eh_gcn_expand_blocks(cap_t_[h]), torch::kInt64));
      scan_flag_.push_back(zeros(eh_gcn_mark_blocks(&a), torch::kInt64));
      a.scan_deg = reinterpret_cast<uint64_t*>(scan_deg_[h].data_ptr<int64_t>());
      a.scan_flag = reinterpret_cast<uint64_t*>(scan_flag_[h].data_ptr<int64_t>());
      a.stamp = stamp_.data_ptr<int32_t>();
      a.overflow = overflow_.data_ptr<int32_t>();
      a.err = err_.data_ptr<int32_t>();
    }
    // hop h + 1's targets are the cumulative set: its capacity bounds theirs
    for (int h = 1; h < L_; ++h) TORCH_CHECK(cap_t_[h] >= cap_n_[h - 1], "GcnPlan: target capacity");
  }

  // FastGCN: "layer_draws" = one entry per hop, None (the full neighbourhood) or a dict
  // {prob, alias, root_rows (optional), count, stream}: the hop keeps the edges into that
  // step's layer (GcnLayerDraw); the layer flags are epoch-stamped, never cleared
  void build_layer_draws() {
    if (!has("layer_draws")) return;
    py::list ld = d_["layer_draws"];
    TORCH_CHECK(static_cast<int>(ld.size()) == L_, "GcnPlan: one layer_draws entry per hop");
    for (int h = 0; h < L_; ++h) {
      if (ld[h].is_none()) continue;
      py::dict q = ld[h].cast<py::dict>();
      if (!lflag_.defined()) lflag_ = full(N_, -1, torch::kInt32);
      const std::string kind = q.contains("kind") ? q["kind"].cast<std::string>() : std::string("fast");
      if (kind == "layer") {
        // AdaptiveGCN: the layer depends on the hop's set; only hop 0 (the roots) is sampled
        // in the fused step (L <= 2), and its draw launch draws the roots too
        TORCH_CHECK(h == 0, "GcnPlan: a layer-wise draw only on hop 0");
        TORCH_CHECK(g_.cumw != nullptr, "GcnPlan: a layer-wise draw needs cumw");
        TORCH_CHECK(B_ <= kGcnLayerMaxRoots, "GcnPlan: a layer-wise draw takes at most ", kGcnLayerMaxRoots,
                    " roots");
        GcnLayerDraw& w = draws_[h];
        w.kind = 1;
        w.prob = prob_.data_ptr<float>();
        w.alias = alias_.data_ptr<int32_t>();
        w.root_rows = root_rows_.defined() ? root_rows_.data_ptr<int32_t>() : nullptr;
        w.pop = prob_.numel();
        w.rng = rng_.data_ptr<int64_t>();
        w.stream = q["stream"].cast<uint64_t>();
        w.stream_u = q["stream_u"].cast<uint64_t>();
        w.count = q["count"].cast<int64_t>();
        TORCH_CHECK(w.count >= 1, "GcnPlan: a layer draw needs a positive count");
        w.lflag = lflag_.data_ptr<int32_t>();
        w.stamp = stamp_.data_ptr<int32_t>();
        w.g = g_;
        w.mask = static_cast<uint32_t>(masks_[h]);
        w.B = static_cast<int32_t>(B_);
        w.roots = roots_.data_ptr<int32_t>();
        hops_[h].lflag = lflag_.data_ptr<int32_t>();
        hops_[h].roots_given = 1;
        ++ndraws_;
        continue;
      }
      torch::Tensor prob = q["prob"].cast<torch::Tensor>(), alias = q["alias"].cast<torch::Tensor>();
      need(prob, torch::kFloat32, -1, "layer prob");
      need(alias, torch::kInt32, prob.numel(), "layer alias");
      GcnLayerDraw& w = draws_[h];
      w.prob = prob.data_ptr<float>();
      w.alias = alias.data_ptr<int32_t>();
      w.root_rows = nullptr;
      if (q.contains("root_rows") && !q["root_rows"].is_none()) {
        torch::Tensor rr = q["root_rows"].cast<torch::Tensor>();
        need(rr, torch::kInt32, prob.numel(), "layer root_rows");
        w.root_rows = rr.data_ptr<int32_t>();
        draw_refs_.push_back(rr);
      }
      w.pop = prob.numel();
      w.rng = rng_.data_ptr<int64_t>();
      w.stream = q["stream"].cast<uint64_t>();
      w.count = q["count"].cast<int64_t>();
      TORCH_CHECK(w.count >= 1 && w.pop >= 1, "GcnPlan: a layer draw needs a positive count and population");
      w.lflag = lflag_.data_ptr<int32_t>();
      w.stamp = stamp_.data_ptr<int32_t>();
      draw_refs_.insert(draw_refs_.end(), {prob, alias});
      hops_[h].lflag = lflag_.data_ptr<int32_t>();
      ++ndraws_;
    }
  }

  GcnLin lin(const char* wname, int64_t out, int64_t in) {
    torch::Tensor w = T(wname);
    need(w, torch::kFloat32, out * in, wname);
    GcnLin l;
    l.w = w.data_ptr<float>();
    l.out = static_cast<int32_t>(out);
    l.in = static_cast<int32_t>(in);
    l.outp = static_cast<int32_t>(round_up(out, 32));
    l.inp = static_cast<int32_t>(round_up(in, 32));
    return l;
  }

  void build_model() {
    const int64_t D = geti("D"), H0 = geti("H0"), H1 = L_ == 2 ? geti("H1") : 0, E = geti("E"), C = geti("C");
    feat_ = T("features");
    TORCH_CHECK(feat_.dim() == 2 && feat_.size(0) == N_ && feat_.size(1) % 8 == 0 && feat_.size(1) >= D,
                "GcnPlan: features must be [N, Dpad] with Dpad % 8 == 0");
    TORCH_CHECK(feat_.scalar_type() == torch::kBFloat16 || feat_.scalar_type() == torch::kFloat32,
                "GcnPlan: features must be bf16 or fp32");
    need(feat_, feat_.scalar_type(), -1, "features");
    torch::Tensor labels = T("labels");
    need(labels, torch::kFloat32, N_ * C, "labels");
    GcnAggSrc fsrc{};
    fsrc.x = feat_.data_ptr();
    fsrc.x_fp32 = feat_.scalar_type() == torch::kFloat32;
    fsrc.by_id = 1;
    fsrc.set = set_.data_ptr<int32_t>();
    fsrc.ld = static_cast<int32_t>(feat_.size(1));
    fsrc.cols = static_cast<int32_t>(D);
    const int64_t Ep = round_up(E, 32), Cp = round_up(C, 32);
    TORCH_CHECK(Ep <= 128 && Cp <= 128, "GcnPlan: fc / label widths <= 128");
    const int64_t nhead = (B_ + 15) / 16;
    GcnLin last = L_ == 2 ? lin("w1", H1, H0) : lin("w0", H0, D);
    TORCH_CHECK(last.outp <= 64 && last.inp <= 128, "GcnPlan: conv widths <= 64 (inputs <= 128)");
    if (L_ == 2) {
      GcnLin first = lin("w0", H0, D);
      TORCH_CHECK(first.outp <= 64 && first.inp <= 128 && fsrc.ld >= first.inp,
                  "GcnPlan: the feature table must be padded to ", first.inp, " columns");
      const int64_t c1 = cap_t_[1];  // rows of S_1 (the layer's targets, the head's sources)
      h1_ = zeros(c1 * first.outp, torch::kBFloat16);
      agg1_ = zeros(c1 * first.inp, torch::kBFloat16);
      GcnLayerArgs& y = layer_;
      y.src = fsrc;
      y.enode = hops_[1].enode;
      y.off = hops_[1].off;
      y.etgt = hops_[1].etgt;
      y.esrc = hops_[1].esrc;
      y.deg_s = hops_[1].deg_s;
      y.cnt = cnt_.data_ptr<int32_t>();
      y.cap_t = c1;
      y.self_loops = self_;
      y.lin = first;
      y.h_out = reinterpret_cast<uint16_t*>(h1_.data_ptr());
      y.agg_out = reinterpret_cast<uint16_t*>(agg1_.data_ptr());
      dw_blocks_ = round_up(hops_[0].cap_e + B_, kGcnDwRows) / kGcnDwRows;
      part_w0_ = zeros(dw_blocks_ * first.outp * first.inp, torch::kFloat32);
      dagg_ = zeros(B_ * first.outp, torch::kFloat32);
      GcnDwArgs& w = dw_;
      w.dagg = dagg_.data_ptr<float>();
      w.h = reinterpret_cast<uint16_t*>(h1_.data_ptr());
      w.agg = reinterpret_cast<uint16_t*>(agg1_.data_ptr());
      w.off = hops_[0].off;
      w.etgt = hops_[0].etgt;
      w.esrc = hops_[0].esrc;
      w.rself = rself_.data_ptr<int32_t>();
      w.deg_s = hops_[0].deg_s;
      w.cap_t = hops_[0].cap_t;
      w.cap_e = hops_[0].cap_e;
      w.B = static_cast<int32_t>(B_);
      w.self_loops = self_;
      w.lin = first;
      w.part = part_w0_.data_ptr<float>();
    } else {
      TORCH_CHECK(fsrc.ld >= last.inp, "GcnPlan: the feature table must be padded to ", last.inp, " columns");
    }
    GcnHeadArgs& a = head_;
    if (L_ == 2) {
      GcnAggSrc hs{};
      hs.x = h1_.data_ptr();
      hs.x_fp32 = 0;
      hs.by_id = 0;
      hs.set = set_.data_ptr<int32_t>();
      hs.ld = layer_.lin.outp;
      hs.cols = layer_.lin.out;
      a.src = hs;
      a.dagg = dagg_.data_ptr<float>();
    } else {
      a.src = fsrc;
      a.dagg = nullptr;
    }
    a.enode = hops_[0].enode;
    a.off = hops_[0].off;
    a.etgt = hops_[0].etgt;
    a.esrc = hops_[0].esrc;
    a.deg_s = hops_[0].deg_s;
    a.rself = rself_.data_ptr<int32_t>();
    a.roots = roots_.data_ptr<int32_t>();
    a.B = static_cast<int32_t>(B_);
    a.self_loops = self_;
    a.lin = last;
    const int64_t Hl = L_ == 2 ? H1 : H0;
    torch::Tensor wfc = T("wfc"), bfc = T("bfc"), wout = T("wout");
    need(wfc, torch::kFloat32, E * Hl, "wfc");
    need(bfc, torch::kFloat32, E, "bfc");
    need(wout, torch::kFloat32, C * E, "wout");
    a.wfc = wfc.data_ptr<float>();
    a.bfc = bfc.data_ptr<float>();
    a.wout = wout.data_ptr<float>();
    a.E = static_cast<int32_t>(E);
    a.Ep = static_cast<int32_t>(Ep);
    a.C = static_cast<int32_t>(C);
    a.Cp = static_cast<int32_t>(Cp);
    a.labels = labels.data_ptr<float>();
    a.inv_scale = 1.f / static_cast<float>(B_ * C);
    part_w_ = zeros(nhead * last.outp * last.inp, torch::kFloat32);
    part_fc_ = zeros(nhead * Ep * last.outp, torch::kFloat32);
    part_bfc_ = zeros(nhead * Ep, torch::kFloat32);
    part_out_ = zeros(nhead * Cp * Ep, torch::kFloat32);
    part_stat_ = zeros(nhead * 4, torch::kFloat32);
    a.part_w = part_w_.data_ptr<float>();
    a.part_fc = part_fc_.data_ptr<float>();
    a.part_bfc = part_bfc_.data_ptr<float>();
    a.part_out = part_out_.data_ptr<float>();
    a.part_stat = part_stat_.data_ptr<float>();
    TORCH_CHECK(eh_gcn_head_lds(&a) <= 160 * 1024, "GcnPlan: head tile does not fit in LDS");
    // bf16 weight images staged every step by extra blocks of hop 0's expand launch
    GcnHop& h0 = hops_[0];
    auto stage = [&](const float* w, int64_t rows, int64_t cols, int64_t rowsp, int64_t ld) {
      TORCH_CHECK(h0.nst < kGcnMaxStage, "GcnPlan: too many staged weights");
      torch::Tensor img = zeros(rowsp * ld, torch::kBFloat16);
      imgs_.push_back(img);
      GcnStageW& q = h0.st[h0.nst++];
      q.w = w;
      q.rows = static_cast<int32_t>(rows);
      q.cols = static_cast<int32_t>(cols);
      q.rowsp = static_cast<int32_t>(rowsp);
      q.ld = static_cast<int32_t>(ld);
      q.img = reinterpret_cast<uint16_t*>(img.data_ptr());
      return q.img;
    };
    if (L_ == 2) layer_.wimg = stage(layer_.lin.w, layer_.lin.out, layer_.lin.in, layer_.lin.outp,
                                     img_ld(layer_.lin.inp));
    a.wl_img = stage(last.w, last.out, last.in, last.outp, img_ld(last.inp));
    a.wfc_img = stage(a.wfc, E, Hl, Ep, img_ld(last.outp));
    a.wout_img = stage(a.wout, C, E, Cp, 144);
    // the reduce: flat-gradient views of every parameter, in the order they are listed
    GcnReduceArgs& r = red_;
    int seg = 0, blk = 0;
    auto add = [&](const char* gname, const torch::Tensor& part, int64_t rows, int64_t cols, int64_t prs, int64_t S,
                   int64_t slab) {
      torch::Tensor g = T(gname);
      need(g, torch::kFloat32, rows * cols, gname);
      GcnRedSeg& q = r.seg[seg++];
      q.grad = g.data_ptr<float>();
      q.part = part.data_ptr<float>();
      q.rows = static_cast<int32_t>(rows);
      q.cols = static_cast<int32_t>(cols);
      q.prs = static_cast<int32_t>(prs);
      q.S = static_cast<int32_t>(S);
      q.slab = slab;
      q.blk0 = blk;
      blk += static_cast<int>((rows * cols + 15) / 16);
    };
    if (L_ == 2) add("g_w0", part_w0_, H0, D, layer_.lin.inp, dw_blocks_, layer_.lin.outp * layer_.lin.inp);
    add(L_ == 2 ? "g_w1" : "g_w0", part_w_, last.out, last.in, last.inp, nhead, last.outp * last.inp);
    add("g_wfc", part_fc_, E, Hl, last.outp, nhead, Ep * last.outp);
    add("g_bfc", part_bfc_, 1, E, Ep, nhead, Ep);
    add("g_wout", part_out_, C, E, Ep, nhead, Cp * Ep);
    r.nseg = seg;
    r.nblk = blk;
    r.part_stat = part_stat_.data_ptr<float>();
    r.nstat = static_cast<int32_t>(nhead);
    torch::Tensor loss = T("loss_out"), counts = T("counts");
    need(loss, torch::kFloat32, 1, "loss_out");
    need(counts, torch::kInt64, 3, "counts");
    r.loss_out = loss.data_ptr<float>();
    r.counts = counts.data_ptr<int64_t>();
    r.stamp = stamp_.data_ptr<int32_t>();
    r.rng = rng_.data_ptr<int64_t>();
  }
};

}  // namespace

void register_gcn_ops(py::module& m) {
  py::class_<GcnPlan>(m, "GcnPlan")
      .def(py::init<py::dict>())
      .def("step", &GcnPlan::step, py::arg("fused_opt") = false)
      .def("set_optimizer", &GcnPlan::set_optimizer)
      .def("flow", &GcnPlan::flow)
      .def("reset_counters", &GcnPlan::reset_counters)
      .def("head_aggregates", &GcnPlan::head_aggregates)
      .def("head_profile", &GcnPlan::head_profile)
      .def_property_readonly("launches", &GcnPlan::launches);
}
