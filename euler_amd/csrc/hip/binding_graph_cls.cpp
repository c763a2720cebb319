// torch binding of the fused graph-classification step (graph_cls.hip, graph_cls_args.h).
//
// A GraphClsPlan is built once per trainer from a dict of device tensors and sizes
// (models/graph_cls_trainer.py); it validates every operand, lays out the step kernel's
// LDS, owns the slab / partial buffers, and step() only launches (hipGraph-capturable: no
// allocation, no host sync) on torch's current stream: gc_step, then gc_reduce into the
// flat gradient or — set_optimizer() on one process — into the flat optimizer's update.
#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>

#include <algorithm>
#include <string>
#include <vector>

#include "hip/graph_cls_args.h"

namespace py = pybind11;
using namespace euler_hip;

namespace {

hipStream_t gc_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void gc_ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "euler_amd graph-classification kernel '", what, "' failed: ", hipGetErrorString(e));
}

class GraphClsPlan {
 public:
  explicit GraphClsPlan(py::dict d) : d_(d) {
    GcStepArgs& a = a_;
    a.L = static_cast<int32_t>(geti("L"));
    a.B = static_cast<int32_t>(geti("B"));
    a.kind = static_cast<int32_t>(geti("kind"));
    a.self_loops = static_cast<int32_t>(geti("self_loops"));
    a.nmax = static_cast<int32_t>(geti("nmax"));
    a.E = static_cast<int32_t>(geti("E"));
    a.C = static_cast<int32_t>(geti("C"));
    a.G = static_cast<int32_t>(geti("G"));
    a.tab_rows = static_cast<int32_t>(geti("tab_rows"));
    TORCH_CHECK(a.L >= 1 && a.L <= kGcMaxLayers, "GraphClsPlan: 1 to ", kGcMaxLayers, " convs");
    TORCH_CHECK(a.kind == 0 || a.kind == 1, "GraphClsPlan: kind 0 (GIN) or 1 (GraphConv)");
    TORCH_CHECK(a.nmax >= 16 && a.nmax % 16 == 0 && a.nmax <= kGcMaxRows, "GraphClsPlan: nmax in [16, 64], % 16");
    std::vector<int64_t> D = getv("D");
    TORCH_CHECK(static_cast<int>(D.size()) == a.L + 1, "GraphClsPlan: L + 1 widths");
    int64_t dmax = 0;
    for (int l = 0; l <= a.L; ++l) {
      TORCH_CHECK(D[l] >= 16 && D[l] % 16 == 0 && D[l] <= kGcMaxWidth, "GraphClsPlan: widths must be 16..128, % 16");
      a.D[l] = static_cast<int32_t>(D[l]);
      dmax = std::max(dmax, D[l]);
    }
    TORCH_CHECK(a.E >= 1 && a.E <= kGcMaxWidth && a.C >= 1 && a.C <= kGcMaxLabels, "GraphClsPlan: fc / label widths");
    TORCH_CHECK(static_cast<int64_t>(a.tab_rows) * a.D[0] <= kGcMaxTable && a.tab_rows >= 1 &&
                    a.tab_rows <= kGcMaxTableRows,
                "GraphClsPlan: the embedding table must have 1..", kGcMaxTableRows, " rows and at most ", kGcMaxTable,
                " elements");
    // graph records, edge pairs of every distinct mask, feature pairs
    py::list pairs = d_["adj_pair"];
    a.nadj = static_cast<int32_t>(pairs.size());
    TORCH_CHECK(a.nadj >= 1 && a.nadj <= kGcMaxAdj, "GraphClsPlan: 1 to ", kGcMaxAdj, " adjacencies");
    torch::Tensor rec = T("rec");
    need(rec, torch::kInt32, static_cast<int64_t>(a.G) * kGcRec, "rec");
    dev_ = rec.device();
    for (int j = 0; j < a.nadj; ++j) {
      torch::Tensor pr = pairs[j].cast<torch::Tensor>();
      need(pr, torch::kInt32, -1, "adj_pair");
      keep_.push_back(pr);
      a.adj[j] = GcAdj{pr.data_ptr<int32_t>()};
    }
    std::vector<int64_t> adj_of = getv("adj_of");
    TORCH_CHECK(static_cast<int>(adj_of.size()) == a.L, "GraphClsPlan: one adjacency per conv");
    for (int l = 0; l < a.L; ++l) {
      TORCH_CHECK(adj_of[l] >= 0 && adj_of[l] < a.nadj, "GraphClsPlan: adjacency index");
      a.adj_of[l] = static_cast<int32_t>(adj_of[l]);
    }
    torch::Tensor gprob = T("gprob"), galias = T("galias"), rng = T("rng"), fpair = T("fpair"), fw = T("fw"),
                  onehot = T("onehot"), table = T("table");
    need(gprob, torch::kFloat32, a.G, "gprob");
    need(galias, torch::kInt32, a.G, "galias");
    need(rng, torch::kInt64, 2, "rng");
    need(fpair, torch::kInt32, -1, "fpair");
    need(fw, torch::kFloat32, fpair.numel(), "fw");
    need(onehot, torch::kFloat32, static_cast<int64_t>(a.G) * a.C, "onehot");
    need(table, torch::kFloat32, static_cast<int64_t>(a.tab_rows) * a.D[0], "table");
    keep_.insert(keep_.end(), {gprob, galias, rng, rec, fpair, fw, onehot, table});
    a.gprob = gprob.data_ptr<float>();
    a.galias = galias.data_ptr<int32_t>();
    a.rng = rng.data_ptr<int64_t>();
    a.rec = rec.data_ptr<int32_t>();
    a.fpair = fpair.data_ptr<int32_t>();
    a.fw = fw.data_ptr<float>();
    a.onehot = onehot.data_ptr<float>();
    a.table = table.data_ptr<float>();
    // parameters
    py::list W = d_["W"], Wf = d_["Wf"], bl = d_["bl"], eps = d_["eps"];
    std::vector<int64_t> oW = getv("o_W"), oWf = getv("o_Wf"), obl = getv("o_bl"), oeps = getv("o_eps");
    TORCH_CHECK(static_cast<int>(W.size()) == a.L && static_cast<int>(oW.size()) == a.L &&
                    static_cast<int>(oWf.size()) == a.L && static_cast<int>(obl.size()) == a.L &&
                    static_cast<int>(oeps.size()) == a.L,
                "GraphClsPlan: per-conv parameter lists");
    for (int l = 0; l < a.L; ++l) {
      const int64_t nw = static_cast<int64_t>(a.D[l + 1]) * a.D[l];
      torch::Tensor w = W[l].cast<torch::Tensor>();
      need(w, torch::kFloat32, nw, "W");
      keep_.push_back(w);
      a.W[l] = w.data_ptr<float>();
      a.o_W[l] = oW[l];
      a.o_Wf[l] = oWf[l];
      a.o_bl[l] = obl[l];
      a.o_eps[l] = oeps[l];
      if (a.kind == 1) {
        torch::Tensor f = Wf[l].cast<torch::Tensor>(), b = bl[l].cast<torch::Tensor>();
        need(f, torch::kFloat32, nw, "Wf");
        need(b, torch::kFloat32, a.D[l + 1], "bl");
        keep_.insert(keep_.end(), {f, b});
        a.Wf[l] = f.data_ptr<float>();
        a.bl[l] = b.data_ptr<float>();
      } else {
        torch::Tensor e = eps[l].cast<torch::Tensor>();
        need(e, torch::kFloat32, 1, "eps");
        keep_.push_back(e);
        a.eps[l] = e.data_ptr<float>();
      }
    }
    torch::Tensor wfc = T("Wfc"), bfc = T("bfc"), wout = T("Wout");
    need(wfc, torch::kFloat32, static_cast<int64_t>(a.E) * a.D[a.L], "Wfc");
    need(bfc, torch::kFloat32, a.E, "bfc");
    need(wout, torch::kFloat32, static_cast<int64_t>(a.C) * a.E, "Wout");
    keep_.insert(keep_.end(), {wfc, bfc, wout});
    a.Wfc = wfc.data_ptr<float>();
    a.bfc = bfc.data_ptr<float>();
    a.Wout = wout.data_ptr<float>();
    a.o_fc = geti("o_fc");
    a.o_bfc = geti("o_bfc");
    a.o_out = geti("o_out");
    a.o_tab = geti("o_tab");
    torch::Tensor warm = T("warm");
    need(warm, torch::kFloat32, -1, "warm");
    keep_.push_back(warm);
    a.warm = warm.data_ptr<float>();
    a.warm_n = warm.numel();
    // outputs
    a.S = geti("S");
    auto opt = [&](c10::ScalarType st) { return torch::TensorOptions().dtype(st).device(dev_); };
    slab_ = torch::zeros({static_cast<int64_t>(a.B) * a.S}, opt(torch::kFloat32));
    loss_part_ = torch::zeros({a.B}, opt(torch::kFloat32));
    acc_part_ = torch::zeros({a.B}, opt(torch::kFloat32));
    gidx_ = torch::zeros({a.B}, opt(torch::kInt32));
    a.slab = slab_.data_ptr<float>();
    a.loss_part = loss_part_.data_ptr<float>();
    a.acc_part = acc_part_.data_ptr<float>();
    a.gidx = gidx_.data_ptr<int32_t>();
    a.inv_scale = 1.f / static_cast<float>(static_cast<int64_t>(a.B) * a.C);
    a.ostep_inc = nullptr;
    if (has("max_lds")) max_lds_ = geti("max_lds");
    layout(dmax);
    // reduce
    GcReduceArgs& r = r_;
    r.slab = a.slab;
    r.S = a.S;
    r.B = a.B;
    torch::Tensor grad = T("grad"), loss = T("loss_out"), right = T("right");
    need(grad, torch::kFloat32, -1, "grad");
    TORCH_CHECK(grad.numel() >= a.S, "GraphClsPlan: the flat gradient is shorter than the slab row");
    need(loss, torch::kFloat32, 1, "loss_out");
    need(right, torch::kFloat64, 2, "right");
    keep_.insert(keep_.end(), {grad, loss, right});
    r.grad = grad.data_ptr<float>();
    r.loss_part = a.loss_part;
    r.acc_part = a.acc_part;
    r.loss_out = loss.data_ptr<float>();
    r.right = right.data_ptr<double>();
    r.rng = rng.data_ptr<int64_t>();
    r.fuse_opt = 0;
  }

  void step(bool fused_opt) {
    const c10::DeviceGuard guard(dev_);
    TORCH_CHECK(!fused_opt || ro_.fuse_opt, "GraphClsPlan: set_optimizer first");
    GcStepArgs a = a_;
    if (fused_opt) a.ostep_inc = const_cast<int64_t*>(ro_.ostep);
    hipStream_t s = gc_stream();
    gc_ok(eh_gc_step(&a, s), "gc_step");
    gc_ok(eh_gc_reduce(fused_opt ? &ro_ : &r_, s), "gc_reduce");
  }

  // the flat optimizer of one process's step: {flat, m, v, step, kind, lr, b1, b2, eps, wd,
  // grad_scale}; the slab row covers flat[0, S)
  bool set_optimizer(py::dict d) {
    auto t = [&](const char* k) { return d[k].cast<torch::Tensor>(); };
    torch::Tensor flat = t("flat"), m = t("m"), v = t("v"), stp = t("step");
    need(flat, torch::kFloat32, -1, "flat");
    need(m, torch::kFloat32, flat.numel(), "m");
    need(v, torch::kFloat32, flat.numel(), "v");
    need(stp, torch::kInt64, 1, "step");
    if (flat.numel() < a_.S) return false;
    GcReduceArgs r = r_;
    r.fuse_opt = 1;
    r.p = flat.data_ptr<float>();
    r.m = m.data_ptr<float>();
    r.v = v.data_ptr<float>();
    r.ostep = stp.data_ptr<int64_t>();
    r.okind = d["kind"].cast<int>();
    r.lr = d["lr"].cast<float>();
    r.b1 = d["b1"].cast<float>();
    r.b2 = d["b2"].cast<float>();
    r.eps = d["eps"].cast<float>();
    r.wd = d["wd"].cast<float>();
    r.grad_scale = d["grad_scale"].cast<float>();
    ro_ = r;
    opt_keep_ = {flat, m, v, stp};
    return true;
  }

  // one eager step (no optimizer) with per-block phase stamps [B][32] (diagnostics)
  torch::Tensor profile() {
    const c10::DeviceGuard guard(dev_);
    torch::Tensor prof = torch::zeros({a_.B, 32}, torch::TensorOptions().dtype(torch::kInt64).device(dev_));
    GcStepArgs a = a_;
    a.prof = reinterpret_cast<long long*>(prof.data_ptr<int64_t>());
    gc_ok(eh_gc_step(&a, gc_stream()), "gc_step(prof)");
    gc_ok(eh_gc_reduce(&r_, gc_stream()), "gc_reduce");
    return prof;
  }
  torch::Tensor gidx() const { return gidx_; }
  int64_t lds_bytes() const { return a_.lds_bytes; }
  bool z_kept() const { return a_.zst != 0; }

 private:
  py::dict d_;
  c10::Device dev_{c10::kCPU};
  GcStepArgs a_{};
  GcReduceArgs r_{}, ro_{};
  std::vector<torch::Tensor> keep_, opt_keep_;
  torch::Tensor slab_, loss_part_, acc_part_, gidx_;
  int64_t max_lds_ = 160 * 1024;  // "max_lds" in the dict: a smaller budget (tests of the global-weight path)

  void layout(int64_t dmax) {
    GcStepArgs& a = a_;
    int64_t off = 0;
    auto take = [&](int64_t bytes) {
      const int64_t o = off;
      off += (bytes + 15) / 16 * 16;
      return static_cast<int32_t>(o);
    };
    const int64_t nmax = a.nmax;
    for (int l = 0; l <= a.L; ++l) {
      a.ldx[l] = a.D[l] + 4;
      a.lds_x[l] = take(nmax * a.ldx[l] * 4);
    }
    const int64_t kmax = a.kind == 1 ? 2 * dmax : dmax;
    a.ldz = static_cast<int32_t>(kmax + 4);
    a.ldy = static_cast<int32_t>(dmax + 4);
    a.lda = static_cast<int32_t>(nmax + 4);
    a.trp = (a.tab_rows + 15) / 16 * 16;
    a.ldsm = a.trp + 4;
    a.ldt = a.D[0] + 4;
    a.lds_dz = take(nmax * a.ldz * 4);
    a.lds_dy = take(nmax * a.ldy * 4);
    a.lds_vec = take((5 * kGcMaxWidth + 4 * kGcMaxLabels) * 4);
    a.lds_a = take(a.nadj * nmax * a.lda * 4);
    a.lds_invc = take(a.nadj * nmax * 4);
    a.lds_s = take(nmax * a.ldsm * 4);
    a.lds_t = take(static_cast<int64_t>(a.trp) * a.ldt * 4);
    a.lds_csum = take(static_cast<int64_t>(kGcMaxRows / 16) * kGcMaxWidth * 4);
    const int64_t z1 = nmax * a.ldz * 4;
    a.lds_z = take(z1);
    TORCH_CHECK(off <= 160 * 1024, "GraphClsPlan: the step needs ", off, " bytes of LDS (> 160 KB)");
    // when it fits: every conv's Z kept for its backward (no recomputed aggregate)
    a.zst = off + (a.L - 1) * z1 <= max_lds_ ? 1 : 0;
    if (a.zst) off += (a.L - 1) * ((z1 + 15) / 16 * 16);
    a.lds_bytes = static_cast<int32_t>(off);
  }

  bool has(const char* k) const { return d_.contains(k) && !d_[k].is_none(); }
  int64_t geti(const char* k) const {
    TORCH_CHECK(d_.contains(k), "GraphClsPlan: missing '", k, "'");
    return d_[k].cast<int64_t>();
  }
  std::vector<int64_t> getv(const char* k) const {
    TORCH_CHECK(d_.contains(k), "GraphClsPlan: missing '", k, "'");
    return d_[k].cast<std::vector<int64_t>>();
  }
  torch::Tensor T(const char* k) const {
    TORCH_CHECK(has(k), "GraphClsPlan: missing tensor '", k, "'");
    return d_[k].cast<torch::Tensor>();
  }
  void need(const torch::Tensor& t, c10::ScalarType st, int64_t numel, const std::string& name) const {
    TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
    if (dev_.is_cuda()) TORCH_CHECK(t.device() == dev_, name, " must be on the plan's GPU");
    TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
    TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
    if (numel >= 0) TORCH_CHECK(t.numel() == numel, name, " has ", t.numel(), " elements, expected ", numel);
  }
};

}  // namespace

void register_graph_cls_ops(py::module& m) {
  py::class_<GraphClsPlan>(m, "GraphClsPlan")
      .def(py::init<py::dict>())
      .def("step", &GraphClsPlan::step, py::arg("fused_opt") = false)
      .def("set_optimizer", &GraphClsPlan::set_optimizer)
      .def("gidx", &GraphClsPlan::gidx)
      .def("profile", &GraphClsPlan::profile)
      .def_property_readonly("lds_bytes", &GraphClsPlan::lds_bytes)
      .def_property_readonly("z_kept", &GraphClsPlan::z_kept);
}
