// torch binding for the euler_amd gfx950 kernels.  Host-only translation unit:
// validates every operand (shape, dtype, device, contiguity) before a launch —
// a kernel is never started on operands whose shapes disagree with the grid it
// assumes — and launches on torch's current HIP stream so the ops compose with
// torch streams and hipGraph capture.
#include <c10/hip/HIPStream.h>
#include <cstring>
#include <string>
#include <vector>
#include <c10/hip/HIPGuard.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>

#include "hip/launchers.h"

namespace {

hipStream_t cur_stream() { return c10::hip::getCurrentHIPStream().stream(); }

void check(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "euler_amd HIP kernel '", what, "' failed: ", hipGetErrorString(e));
}

void need_cuda(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void need_i32(const torch::Tensor& t, const char* name) {
  need_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kInt32, name, " must be int32");
}

void need_i64(const torch::Tensor& t, const char* name) {
  need_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kInt64, name, " must be int64");
}

bool is_bf16(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16 || t.scalar_type() == torch::kFloat32, name,
              " must be bfloat16 or float32");
  return t.scalar_type() == torch::kBFloat16;
}

const void* opt_ptr(const c10::optional<torch::Tensor>& t) { return t.has_value() ? t->data_ptr() : nullptr; }

// ----------------------------------------------------------------------------- sampling
void rng_advance(torch::Tensor state, int64_t inc) {
  need_i64(state, "rng_state");
  TORCH_CHECK(state.numel() == 2, "rng_state must have 2 elements");
  const c10::DeviceGuard g(state.device());
  check(eh_rng_advance(state.data_ptr<int64_t>(), inc, cur_stream()), "rng_advance");
}

std::vector<torch::Tensor> sample_neighbor(torch::Tensor indptr, torch::Tensor nbr, torch::Tensor cumw,
                                           int64_t num_rows, int64_t num_types, int64_t type_mask,
                                           torch::Tensor nodes, int64_t count, int64_t default_row,
                                           torch::Tensor rng, int64_t stream_id, bool with_wt) {
  need_i64(indptr, "indptr");
  need_i32(nbr, "nbr");
  need_cuda(cumw, "cumw");
  need_i64(rng, "rng_state");
  need_cuda(nodes, "nodes");
  TORCH_CHECK(cumw.scalar_type() == torch::kFloat32, "cumw must be float32");
  TORCH_CHECK(indptr.numel() == num_rows * num_types + 1, "indptr size mismatch: ", indptr.numel(), " vs ",
              num_rows * num_types + 1);
  TORCH_CHECK(nbr.numel() == cumw.numel(), "nbr/cumw size mismatch");
  TORCH_CHECK(nodes.scalar_type() == torch::kInt32 || nodes.scalar_type() == torch::kInt64, "nodes must be int");
  TORCH_CHECK(num_types >= 1 && num_types <= 32, "num_types must be in [1, 32]");
  TORCH_CHECK(count >= 0, "count must be >= 0");
  const c10::DeviceGuard g(nodes.device());
  const int64_t n = nodes.numel();
  auto opts = nodes.options().dtype(torch::kInt32);
  auto out = torch::empty({n, count}, opts);
  torch::Tensor w, t;
  if (with_wt) {
    w = torch::empty({n, count}, opts.dtype(torch::kFloat32));
    t = torch::empty({n, count}, opts);
  }
  check(eh_sample_neighbor(indptr.data_ptr<int64_t>(), nbr.data_ptr<int32_t>(), cumw.data_ptr<float>(), num_rows,
                           static_cast<int>(num_types), static_cast<uint32_t>(type_mask), nodes.data_ptr(),
                           nodes.scalar_type() == torch::kInt64, n, static_cast<int>(count),
                           static_cast<int32_t>(default_row), rng.data_ptr<int64_t>(),
                           static_cast<uint64_t>(stream_id), out.data_ptr<int32_t>(),
                           with_wt ? w.data_ptr<float>() : nullptr, with_wt ? t.data_ptr<int32_t>() : nullptr,
                           cur_stream()),
        "sample_neighbor");
  if (with_wt) return {out, w, t};
  return {out};
}

torch::Tensor alias_sample(torch::Tensor prob, torch::Tensor alias, c10::optional<torch::Tensor> rows, int64_t count,
                           torch::Tensor rng, int64_t stream_id) {
  need_cuda(prob, "prob");
  need_i32(alias, "alias");
  need_i64(rng, "rng_state");
  TORCH_CHECK(prob.scalar_type() == torch::kFloat32, "prob must be float32");
  TORCH_CHECK(prob.numel() == alias.numel() && prob.numel() > 0, "prob/alias size mismatch or empty");
  if (rows.has_value()) {
    need_i32(*rows, "rows");
    TORCH_CHECK(rows->numel() == prob.numel(), "rows size mismatch");
  }
  const c10::DeviceGuard g(prob.device());
  auto out = torch::empty({count}, prob.options().dtype(torch::kInt32));
  check(eh_alias_sample(prob.data_ptr<float>(), alias.data_ptr<int32_t>(),
                        rows.has_value() ? rows->data_ptr<int32_t>() : nullptr, prob.numel(), count,
                        rng.data_ptr<int64_t>(), static_cast<uint64_t>(stream_id), out.data_ptr<int32_t>(),
                        cur_stream()),
        "alias_sample");
  return out;
}

torch::Tensor random_walk(torch::Tensor indptr, torch::Tensor nbr, torch::Tensor cumw, int64_t num_rows,
                          int64_t num_types, torch::Tensor step_masks, torch::Tensor starts, int64_t default_row,
                          torch::Tensor rng, int64_t stream_id, double p, double q) {
  TORCH_CHECK(p > 0.0 && q > 0.0, "random_walk: p and q must be positive");
  need_i64(indptr, "indptr");
  need_i32(nbr, "nbr");
  need_cuda(cumw, "cumw");
  need_i32(starts, "starts");
  need_i32(step_masks, "step_masks");
  need_i64(rng, "rng_state");
  TORCH_CHECK(indptr.numel() == num_rows * num_types + 1, "indptr size mismatch");
  const c10::DeviceGuard g(starts.device());
  const int64_t walk_len = step_masks.numel();
  auto out = torch::empty({starts.numel(), walk_len + 1}, starts.options());
  check(eh_random_walk(indptr.data_ptr<int64_t>(), nbr.data_ptr<int32_t>(), cumw.data_ptr<float>(), num_rows,
                       static_cast<int>(num_types), reinterpret_cast<const uint32_t*>(step_masks.data_ptr<int32_t>()),
                       starts.data_ptr<int32_t>(), starts.numel(), static_cast<int>(walk_len),
                       static_cast<int32_t>(default_row), rng.data_ptr<int64_t>(), static_cast<uint64_t>(stream_id),
                       static_cast<float>(p), static_cast<float>(q), out.data_ptr<int32_t>(), cur_stream()),
        "random_walk");
  return out;
}

std::vector<torch::Tensor> synth_csr(int64_t n, double avg_deg, int64_t max_deg, int64_t seed, int64_t device) {
  TORCH_CHECK(n > 0 && n < (1ll << 31), "synth_csr: n must be in (0, 2^31)");
  const c10::DeviceGuard g(c10::Device(c10::DeviceType::CUDA, static_cast<c10::DeviceIndex>(device)));
  auto opts = torch::TensorOptions().device(torch::kCUDA, device);
  auto deg = torch::empty({n}, opts.dtype(torch::kInt64));
  check(eh_synth_degree(n, static_cast<float>(avg_deg), static_cast<int>(max_deg), static_cast<uint64_t>(seed),
                        deg.data_ptr<int64_t>(), cur_stream()),
        "synth_degree");
  auto indptr = torch::zeros({n + 1}, opts.dtype(torch::kInt64));
  indptr.slice(0, 1).copy_(torch::cumsum(deg, 0));
  const int64_t e = indptr[n].item<int64_t>();
  auto nbr = torch::empty({e}, opts.dtype(torch::kInt32));
  auto cumw = torch::empty({e}, opts.dtype(torch::kFloat32));
  check(eh_synth_fill(n, indptr.data_ptr<int64_t>(), static_cast<uint64_t>(seed), nbr.data_ptr<int32_t>(),
                      cumw.data_ptr<float>(), cur_stream()),
        "synth_fill");
  return {indptr, nbr, cumw};
}

// ----------------------------------------------------------------------------- fused SAGE layer
void check_sage_operands(const torch::Tensor& x, const torch::Tensor& self_idx, const torch::Tensor& nbr_idx,
                         const torch::Tensor& W) {
  need_cuda(x, "x");
  need_i32(self_idx, "self_idx");
  need_i32(nbr_idx, "nbr_idx");
  need_cuda(W, "weight");
  TORCH_CHECK(x.scalar_type() == torch::kBFloat16 && W.scalar_type() == torch::kBFloat16,
              "fused sage layer needs bf16 x and weight");
  TORCH_CHECK(x.dim() == 2 && W.dim() == 2 && nbr_idx.dim() == 2, "x, weight, nbr_idx must be 2-D");
  TORCH_CHECK(self_idx.numel() == nbr_idx.size(0), "self_idx / nbr_idx row mismatch");
  TORCH_CHECK(W.size(1) == 2 * x.size(1), "weight must be [H, 2*D]");
  TORCH_CHECK(x.size(1) % 16 == 0 && x.size(1) <= 512, "fused sage layer needs D % 16 == 0 and D <= 512");
}

std::vector<torch::Tensor> sage_fwd(torch::Tensor x, torch::Tensor self_idx, torch::Tensor nbr_idx,
                                    torch::Tensor W, c10::optional<torch::Tensor> bias, bool include_self,
                                    bool relu, bool save_a) {
  check_sage_operands(x, self_idx, nbr_idx, W);
  if (bias.has_value()) {
    need_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == W.size(0), "bias must be fp32 [H]");
  }
  const c10::DeviceGuard g(x.device());
  const int64_t M = nbr_idx.size(0), F = nbr_idx.size(1), D = x.size(1), H = W.size(0);
  auto out = torch::empty({M, H}, x.options());
  torch::Tensor a;
  if (save_a) a = torch::empty({M, 2 * D}, x.options());
  const float inv_cnt = 1.f / static_cast<float>(F + (include_self ? 1 : 0));
  check(eh_sage_fwd(x.data_ptr(), static_cast<int>(D), self_idx.data_ptr<int32_t>(), nbr_idx.data_ptr<int32_t>(),
                    static_cast<int>(F), include_self, inv_cnt, W.data_ptr(),
                    bias.has_value() ? bias->data_ptr<float>() : nullptr, static_cast<int>(H), M, out.data_ptr(),
                    save_a ? a.data_ptr() : nullptr, relu, cur_stream()),
        "sage_fwd");
  if (save_a) return {out, a};
  return {out};
}

torch::Tensor linear_fwd(torch::Tensor A, torch::Tensor W, c10::optional<torch::Tensor> bias, bool relu) {
  need_cuda(A, "A");
  need_cuda(W, "weight");
  TORCH_CHECK(A.scalar_type() == torch::kBFloat16 && W.scalar_type() == torch::kBFloat16, "linear needs bf16");
  TORCH_CHECK(A.dim() == 2 && W.dim() == 2 && W.size(1) == A.size(1), "linear shape mismatch");
  TORCH_CHECK(A.size(1) % 32 == 0 && A.size(1) <= 1024, "linear needs K % 32 == 0 and K <= 1024");
  if (bias.has_value()) {
    need_cuda(*bias, "bias");
    TORCH_CHECK(bias->scalar_type() == torch::kFloat32 && bias->numel() == W.size(0), "bias must be fp32 [H]");
  }
  const c10::DeviceGuard g(A.device());
  auto out = torch::empty({A.size(0), W.size(0)}, A.options());
  check(eh_linear_fwd(A.data_ptr(), static_cast<int>(A.size(1)), W.data_ptr(),
                      bias.has_value() ? bias->data_ptr<float>() : nullptr, static_cast<int>(W.size(0)), A.size(0),
                      out.data_ptr(), relu, cur_stream()),
        "linear_fwd");
  return out;
}

void sage_bwd_scatter(torch::Tensor dA, torch::Tensor self_idx, torch::Tensor nbr_idx, bool include_self,
                      bool disjoint, torch::Tensor dx) {
  need_cuda(dA, "dA");
  need_i32(self_idx, "self_idx");
  need_i32(nbr_idx, "nbr_idx");
  need_cuda(dx, "dx");
  TORCH_CHECK(dA.scalar_type() == torch::kBFloat16, "dA must be bf16");
  TORCH_CHECK(dx.scalar_type() == torch::kFloat32, "dx must be fp32");
  const int64_t M = nbr_idx.size(0), F = nbr_idx.size(1), D = dx.size(1);
  TORCH_CHECK(dA.size(0) == M && dA.size(1) == 2 * D, "dA must be [M, 2D]");
  TORCH_CHECK(self_idx.numel() == M, "self_idx size mismatch");
  TORCH_CHECK(D % 8 == 0, "D must be a multiple of 8");
  const c10::DeviceGuard g(dA.device());
  const float inv_cnt = 1.f / static_cast<float>(F + (include_self ? 1 : 0));
  check(eh_sage_bwd_scatter(dA.data_ptr(), static_cast<int>(D), self_idx.data_ptr<int32_t>(),
                            nbr_idx.data_ptr<int32_t>(), static_cast<int>(F), include_self, inv_cnt, M, disjoint,
                            dx.data_ptr<float>(), cur_stream()),
        "sage_bwd_scatter");
}

void relu_bwd_(torch::Tensor g, torch::Tensor y) {
  need_cuda(g, "grad");
  need_cuda(y, "y");
  TORCH_CHECK(g.scalar_type() == torch::kBFloat16 && y.scalar_type() == torch::kBFloat16, "relu_bwd needs bf16");
  TORCH_CHECK(g.numel() == y.numel() && g.numel() % 8 == 0, "relu_bwd size mismatch / not a multiple of 8");
  const c10::DeviceGuard gd(g.device());
  check(eh_relu_bwd(g.data_ptr(), y.data_ptr(), g.numel(), cur_stream()), "relu_bwd");
}

// ----------------------------------------------------------------------------- message passing
// out [n, D] fp32 = sum over f of x[idx[:, f]] (idx [n, F] int64; -1 entries skipped)
torch::Tensor gather_sum(torch::Tensor x, torch::Tensor idx) {
  need_cuda(x, "x");
  need_i64(idx, "idx");
  const bool bf = is_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2 && x.is_contiguous() && idx.dim() == 2 && idx.is_contiguous(),
              "gather_sum: x [N, D] and idx [n, F] must be contiguous");
  TORCH_CHECK((x.size(1) * x.element_size()) % 16 == 0, "gather_sum: rows must be a multiple of 16 bytes");
  const c10::DeviceGuard g(x.device());
  auto out = torch::empty({idx.size(0), x.size(1)}, x.options().dtype(torch::kFloat32));
  check(eh_gather_sum(x.data_ptr(), bf, x.size(0), x.size(1) * x.element_size(), idx.data_ptr<int64_t>(), idx.size(0),
                      static_cast<int>(idx.size(1)), out.data_ptr<float>(), cur_stream()),
        "gather_sum");
  return out;
}

torch::Tensor gather_rows(torch::Tensor x, torch::Tensor idx) {
  need_cuda(x, "x");
  need_cuda(idx, "idx");
  TORCH_CHECK(idx.scalar_type() == torch::kInt32 || idx.scalar_type() == torch::kInt64, "idx must be int");
  TORCH_CHECK(x.dim() >= 1, "x must have a row dimension");
  const c10::DeviceGuard g(x.device());
  auto sizes = x.sizes().vec();
  sizes[0] = idx.numel();
  auto out = torch::empty(sizes, x.options());
  const int64_t row_bytes = x.dim() == 1 ? x.element_size() : x.stride(0) * x.element_size();
  check(eh_gather_rows(x.data_ptr(), x.size(0), row_bytes, idx.data_ptr(), idx.scalar_type() == torch::kInt64,
                       idx.numel(), out.data_ptr(), cur_stream()),
        "gather_rows");
  return out;
}

std::vector<torch::Tensor> segment_reduce(torch::Tensor src, torch::Tensor indptr, c10::optional<torch::Tensor> perm,
                                          int64_t op, double empty_val) {
  need_cuda(src, "src");
  need_i64(indptr, "indptr");
  const bool bf = is_bf16(src, "src");
  TORCH_CHECK(src.dim() == 2, "src must be 2-D");
  if (perm.has_value()) {
    need_i64(*perm, "perm");
    TORCH_CHECK(perm->numel() == src.size(0), "perm must cover src rows");
  }
  TORCH_CHECK(op >= 0 && op <= 2, "op must be 0(sum) 1(mean) 2(max)");
  const c10::DeviceGuard g(src.device());
  const int64_t S = indptr.numel() - 1, D = src.size(1);
  auto out = torch::empty({S, D}, src.options());
  torch::Tensor am;
  if (op == 2) am = torch::empty({S, D}, src.options().dtype(torch::kInt64));
  check(eh_segment_reduce(src.data_ptr(), bf, static_cast<int>(D), indptr.data_ptr<int64_t>(),
                          perm.has_value() ? perm->data_ptr<int64_t>() : nullptr, S, static_cast<int>(op),
                          static_cast<float>(empty_val), out.data_ptr(), op == 2 ? am.data_ptr<int64_t>() : nullptr,
                          cur_stream()),
        "segment_reduce");
  if (op == 2) return {out, am};
  return {out};
}

// wave-per-segment sum / mean (skewed segment lengths); D / (8 bf16 | 4 fp32) a power of two <= 64
torch::Tensor segment_reduce_wave(torch::Tensor src, torch::Tensor indptr, c10::optional<torch::Tensor> perm,
                                  int64_t op, c10::optional<torch::Tensor> out_) {
  need_cuda(src, "src");
  need_i64(indptr, "indptr");
  const bool bf = is_bf16(src, "src");
  TORCH_CHECK(src.dim() == 2 && src.is_contiguous(), "src must be a contiguous 2-D tensor");
  if (perm.has_value()) {
    need_i64(*perm, "perm");
    TORCH_CHECK(perm->numel() == src.size(0), "perm must cover src rows");
  }
  TORCH_CHECK(op == 0 || op == 1, "op must be 0(sum) 1(mean)");
  const int64_t S = indptr.numel() - 1, D = src.size(1), LP = D / (bf ? 8 : 4);
  TORCH_CHECK(D % (bf ? 8 : 4) == 0 && LP <= 64 && (LP & (LP - 1)) == 0,
              "segment_reduce_wave needs D / (8 bf16 | 4 fp32) to be a power of two <= 64");
  const c10::DeviceGuard g(src.device());
  torch::Tensor out;
  if (out_.has_value()) {  // written in place (every row: empty segments get zeros)
    out = *out_;
    TORCH_CHECK(out.scalar_type() == src.scalar_type() && out.is_contiguous() && out.dim() == 2 &&
                    out.size(0) == S && out.size(1) == D && out.device() == src.device(),
                "segment_reduce_wave: out must be a contiguous [S, D] tensor like src");
  } else {
    out = torch::empty({S, D}, src.options());
  }
  check(eh_segment_reduce_wave(src.data_ptr(), bf, static_cast<int>(D), indptr.data_ptr<int64_t>(),
                               perm.has_value() ? perm->data_ptr<int64_t>() : nullptr, S, static_cast<int>(op),
                               out.data_ptr(), cur_stream()),
        "segment_reduce_wave");
  return out;
}

void index_add_rows_(torch::Tensor out, torch::Tensor idx, torch::Tensor src) {
  need_cuda(out, "out");
  need_i64(idx, "idx");
  need_cuda(src, "src");
  TORCH_CHECK(out.scalar_type() == torch::kFloat32, "out must be fp32");
  const bool bf = is_bf16(src, "src");
  TORCH_CHECK(src.dim() == 2 && out.dim() == 2 && src.size(1) == out.size(1) && src.size(0) == idx.numel(),
              "index_add_rows shape mismatch");
  const c10::DeviceGuard g(src.device());
  check(eh_index_add_rows(src.data_ptr(), bf, static_cast<int>(src.size(1)), idx.data_ptr<int64_t>(), idx.numel(),
                          out.data_ptr<float>(), out.size(0), cur_stream()),
        "index_add_rows");
}

torch::Tensor max_bwd(torch::Tensor gout, torch::Tensor argmax, int64_t n_src) {
  need_cuda(gout, "grad_out");
  need_i64(argmax, "argmax");
  const bool bf = is_bf16(gout, "grad_out");
  TORCH_CHECK(gout.sizes() == argmax.sizes() && gout.dim() == 2, "max_bwd shape mismatch");
  const c10::DeviceGuard g(gout.device());
  auto gsrc = torch::zeros({n_src, gout.size(1)}, gout.options());
  check(eh_max_bwd(gout.data_ptr(), bf, argmax.data_ptr<int64_t>(), gout.size(0), static_cast<int>(gout.size(1)),
                   gsrc.data_ptr(), cur_stream()),
        "max_bwd");
  return gsrc;
}

torch::Tensor edge_softmax(torch::Tensor logits, torch::Tensor indptr, c10::optional<torch::Tensor> perm) {
  need_cuda(logits, "logits");
  need_i64(indptr, "indptr");
  const bool bf = is_bf16(logits, "logits");
  TORCH_CHECK(logits.dim() == 2, "logits must be [E, H]");
  if (perm.has_value()) {
    need_i64(*perm, "perm");
    TORCH_CHECK(perm->numel() == logits.size(0), "perm must cover every edge");
  }
  const c10::DeviceGuard g(logits.device());
  auto out = torch::zeros_like(logits);
  check(eh_edge_softmax(logits.data_ptr(), bf, static_cast<int>(logits.size(1)), indptr.data_ptr<int64_t>(),
                        perm.has_value() ? perm->data_ptr<int64_t>() : nullptr, indptr.numel() - 1, out.data_ptr(),
                        cur_stream()),
        "edge_softmax");
  return out;
}

torch::Tensor edge_softmax_bwd(torch::Tensor p, torch::Tensor grad, torch::Tensor indptr,
                               c10::optional<torch::Tensor> perm) {
  need_cuda(p, "p");
  need_cuda(grad, "grad");
  need_i64(indptr, "indptr");
  const bool bf = is_bf16(p, "p");
  TORCH_CHECK(p.sizes() == grad.sizes() && p.scalar_type() == grad.scalar_type(), "edge_softmax_bwd mismatch");
  if (perm.has_value()) need_i64(*perm, "perm");
  const c10::DeviceGuard g(p.device());
  auto gin = torch::zeros_like(p);
  check(eh_edge_softmax_bwd(p.data_ptr(), grad.data_ptr(), bf, static_cast<int>(p.size(1)),
                            indptr.data_ptr<int64_t>(), perm.has_value() ? perm->data_ptr<int64_t>() : nullptr,
                            indptr.numel() - 1, gin.data_ptr(), cur_stream()),
        "edge_softmax_bwd");
  return gin;
}

torch::Tensor spmm_csr(torch::Tensor indptr, torch::Tensor col, c10::optional<torch::Tensor> w, torch::Tensor x) {
  need_i64(indptr, "indptr");
  need_i64(col, "col");
  need_cuda(x, "x");
  const bool bf = is_bf16(x, "x");
  TORCH_CHECK(x.dim() == 2, "x must be 2-D");
  if (w.has_value()) {
    need_cuda(*w, "w");
    TORCH_CHECK(w->scalar_type() == torch::kFloat32 && w->numel() == col.numel(), "w must be fp32 [nnz]");
  }
  const c10::DeviceGuard g(x.device());
  const int64_t S = indptr.numel() - 1;
  auto out = torch::empty({S, x.size(1)}, x.options());
  check(eh_spmm_csr(indptr.data_ptr<int64_t>(), col.data_ptr<int64_t>(),
                    w.has_value() ? w->data_ptr<float>() : nullptr, x.data_ptr(), bf, static_cast<int>(x.size(1)), S,
                    out.data_ptr(), cur_stream()),
        "spmm_csr");
  return out;
}

// ----------------------------------------------------------------------------- optimizers
void flat_optim_(torch::Tensor p, torch::Tensor g, torch::Tensor m, torch::Tensor v, torch::Tensor step, double lr,
                 double b1, double b2, double eps, double wd, double grad_scale, int64_t kind,
                 c10::optional<torch::Tensor> ticket, double wd2, int64_t w0, int64_t w1) {
  for (auto* t : {&p, &g, &m, &v}) {
    need_cuda(*t, "optimizer buffer");
    TORCH_CHECK(t->scalar_type() == torch::kFloat32 && t->numel() == p.numel() && t->is_contiguous(),
                "optimizer buffers: fp32, same size, contiguous");
  }
  need_i64(step, "step");
  int32_t* tk = nullptr;
  if (ticket.has_value()) {
    need_cuda(*ticket, "ticket");
    TORCH_CHECK(ticket->scalar_type() == torch::kInt32 && ticket->numel() >= 1, "ticket: int32 [1]");
    tk = ticket->data_ptr<int32_t>();
  }
  const c10::DeviceGuard gd(p.device());
  check(eh_flat_optim2(p.data_ptr<float>(), g.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), p.numel(),
                       step.data_ptr<int64_t>(), tk, static_cast<float>(lr), static_cast<float>(b1),
                       static_cast<float>(b2), static_cast<float>(eps), static_cast<float>(wd), static_cast<float>(wd2),
                       w0, w1, static_cast<float>(grad_scale), static_cast<int>(kind), cur_stream()),
        "flat_optim");
}

void sparse_optim_(torch::Tensor table, torch::Tensor m, torch::Tensor v, torch::Tensor rows, torch::Tensor grads,
                   torch::Tensor step, double lr, double b1, double b2, double eps, int64_t kind) {
  need_cuda(table, "table");
  need_cuda(m, "m");
  need_cuda(v, "v");
  need_i64(rows, "rows");
  need_cuda(grads, "grads");
  need_i64(step, "step");
  const bool gbf = grads.scalar_type() == torch::kBFloat16;
  TORCH_CHECK(table.scalar_type() == torch::kFloat32 && (gbf || grads.scalar_type() == torch::kFloat32),
              "fp32 table, fp32 or bf16 grads");
  TORCH_CHECK(grads.is_contiguous() && (!gbf || table.size(1) % 4 == 0), "contiguous grads (bf16: D % 4 == 0)");
  TORCH_CHECK(table.dim() == 2 && grads.dim() == 2 && grads.size(1) == table.size(1) && grads.size(0) == rows.numel(),
              "sparse_optim shape mismatch");
  TORCH_CHECK(m.sizes() == table.sizes() && v.sizes() == table.sizes(), "optimizer state shape mismatch");
  const c10::DeviceGuard gd(table.device());
  check(eh_sparse_optim(table.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), rows.data_ptr<int64_t>(),
                        grads.data_ptr(), gbf ? 1 : 0, rows.numel(), static_cast<int>(table.size(1)), table.size(0),
                        step.data_ptr<int64_t>(), static_cast<float>(lr), static_cast<float>(b1),
                        static_cast<float>(b2), static_cast<float>(eps), static_cast<int>(kind), cur_stream()),
        "sparse_optim");
}

// ----------------------------------------------------------------------------- fused SAGE training step
void need_bf16(const torch::Tensor& t, const char* name) {
  need_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16, name, " must be bfloat16");
}

void need_f32(const torch::Tensor& t, const char* name) {
  need_cuda(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kFloat32, name, " must be float32");
}

// sample_neighbor writing into a caller-provided int32 buffer (no allocation)
void sample_neighbor_into(torch::Tensor indptr, torch::Tensor nbr, torch::Tensor cumw, int64_t num_rows,
                          int64_t num_types, int64_t type_mask, torch::Tensor nodes, int64_t count,
                          int64_t default_row, torch::Tensor rng, int64_t stream_id, torch::Tensor out) {
  need_i64(indptr, "indptr");
  need_i32(nbr, "nbr");
  need_f32(cumw, "cumw");
  need_i64(rng, "rng_state");
  need_i32(nodes, "nodes");
  need_i32(out, "out");
  TORCH_CHECK(indptr.numel() == num_rows * num_types + 1, "indptr size mismatch");
  TORCH_CHECK(nbr.numel() == cumw.numel(), "nbr/cumw size mismatch");
  TORCH_CHECK(num_types >= 1 && num_types <= 32, "num_types must be in [1, 32]");
  TORCH_CHECK(out.numel() >= nodes.numel() * count, "out too small");
  const c10::DeviceGuard g(nodes.device());
  check(eh_sample_neighbor(indptr.data_ptr<int64_t>(), nbr.data_ptr<int32_t>(), cumw.data_ptr<float>(), num_rows,
                           static_cast<int>(num_types), static_cast<uint32_t>(type_mask), nodes.data_ptr(), 0,
                           nodes.numel(), static_cast<int>(count), static_cast<int32_t>(default_row),
                           rng.data_ptr<int64_t>(), static_cast<uint64_t>(stream_id), out.data_ptr<int32_t>(),
                           nullptr, nullptr, cur_stream()),
        "sample_neighbor_into");
}


// ----------------------------------------------------------------------------- xGMI all-reduce
// One rank's side of the two-shot peer-memory all-reduce (xgmi_ar.hip): owns the rank's
// uncached IPC buffer, maps the peers' buffers from their IPC handles, launches the kernel on
// the current stream (hipGraph-capturable: no allocation, no sync).
class XgmiAr : public std::enable_shared_from_this<XgmiAr> {
 public:
  XgmiAr(int64_t cap, double timeout_s) : cap_(cap) {
    TORCH_CHECK(cap > 0 && cap % 16 == 0, "xgmi all-reduce capacity must be a positive multiple of 16 bytes");
    check(hipGetDevice(&dev_), "xar get device");
    check(eh_xar_alloc(cap, &own_sig_, &own_buf_), "xar alloc");
    check(hipMalloc(reinterpret_cast<void**>(&epoch_), eh_xar_max_blocks() * sizeof(uint32_t)), "xar epoch");
    check(hipMalloc(reinterpret_cast<void**>(&err_), sizeof(int)), "xar err");
    check(hipMemset(epoch_, 0, eh_xar_max_blocks() * sizeof(uint32_t)), "xar epoch zero");
    check(hipMemset(err_, 0, sizeof(int)), "xar err zero");
    int khz = 0;
    check(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev_), "xar wall clock rate");
    timeout_ = static_cast<long long>(timeout_s * 1000.0 * (khz > 0 ? khz : 100000));
    check(hipDeviceSynchronize(), "xar init sync");
  }
  ~XgmiAr() {
    hipSetDevice(dev_);
    for (size_t r = 0; r < bufs_.size(); ++r) {
      if (static_cast<int>(r) == rank_) continue;
      if (sigs_[r]) hipIpcCloseMemHandle(sigs_[r]);
      if (bufs_[r]) hipIpcCloseMemHandle(bufs_[r]);
    }
    if (own_sig_) hipFree(own_sig_);
    if (own_buf_) hipFree(own_buf_);
    if (epoch_) hipFree(epoch_);
    if (err_) hipFree(err_);
  }
  // the flag area's handle followed by the data area's
  py::bytes handle() const {
    hipIpcMemHandle_t h[2];
    check(hipIpcGetMemHandle(&h[0], own_sig_), "xar ipc handle (flags)");
    check(hipIpcGetMemHandle(&h[1], own_buf_), "xar ipc handle (data)");
    return py::bytes(reinterpret_cast<const char*>(h), sizeof(h));
  }
  void open(const std::vector<std::string>& handles, int rank) {
    const int world = static_cast<int>(handles.size());
    TORCH_CHECK(world >= 1 && world <= eh_xar_max_ranks() && rank >= 0 && rank < world, "xar: bad world/rank");
    TORCH_CHECK(bufs_.empty(), "xar: peers already opened");
    sigs_.assign(world, nullptr);
    bufs_.assign(world, nullptr);
    rank_ = rank;
    for (int r = 0; r < world; ++r) {
      if (r == rank) {
        sigs_[r] = own_sig_;
        bufs_[r] = own_buf_;
        continue;
      }
      TORCH_CHECK(handles[r].size() == 2 * sizeof(hipIpcMemHandle_t), "xar: bad ipc handle size");
      hipIpcMemHandle_t h[2];
      std::memcpy(h, handles[r].data(), sizeof(h));
      check(hipIpcOpenMemHandle(&sigs_[r], h[0], hipIpcMemLazyEnablePeerAccess), "xar ipc open (flags)");
      check(hipIpcOpenMemHandle(&bufs_[r], h[1], hipIpcMemLazyEnablePeerAccess), "xar ipc open (data)");
    }
  }
  void run(torch::Tensor t, int64_t blocks) {
    need_cuda(t, "xgmi all-reduce tensor");
    TORCH_CHECK(!bufs_.empty(), "xar: open() the peers first");
    TORCH_CHECK(t.get_device() == dev_, "xar: tensor on another device");
    const bool bf = is_bf16(t, "xgmi all-reduce tensor");
    check(eh_xar_run(sigs_.data(), bufs_.data(), static_cast<int>(bufs_.size()), rank_, t.data_ptr(), bf ? 1 : 0,
                     t.numel(), cap_, static_cast<int>(blocks), epoch_, err_, timeout_, cur_stream()),
          "xgmi_allreduce");
  }
  int error() const {
    int v = 0;
    check(hipMemcpy(&v, err_, sizeof(int), hipMemcpyDeviceToHost), "xar read error");
    return v;
  }
  int64_t capacity() const { return cap_; }
  // a tensor over this rank's `in` region: a producer that writes its gradient here lets
  // run() reduce in place (no staging copy).  The tensor's deleter holds a reference to
  // this object, so the IPC region outlives every view (a trainer that adopted the view as
  // its gradient keeps it mapped after the Python all-reduce object is gone)
  torch::Tensor input_view(int64_t numel, bool bf16) {
    const int64_t esz = bf16 ? 2 : 4;
    TORCH_CHECK(numel >= 0 && numel * esz <= cap_, "xar: input view exceeds the capacity");
    auto opts = torch::TensorOptions().dtype(bf16 ? torch::kBFloat16 : torch::kFloat32).device(torch::kCUDA, dev_);
    std::shared_ptr<XgmiAr> keep = shared_from_this();
    return torch::from_blob(own_buf_, {numel}, [keep](void*) mutable { keep.reset(); }, opts);
  }

 private:
  int64_t cap_;
  int dev_ = 0, rank_ = -1;
  void* own_sig_ = nullptr;
  void* own_buf_ = nullptr;
  uint32_t* epoch_ = nullptr;
  int* err_ = nullptr;
  long long timeout_ = 0;
  std::vector<void*> sigs_, bufs_;
};

}  // namespace

// binding_gnn.cpp: GAT / R-GCN / embedding-loss / unique kernels
void register_gnn_ops(pybind11::module& m);
// binding_tree.cpp: fused GraphSAGE tree-step plan
void register_tree_ops(pybind11::module& m);
// binding_gcn.cpp: fused GCN step plan
void register_gcn_ops(pybind11::module& m);
// binding_graph_cls.cpp: fused graph-classification step plan
void register_graph_cls_ops(pybind11::module& m);

PYBIND11_MODULE(_hip_ops, m) {
  register_gnn_ops(m);
  register_tree_ops(m);
  register_gcn_ops(m);
  register_graph_cls_ops(m);
  m.doc() = "euler_amd hand-written CDNA4 (gfx950) HIP kernels";
  m.attr("arch") = "gfx950";
  m.def("rng_advance", &rng_advance);
  m.def("sample_neighbor", &sample_neighbor);
  m.def("alias_sample", &alias_sample);
  m.def("random_walk", &random_walk, py::arg("indptr"), py::arg("nbr"), py::arg("cumw"), py::arg("num_rows"),
        py::arg("num_types"), py::arg("step_masks"), py::arg("starts"), py::arg("default_row"), py::arg("rng"),
        py::arg("stream_id"), py::arg("p") = 1.0, py::arg("q") = 1.0);
  m.def("synth_csr", &synth_csr);
  m.def("sage_fwd", &sage_fwd);
  m.def("linear_fwd", &linear_fwd);
  m.def("sage_bwd_scatter", &sage_bwd_scatter);
  m.def("relu_bwd_", &relu_bwd_);
  m.def("gather_rows", &gather_rows);
  m.def("gather_sum", &gather_sum);
  m.def("segment_reduce", &segment_reduce);
  m.def("segment_reduce_wave", &segment_reduce_wave, py::arg("src"), py::arg("indptr"), py::arg("perm"), py::arg("op"),
        py::arg("out") = py::none());
  m.def("index_add_rows_", &index_add_rows_);
  m.def("max_bwd", &max_bwd);
  m.def("edge_softmax", &edge_softmax);
  m.def("edge_softmax_bwd", &edge_softmax_bwd);
  m.def("spmm_csr", &spmm_csr);
  m.def("flat_optim_", &flat_optim_, py::arg("p"), py::arg("g"), py::arg("m"), py::arg("v"), py::arg("step"),
        py::arg("lr"), py::arg("b1"), py::arg("b2"), py::arg("eps"), py::arg("wd"), py::arg("grad_scale"),
        py::arg("kind"), py::arg("ticket") = py::none(), py::arg("wd2") = 0.0, py::arg("w0") = 0, py::arg("w1") = 0);
  m.def("sparse_optim_", &sparse_optim_);
  m.def("sample_neighbor_into", &sample_neighbor_into);
  py::class_<XgmiAr, std::shared_ptr<XgmiAr>>(m, "XgmiAr")
      .def(py::init<int64_t, double>(), py::arg("capacity_bytes"), py::arg("timeout_s") = 2.0)
      .def("handle", &XgmiAr::handle)
      .def("open", &XgmiAr::open)
      .def("run", &XgmiAr::run)
      .def("error", &XgmiAr::error)
      .def("capacity", &XgmiAr::capacity)
      .def("input_view", &XgmiAr::input_view, py::arg("numel"), py::arg("bf16"));
  m.attr("xar_max_ranks") = eh_xar_max_ranks();
  m.attr("xar_max_blocks") = eh_xar_max_blocks();
  m.attr("xar_vec_per_thread") = eh_xar_vec_per_thread();
}
