// torch binding for the GAT / R-GCN / embedding / unique kernels (gat.hip, rgcn.hip,
// embed.hip, unique.hip).  Host-only, same rules as binding.cpp: every operand is
// validated (dtype, device, contiguity, shape) before a launch, launches go to torch's
// current HIP stream, outputs are allocated by torch's caching allocator.
#include <cstdlib>
#include <map>

#include <c10/hip/HIPGuard.h>
#include <c10/hip/HIPStream.h>
#include <hip/hip_runtime_api.h>
#include <torch/extension.h>

#include "hip/launchers.h"

namespace {

hipStream_t stream() { return c10::hip::getCurrentHIPStream().stream(); }

void ok(hipError_t e, const char* what) {
  TORCH_CHECK(e == hipSuccess, "euler_amd HIP kernel '", what, "' failed: ", hipGetErrorString(e));
}

void dev(const torch::Tensor& t, const char* name) {
  TORCH_CHECK(t.is_cuda(), name, " must be a GPU tensor");
  TORCH_CHECK(t.is_contiguous(), name, " must be contiguous");
}

void typed(const torch::Tensor& t, c10::ScalarType st, const char* name) {
  dev(t, name);
  TORCH_CHECK(t.scalar_type() == st, name, " has dtype ", t.scalar_type(), ", expected ", st);
}

bool bf16_or_f32(const torch::Tensor& t, const char* name) {
  dev(t, name);
  TORCH_CHECK(t.scalar_type() == torch::kBFloat16 || t.scalar_type() == torch::kFloat32, name,
              " must be bfloat16 or float32");
  return t.scalar_type() == torch::kBFloat16;
}

// ----------------------------------------------------------------------------- GAT
bool gat_supported(int64_t H, int64_t C, bool is_bf16) {
  return eh_gat_supported(static_cast<int>(H), static_cast<int>(C), is_bf16 ? 1 : 0) != 0;
}

void gat_common(const torch::Tensor& indptr, const torch::Tensor& col, const torch::Tensor& h,
                const torch::Tensor& al, const torch::Tensor& ar, int64_t H, int64_t C) {
  typed(indptr, torch::kInt64, "indptr");
  typed(col, torch::kInt32, "col");
  bf16_or_f32(h, "h");
  typed(al, torch::kFloat32, "al");
  typed(ar, torch::kFloat32, "ar");
  TORCH_CHECK(h.dim() == 2 && h.size(1) == H * C, "h must be [N, H*C]");
  TORCH_CHECK(al.dim() == 2 && al.size(0) == h.size(0) && al.size(1) == H, "al must be [N, H]");
  TORCH_CHECK(ar.dim() == 2 && ar.size(1) == H && ar.size(0) == indptr.numel() - 1, "ar must be [S, H]");
  TORCH_CHECK(gat_supported(H, C, h.scalar_type() == torch::kBFloat16), "GAT shape H=", H, " C=", C,
              " is not supported by the fused kernel");
}

const int32_t* order_ptr(const c10::optional<torch::Tensor>& order, int64_t rows, const char* name) {
  if (!order.has_value()) return nullptr;
  typed(*order, torch::kInt32, name);
  TORCH_CHECK(order->numel() == rows, name, " must be a permutation of the ", rows, " rows");
  return order->data_ptr<int32_t>();
}

const float* asrc_ptr(const c10::optional<torch::Tensor>& a_src, int64_t H, int64_t C) {
  if (!a_src.has_value()) return nullptr;
  typed(*a_src, torch::kFloat32, "a_src");
  TORCH_CHECK(a_src->numel() == H * C && a_src->is_contiguous(), "a_src must be a contiguous [H, C] fp32 tensor");
  return a_src->data_ptr<float>();
}

std::vector<torch::Tensor> gat_fwd(torch::Tensor indptr, torch::Tensor col, c10::optional<torch::Tensor> order,
                                   torch::Tensor h, torch::Tensor al, torch::Tensor ar, int64_t H, int64_t C,
                                   double slope, c10::optional<torch::Tensor> a_src) {
  gat_common(indptr, col, h, al, ar, H, C);
  const c10::DeviceGuard g(h.device());
  const int64_t S = indptr.numel() - 1;
  auto out = torch::empty({S, H * C}, h.options());
  auto lse = torch::empty({S, H}, al.options());
  ok(eh_gat_fwd(indptr.data_ptr<int64_t>(), col.data_ptr<int32_t>(), order_ptr(order, S, "order"), S, h.data_ptr(),
                h.scalar_type() == torch::kBFloat16, al.data_ptr<float>(), ar.data_ptr<float>(), static_cast<int>(H),
                static_cast<int>(C), static_cast<float>(slope), out.data_ptr(), lse.data_ptr<float>(),
                asrc_ptr(a_src, H, C), stream()),
     "gat_fwd");
  return {out, lse};
}

std::vector<torch::Tensor> gat_bwd(torch::Tensor indptr, torch::Tensor col, c10::optional<torch::Tensor> order,
                                   torch::Tensor cindptr, torch::Tensor crow, c10::optional<torch::Tensor> corder,
                                   torch::Tensor h, torch::Tensor al, torch::Tensor ar, int64_t H, int64_t C,
                                   double slope, torch::Tensor out, torch::Tensor dout, torch::Tensor lse,
                                   c10::optional<torch::Tensor> a_src) {
  gat_common(indptr, col, h, al, ar, H, C);
  typed(cindptr, torch::kInt64, "cindptr");
  typed(crow, torch::kInt32, "crow");
  TORCH_CHECK(cindptr.numel() == h.size(0) + 1, "cindptr must have N+1 entries");
  TORCH_CHECK(crow.numel() == col.numel(), "CSC and CSR must hold the same edges");
  const int64_t S = indptr.numel() - 1, N = h.size(0);
  TORCH_CHECK(out.sizes() == dout.sizes() && out.size(0) == S && out.size(1) == H * C, "out/dout must be [S, H*C]");
  typed(out, h.scalar_type(), "out");
  typed(dout, h.scalar_type(), "dout");
  typed(lse, torch::kFloat32, "lse");
  TORCH_CHECK(lse.numel() == S * H, "lse must be [S, H]");
  const c10::DeviceGuard g(h.device());
  auto dh = torch::empty_like(h);
  auto dal = torch::empty_like(al);
  auto dar = torch::empty_like(ar);
  auto stat = torch::empty({S, H, 4}, al.options());
  ok(eh_gat_bwd(indptr.data_ptr<int64_t>(), col.data_ptr<int32_t>(), order_ptr(order, S, "order"), S,
                cindptr.data_ptr<int64_t>(), crow.data_ptr<int32_t>(), order_ptr(corder, N, "corder"), N,
                h.data_ptr(), h.scalar_type() == torch::kBFloat16, al.data_ptr<float>(), ar.data_ptr<float>(),
                static_cast<int>(H), static_cast<int>(C), static_cast<float>(slope), out.data_ptr(), dout.data_ptr(),
                lse.data_ptr<float>(), stat.data_ptr<float>(), dh.data_ptr(), dal.data_ptr<float>(),
                dar.data_ptr<float>(), asrc_ptr(a_src, H, C), stream()),
     "gat_bwd");
  return {dh, dal, dar};
}

void att_check(const torch::Tensor& z, const torch::Tensor& a_src, const torch::Tensor& a_dst, int64_t H,
               int64_t C) {
  bf16_or_f32(z, "z");
  typed(a_src, torch::kFloat32, "a_src");
  typed(a_dst, torch::kFloat32, "a_dst");
  TORCH_CHECK(z.dim() == 2 && z.size(1) == H * C, "z must be [N, H*C]");
  TORCH_CHECK(a_src.numel() == H * C && a_dst.numel() == H * C, "attention vectors must be [H, C]");
  TORCH_CHECK(gat_supported(H, C, z.scalar_type() == torch::kBFloat16), "unsupported GAT shape");
}

std::vector<torch::Tensor> gat_att_fwd(torch::Tensor z, torch::Tensor a_src, torch::Tensor a_dst, int64_t H,
                                       int64_t C) {
  att_check(z, a_src, a_dst, H, C);
  const c10::DeviceGuard g(z.device());
  auto fopt = z.options().dtype(torch::kFloat32);
  auto al = torch::empty({z.size(0), H}, fopt);
  auto ar = torch::empty({z.size(0), H}, fopt);
  ok(eh_gat_att_fwd(z.data_ptr(), z.scalar_type() == torch::kBFloat16, z.size(0), static_cast<int>(H),
                    static_cast<int>(C), a_src.data_ptr<float>(), a_dst.data_ptr<float>(), al.data_ptr<float>(),
                    ar.data_ptr<float>(), stream()),
     "gat_att_fwd");
  return {al, ar};
}

// dz is updated in place; returns (da_src, da_dst)
std::vector<torch::Tensor> gat_att_bwd_(torch::Tensor z, torch::Tensor a_src, torch::Tensor a_dst, int64_t H,
                                        int64_t C, torch::Tensor dal, torch::Tensor dar, torch::Tensor dz) {
  att_check(z, a_src, a_dst, H, C);
  typed(dal, torch::kFloat32, "dal");
  typed(dar, torch::kFloat32, "dar");
  typed(dz, z.scalar_type(), "dz");
  TORCH_CHECK(dz.sizes() == z.sizes() && dal.numel() == z.size(0) * H && dar.numel() == z.size(0) * H,
              "gat_att_bwd shape mismatch");
  const c10::DeviceGuard g(z.device());
  const bool bf = z.scalar_type() == torch::kBFloat16;
  const int64_t nb = eh_gat_att_bwd_blocks(z.size(0), static_cast<int>(H), static_cast<int>(C), bf);
  auto ps = torch::zeros({nb, H, C}, a_src.options());
  auto pd = torch::zeros({nb, H, C}, a_dst.options());
  ok(eh_gat_att_bwd(z.data_ptr(), bf, z.size(0), static_cast<int>(H), static_cast<int>(C), a_src.data_ptr<float>(),
                    a_dst.data_ptr<float>(), dal.data_ptr<float>(), dar.data_ptr<float>(), dz.data_ptr(),
                    ps.data_ptr<float>(), pd.data_ptr<float>(), stream()),
     "gat_att_bwd");
  return {ps.sum(0), pd.sum(0)};
}

// ----------------------------------------------------------------------------- R-GCN
void tiles_check(const torch::Tensor& trel, const torch::Tensor& tstart, const torch::Tensor& tlen) {
  typed(trel, torch::kInt32, "tile_rel");
  typed(tstart, torch::kInt32, "tile_start");
  typed(tlen, torch::kInt32, "tile_len");
  TORCH_CHECK(trel.numel() == tstart.numel() && trel.numel() == tlen.numel(), "tile arrays must match");
}

void rel_gemm(torch::Tensor A, torch::Tensor a_idx, torch::Tensor trel, torch::Tensor tstart, torch::Tensor tlen,
              torch::Tensor B, c10::optional<torch::Tensor> scale, torch::Tensor o_idx, int64_t mode, int64_t tm, torch::Tensor Y) {
  typed(A, torch::kBFloat16, "A");
  typed(B, torch::kBFloat16, "B");
  typed(a_idx, torch::kInt32, "a_idx");
  typed(o_idx, torch::kInt32, "o_idx");
  tiles_check(trel, tstart, tlen);
  TORCH_CHECK(A.dim() == 2 && B.dim() == 3 && B.size(2) == A.size(1), "A [*, K], B [R, N, K]");
  const int64_t K = A.size(1), N = B.size(1);
  TORCH_CHECK(K % 32 == 0 && K <= 1024 && N % 16 == 0, "rel_gemm needs K % 32 == 0, K <= 1024, N % 16 == 0");
  TORCH_CHECK(eh_rel_gemm_lds(static_cast<int>(K), static_cast<int>(N), static_cast<int>(mode), static_cast<int>(tm)) <= 160 * 1024 - 2048,
              "rel_gemm: K + N too large for the LDS tiles");
  TORCH_CHECK(a_idx.numel() == o_idx.numel(), "a_idx / o_idx must cover the same edges");
  TORCH_CHECK(tm % 16 == 0 && tm >= 16 && tm <= eh_rel_gemm_tile(), "rel_gemm: tile rows tm must be a multiple of 16 in [16, rel_gemm_tile]");
  if (scale.has_value()) {
    typed(*scale, torch::kFloat32, "scale");
    TORCH_CHECK(scale->numel() == a_idx.numel(), "scale must be per edge");
  }
  TORCH_CHECK(mode == 0 || mode == 1, "mode: 0 store bf16, 1 atomic-add fp32");
  typed(Y, mode == 0 ? torch::kBFloat16 : torch::kFloat32, "Y");
  TORCH_CHECK(Y.dim() == 2 && Y.size(1) == N, "Y must be [rows, N]");
  const c10::DeviceGuard g(A.device());
  ok(eh_rel_gemm(A.data_ptr(), static_cast<int>(K), a_idx.data_ptr<int32_t>(), trel.data_ptr<int32_t>(),
                 tstart.data_ptr<int32_t>(), tlen.data_ptr<int32_t>(), static_cast<int>(trel.numel()), B.data_ptr(),
                 static_cast<int>(N), scale.has_value() ? scale->data_ptr<float>() : nullptr,
                 o_idx.data_ptr<int32_t>(), static_cast<int>(mode), static_cast<int>(tm), Y.data_ptr(), stream()),
     "rel_gemm");
}

std::vector<torch::Tensor> rel_weight_bf16(torch::Tensor W) {
  typed(W, torch::kFloat32, "W");
  TORCH_CHECK(W.dim() == 3 && W.is_contiguous(), "W must be a contiguous [R, N, K] tensor");
  const int64_t R = W.size(0), N = W.size(1), K = W.size(2);
  TORCH_CHECK(N % 64 == 0 && K % 64 == 0, "rel_weight_bf16 needs N, K multiples of 64");
  auto opt = W.options().dtype(torch::kBFloat16);
  torch::Tensor wb = torch::empty({R, N, K}, opt), wt = torch::empty({R, K, N}, opt);
  const c10::DeviceGuard g(W.device());
  ok(eh_rel_weight_bf16(W.data_ptr<float>(), R, static_cast<int>(N), static_cast<int>(K), wb.data_ptr(), wt.data_ptr(),
                        stream()),
     "rel_weight_bf16");
  return {wb, wt};
}

void rel_gemm_dw(torch::Tensor G, torch::Tensor g_idx, torch::Tensor X, torch::Tensor x_idx,
                 c10::optional<torch::Tensor> scale, torch::Tensor trel, torch::Tensor tstart, torch::Tensor tlen,
                 c10::optional<torch::Tensor> solo, torch::Tensor dW, bool accumulate,
                 c10::optional<torch::Tensor> slot, c10::optional<torch::Tensor> part,
                 c10::optional<torch::Tensor> mrel, c10::optional<torch::Tensor> mrp) {
  typed(G, torch::kBFloat16, "G");
  typed(X, torch::kBFloat16, "X");
  typed(g_idx, torch::kInt32, "g_idx");
  typed(x_idx, torch::kInt32, "x_idx");
  typed(dW, torch::kFloat32, "dW");
  tiles_check(trel, tstart, tlen);
  TORCH_CHECK(G.dim() == 2 && X.dim() == 2 && dW.dim() == 3, "G [*, N], X [*, K], dW [R, N, K]");
  const int64_t N = G.size(1), K = X.size(1);
  TORCH_CHECK(dW.size(1) == N && dW.size(2) == K, "dW must be [R, N, K]");
  TORCH_CHECK(N % 64 == 0 && K % 64 == 0, "rel_gemm_dw needs N, K multiples of 64");
  TORCH_CHECK(g_idx.numel() == x_idx.numel(), "g_idx / x_idx must cover the same edges");
  if (scale.has_value()) {
    typed(*scale, torch::kFloat32, "scale");
    TORCH_CHECK(scale->numel() == g_idx.numel(), "scale must be per edge");
  }
  if (solo.has_value()) {
    typed(*solo, torch::kInt32, "solo");
    TORCH_CHECK(solo->numel() == trel.numel(), "solo must hold one flag per chunk");
  }
  // deterministic mode: chunk -> partial slot (-1 for solo chunks), the slot buffer, and
  // the multi-chunk relations with their slot ranges (mrp: CSR over mrel)
  const int32_t *sl = nullptr, *mr = nullptr, *mp = nullptr;
  float* pp = nullptr;
  int nmulti = 0;
  if (slot.has_value()) {
    TORCH_CHECK(solo.has_value() && part.has_value() && mrel.has_value() && mrp.has_value(),
                "deterministic rel_gemm_dw needs solo, slot, part, mrel and mrp");
    typed(*slot, torch::kInt32, "slot");
    typed(*mrel, torch::kInt32, "mrel");
    typed(*mrp, torch::kInt32, "mrp");
    typed(*part, torch::kFloat32, "part");
    TORCH_CHECK(slot->numel() == trel.numel() && mrp->numel() == mrel->numel() + 1, "slot / mrp sizes");
    TORCH_CHECK(part->dim() == 3 && part->size(1) == N && part->size(2) == K, "part must be [slots, N, K]");
    sl = slot->data_ptr<int32_t>();
    mr = mrel->data_ptr<int32_t>();
    mp = mrp->data_ptr<int32_t>();
    pp = part->data_ptr<float>();
    nmulti = static_cast<int>(mrel->numel());
  }
  const c10::DeviceGuard g(G.device());
  ok(eh_rel_gemm_dw(G.data_ptr(), static_cast<int>(N), g_idx.data_ptr<int32_t>(), X.data_ptr(), static_cast<int>(K),
                    x_idx.data_ptr<int32_t>(), scale.has_value() ? scale->data_ptr<float>() : nullptr,
                    trel.data_ptr<int32_t>(), tstart.data_ptr<int32_t>(), tlen.data_ptr<int32_t>(),
                    solo.has_value() ? solo->data_ptr<int32_t>() : nullptr, static_cast<int>(trel.numel()),
                    dW.data_ptr<float>(), accumulate ? 1 : 0, stream(), sl, pp, mr, mp, nmulti),
     "rel_gemm_dw");
}

// ----------------------------------------------------------------------------- skip-gram loss
void sgns_check(const torch::Tensor& emb, const torch::Tensor& pos, const torch::Tensor& neg) {
  const bool bf = bf16_or_f32(emb, "emb");
  typed(pos, emb.scalar_type(), "pos");
  typed(neg, emb.scalar_type(), "neg");
  TORCH_CHECK(emb.dim() == 2 && pos.dim() == 3 && neg.dim() == 3, "emb [B, D], pos [B, P, D], neg [B, K, D]");
  const int64_t B = emb.size(0), D = emb.size(1);
  TORCH_CHECK(pos.size(0) == B && neg.size(0) == B && pos.size(2) == D && neg.size(2) == D, "sgns shape mismatch");
  const int V = bf ? 8 : 4;
  TORCH_CHECK(D % V == 0 && D / V <= 64, "sgns needs D % ", V, " == 0 and D <= ", 64 * V);
}

std::vector<torch::Tensor> sgns_fwd(torch::Tensor emb, torch::Tensor pos, torch::Tensor neg) {
  sgns_check(emb, pos, neg);
  const c10::DeviceGuard g(emb.device());
  const int64_t B = emb.size(0), P = pos.size(1), K = neg.size(1);
  auto fopt = emb.options().dtype(torch::kFloat32);
  auto logits = torch::empty({B, P + K}, fopt);
  auto loss_rows = torch::empty({B}, fopt);
  ok(eh_sgns_fwd(emb.data_ptr(), pos.data_ptr(), neg.data_ptr(), emb.scalar_type() == torch::kBFloat16, B,
                 static_cast<int>(P), static_cast<int>(K), static_cast<int>(emb.size(1)), logits.data_ptr<float>(),
                 loss_rows.data_ptr<float>(), stream()),
     "sgns_fwd");
  return {logits, loss_rows};
}

std::vector<torch::Tensor> sgns_bwd(torch::Tensor emb, torch::Tensor pos, torch::Tensor neg, torch::Tensor logits,
                                    double gscale) {
  sgns_check(emb, pos, neg);
  typed(logits, torch::kFloat32, "logits");
  const int64_t B = emb.size(0), P = pos.size(1), K = neg.size(1);
  TORCH_CHECK(logits.numel() == B * (P + K), "logits must be [B, P+K]");
  const c10::DeviceGuard g(emb.device());
  auto demb = torch::empty_like(emb);
  auto dpos = torch::empty_like(pos);
  auto dneg = torch::empty_like(neg);
  ok(eh_sgns_bwd(emb.data_ptr(), pos.data_ptr(), neg.data_ptr(), emb.scalar_type() == torch::kBFloat16, B,
                 static_cast<int>(P), static_cast<int>(K), static_cast<int>(emb.size(1)), logits.data_ptr<float>(),
                 static_cast<float>(gscale), demb.data_ptr(), dpos.data_ptr(), dneg.data_ptr(), stream()),
     "sgns_bwd");
  return {demb, dpos, dneg};
}

// ----------------------------------------------------------------------------- index-driven SGNS
const int64_t* map_ptr(const c10::optional<torch::Tensor>& map, int64_t& n, const char* name) {
  n = 0;
  if (!map.has_value()) return nullptr;
  typed(*map, torch::kInt64, name);
  n = map->numel();
  return map->data_ptr<int64_t>();
}

// T / C fp32 row tables; tinv [P], cinv [P*(1+K)] (positives then negatives) index the
// unique ids, tmap / cmap map those to table rows (absent: the ids are rows)
std::vector<torch::Tensor> sgns_fwd_idx(torch::Tensor T, c10::optional<torch::Tensor> tmap, torch::Tensor tinv,
                                        torch::Tensor C, c10::optional<torch::Tensor> cmap, torch::Tensor cinv,
                                        int64_t K, double gscale) {
  const bool bf = T.scalar_type() == torch::kBFloat16;
  typed(T, bf ? torch::kBFloat16 : torch::kFloat32, "T");
  typed(C, bf ? torch::kBFloat16 : torch::kFloat32, "C");
  typed(tinv, torch::kInt64, "tinv");
  typed(cinv, torch::kInt64, "cinv");
  TORCH_CHECK(T.dim() == 2 && C.dim() == 2 && T.size(1) == C.size(1), "T [*, D], C [*, D]");
  const int64_t P = tinv.numel(), D = T.size(1);
  TORCH_CHECK(K >= 0 && cinv.numel() == P * (1 + K), "cinv must hold P*(1+K) entries");
  TORCH_CHECK(D % 4 == 0 && D <= 256, "sgns_fwd_idx needs D % 4 == 0 and D <= 256");
  int64_t nTm, nCm;
  const int64_t* tm = map_ptr(tmap, nTm, "tmap");
  const int64_t* cm = map_ptr(cmap, nCm, "cmap");
  const c10::DeviceGuard g(T.device());
  auto fopt = T.options().dtype(torch::kFloat32);
  auto coef = torch::empty({P, 1 + K}, fopt);
  auto loss_rows = torch::empty({P}, fopt);
  ok(eh_sgns_fwd_idx(T.data_ptr(), tm, nTm, tinv.data_ptr<int64_t>(), T.size(0), C.data_ptr(), cm, nCm,
                     cinv.data_ptr<int64_t>(), C.size(0), P, static_cast<int>(K), static_cast<int>(D),
                     static_cast<float>(gscale), coef.data_ptr<float>(), loss_rows.data_ptr<float>(), bf ? 1 : 0,
                     stream()),
     "sgns_fwd_idx");
  return {coef, loss_rows};
}

// rows idx [n] (int64; < 0: zero row) of an fp32 table, packed as bf16 [n, D]
torch::Tensor gather_f32_bf16(torch::Tensor x, torch::Tensor idx, c10::optional<torch::Tensor> out) {
  typed(x, torch::kFloat32, "x");
  typed(idx, torch::kInt64, "idx");
  TORCH_CHECK(x.dim() == 2 && x.size(1) % 4 == 0, "x [rows, D], D % 4 == 0");
  const int64_t n = idx.numel(), D = x.size(1);
  torch::Tensor o;
  if (out.has_value()) {
    typed(*out, torch::kBFloat16, "out");
    TORCH_CHECK(out->dim() == 2 && out->size(0) == n && out->size(1) == D, "out must be [n, D]");
    o = *out;
  } else {
    o = torch::empty({n, D}, x.options().dtype(torch::kBFloat16));
  }
  const c10::DeviceGuard g(x.device());
  ok(eh_gather_f32_bf16(x.data_ptr<float>(), x.size(0), static_cast<int>(D), idx.data_ptr<int64_t>(), n, o.data_ptr(),
                        stream()),
     "gather_f32_bf16");
  return o;
}

// unsupervised pair objective: es [B, E] sources, ec [B + B K, E] contexts (B positives,
// then the B x K negatives source-major) -> (logits [B, 1 + K], loss [] = mean sigmoid CE);
// the batch's summed reciprocal ranks of the positives are added to mrr[0] when given
std::vector<torch::Tensor> pair_fwd(torch::Tensor es, torch::Tensor ec, int64_t B, int64_t K,
                                    c10::optional<torch::Tensor> mrr) {
  typed(es, torch::kFloat32, "es");
  typed(ec, torch::kFloat32, "ec");
  TORCH_CHECK(es.dim() == 2 && ec.dim() == 2 && es.size(0) == B && ec.size(0) == B * (1 + K) &&
                  es.size(1) == ec.size(1) && es.is_contiguous() && ec.is_contiguous(),
              "pair_fwd: es [B, E], ec [B (1 + K), E], contiguous");
  const int64_t E = es.size(1);
  TORCH_CHECK(E % 4 == 0 && E <= 256 && K >= 0 && K <= 15, "pair_fwd: E % 4 == 0, E <= 256, K <= 15");
  float* mp = nullptr;
  if (mrr.has_value()) {
    typed(*mrr, torch::kFloat32, "mrr");
    TORCH_CHECK(mrr->numel() == 1, "mrr must hold one value");
    mp = mrr->data_ptr<float>();
  }
  const c10::DeviceGuard g(es.device());
  auto logits = torch::empty({B, 1 + K}, es.options());
  auto part = torch::empty({2 * B}, es.options());
  auto loss = torch::empty({}, es.options());
  ok(eh_pair_fwd(es.data_ptr<float>(), ec.data_ptr<float>(), static_cast<int>(B), static_cast<int>(K),
                 static_cast<int>(E), 1.f / static_cast<float>(B * (1 + K)), logits.data_ptr<float>(),
                 part.data_ptr<float>(), loss.data_ptr<float>(), mp, stream()),
     "pair_fwd");
  return {logits, loss};
}

void pair_bwd(torch::Tensor es, torch::Tensor ec, int64_t B, int64_t K, torch::Tensor logits, torch::Tensor dloss,
              torch::Tensor des, torch::Tensor dec) {
  typed(logits, torch::kFloat32, "logits");
  typed(dloss, torch::kFloat32, "dloss");
  typed(des, torch::kFloat32, "des");
  typed(dec, torch::kFloat32, "dec");
  TORCH_CHECK(logits.numel() == B * (1 + K) && dloss.numel() == 1 && des.sizes() == es.sizes() &&
                  dec.sizes() == ec.sizes() && des.is_contiguous() && dec.is_contiguous() && es.is_contiguous() &&
                  ec.is_contiguous(),
              "pair_bwd shapes");
  const c10::DeviceGuard g(es.device());
  ok(eh_pair_bwd(es.data_ptr<float>(), ec.data_ptr<float>(), static_cast<int>(B), static_cast<int>(K),
                 static_cast<int>(es.size(1)), 1.f / static_cast<float>(B * (1 + K)), logits.data_ptr<float>(),
                 dloss.data_ptr<float>(), des.data_ptr<float>(), dec.data_ptr<float>(), stream()),
     "pair_bwd");
}

// occurrence lists of inv (values in [0, n_u)): ptr [n_u + 1] int64, list [n] int32
std::vector<torch::Tensor> occ_csr(torch::Tensor inv, int64_t n_u) {
  typed(inv, torch::kInt64, "inv");
  TORCH_CHECK(inv.numel() < (int64_t{1} << 31), "occ_csr: too many occurrences");
  const c10::DeviceGuard g(inv.device());
  TORCH_CHECK(n_u < (int64_t{1} << 31), "occ_csr: too many unique ids");
  auto iopt = inv.options();
  auto list = torch::empty({inv.numel()}, iopt.dtype(torch::kInt32));
  if (n_u <= 0) return {torch::zeros({1}, iopt), list};
  // one zero fill for the counts and the fill cursors; counts by atomics (bincount would
  // read max(inv) back to the host: a sync that also breaks hipGraph capture), then one
  // device scan straight into ptr[1:]; inv values must lie in [0, n_u)
  auto ptr = torch::empty({n_u + 1}, iopt);
  auto cc = torch::zeros({2 * n_u}, iopt.dtype(torch::kInt32));
  size_t bytes = 0;
  ok(eh_occ_count_scan(nullptr, 0, n_u, cc.data_ptr<int32_t>(), ptr.data_ptr<int64_t>(), nullptr, &bytes, stream()),
     "occ_count_scan(size)");
  auto temp = torch::empty({static_cast<int64_t>(bytes) + 1}, iopt.dtype(torch::kUInt8));
  ok(eh_occ_count_scan(inv.data_ptr<int64_t>(), inv.numel(), n_u, cc.data_ptr<int32_t>(), ptr.data_ptr<int64_t>(),
                       temp.data_ptr(), &bytes, stream()),
     "occ_count_scan");
  auto cursor = cc.narrow(0, n_u, n_u);
  ok(eh_occ_fill(inv.data_ptr<int64_t>(), inv.numel(), ptr.data_ptr<int64_t>(), cursor.data_ptr<int32_t>(),
                 list.data_ptr<int32_t>(), stream()),
     "occ_fill");
  return {ptr, list};
}

// deterministic occurrence CSR of `keys` over S segments (keys < 0 skipped): (ptr [S + 1]
// int64, perm [n] int32: each segment's occurrence ids ascending) — det_segment_sum's
// inputs for a fixed-order per-row sum
std::vector<torch::Tensor> det_occ(torch::Tensor keys, int64_t S) {
  typed(keys, torch::kInt64, "keys");
  TORCH_CHECK(S > 0 && S < (int64_t{1} << 30) && keys.numel() < (int64_t{1} << 31), "det_occ: sizes");
  const c10::DeviceGuard g(keys.device());
  auto o = keys.options();
  const int64_t n = keys.numel();
  auto ptr = torch::empty({S + 1}, o);
  auto perm = torch::empty({n}, o.dtype(torch::kInt32));
  auto cnt = torch::zeros({S}, o.dtype(torch::kInt32));
  auto work = torch::empty({3 * n + 1}, o.dtype(torch::kInt32));
  size_t bytes = 0;
  ok(eh_det_occ(keys.data_ptr<int64_t>(), n, S, cnt.data_ptr<int32_t>(), ptr.data_ptr<int64_t>(),
                work.data_ptr<int32_t>(), perm.data_ptr<int32_t>(), nullptr, &bytes, stream()),
     "det_occ(size)");
  auto temp = torch::empty({static_cast<int64_t>(bytes) + 1}, o.dtype(torch::kUInt8));
  ok(eh_det_occ(keys.data_ptr<int64_t>(), n, S, cnt.data_ptr<int32_t>(), ptr.data_ptr<int64_t>(),
                work.data_ptr<int32_t>(), perm.data_ptr<int32_t>(), temp.data_ptr(), &bytes, stream()),
     "det_occ");
  return {ptr, perm};
}

// out [S, D] = per-segment sums of src rows over (ptr, perm) in a fixed order (det_occ's
// CSR): deterministic, hot segments spread over a whole block
void det_segment_sum(torch::Tensor src, torch::Tensor ptr, torch::Tensor perm, torch::Tensor out) {
  typed(src, torch::kFloat32, "src");
  typed(out, torch::kFloat32, "out");
  typed(ptr, torch::kInt64, "ptr");
  typed(perm, torch::kInt32, "perm");
  const int64_t S = ptr.numel() - 1, D = src.size(1);
  TORCH_CHECK(src.dim() == 2 && out.dim() == 2 && out.size(0) == S && out.size(1) == D, "det_segment_sum: shapes");
  TORCH_CHECK(src.is_contiguous() && out.is_contiguous(), "det_segment_sum: contiguous tensors");
  const c10::DeviceGuard g(src.device());
  ok(eh_det_segsum(src.data_ptr<float>(), static_cast<int>(D), ptr.data_ptr<int64_t>(), perm.data_ptr<int32_t>(), S,
                   out.data_ptr<float>(), stream()),
     "det_segment_sum");
}

struct UpdIn {
  int64_t n_u, P, n_smap;
  const int64_t* smap;
};

UpdIn upd_check(int64_t side, const torch::Tensor& ptr, const torch::Tensor& list, const torch::Tensor& coef, int64_t K,
                const torch::Tensor& src, const c10::optional<torch::Tensor>& smap, const torch::Tensor& sinv) {
  TORCH_CHECK(side == 0 || side == 1, "side: 0 target, 1 context");
  typed(ptr, torch::kInt64, "ptr");
  typed(list, torch::kInt32, "list");
  typed(coef, torch::kFloat32, "coef");
  typed(src, src.scalar_type() == torch::kBFloat16 ? torch::kBFloat16 : torch::kFloat32, "src");
  typed(sinv, torch::kInt64, "sinv");
  TORCH_CHECK(coef.dim() == 2 && coef.size(1) == K + 1 && K >= (side == 1 ? 1 : 0), "coef must be [P, 1+K]");
  TORCH_CHECK(src.dim() == 2 && src.size(1) % 4 == 0 && src.size(1) <= 256, "src [*, D], D % 4 == 0, D <= 256");
  const int64_t P = coef.size(0);
  TORCH_CHECK(sinv.numel() == (side == 0 ? P * (1 + K) : P), "sinv: context occurrences (side 0) or targets (side 1)");
  TORCH_CHECK(list.numel() == (side == 0 ? P : P * (1 + K)), "list must cover every occurrence of this side");
  UpdIn r;
  r.n_u = ptr.numel() - 1;
  r.P = P;
  r.smap = map_ptr(smap, r.n_smap, "smap");
  return r;
}

// per-unique-row gradients of one side; rows with no occurrence on this side are written
// only when the buffer is allocated here (zeros) — with ``out`` they are left untouched
torch::Tensor sgns_grad(int64_t side, torch::Tensor ptr, torch::Tensor list, torch::Tensor coef, int64_t K,
                        torch::Tensor src, c10::optional<torch::Tensor> smap, torch::Tensor sinv,
                        c10::optional<torch::Tensor> out) {
  const UpdIn u = upd_check(side, ptr, list, coef, K, src, smap, sinv);
  const c10::DeviceGuard g(src.device());
  const int64_t D = src.size(1);
  torch::Tensor gout;
  if (out.has_value()) {
    typed(*out, out->scalar_type() == torch::kBFloat16 ? torch::kBFloat16 : torch::kFloat32, "out");
    TORCH_CHECK(out->dim() == 2 && out->size(0) == u.n_u && out->size(1) == D, "out must be [n_u, D]");
    gout = *out;
  } else {
    gout = torch::zeros({u.n_u, D}, src.options().dtype(torch::kFloat32));
  }
  const int sbf = src.scalar_type() == torch::kBFloat16, gbf = gout.scalar_type() == torch::kBFloat16;
  ok(eh_sgns_update(static_cast<int>(side), u.n_u, ptr.data_ptr<int64_t>(), list.data_ptr<int32_t>(),
                    coef.data_ptr<float>(), u.P, static_cast<int>(K), static_cast<int>(D), src.data_ptr(), sbf,
                    src.size(0), u.smap, u.n_smap, sinv.data_ptr<int64_t>(), gout.data_ptr(), gbf, nullptr, nullptr,
                    nullptr, nullptr, 0, nullptr, 0, 0.f, 0.f, 0.f, 0.f, 2, stream()),
     "sgns_grad");
  return gout;
}

void sgns_apply_(int64_t side, torch::Tensor ptr, torch::Tensor list, torch::Tensor coef, int64_t K, torch::Tensor src,
                 c10::optional<torch::Tensor> smap, torch::Tensor sinv, torch::Tensor table, torch::Tensor m,
                 torch::Tensor v, c10::optional<torch::Tensor> rows, torch::Tensor step, bool inc_step, double lr,
                 double b1, double b2, double eps, int64_t kind) {
  const UpdIn u = upd_check(side, ptr, list, coef, K, src, smap, sinv);
  typed(table, torch::kFloat32, "table");
  typed(m, torch::kFloat32, "m");
  typed(v, torch::kFloat32, "v");
  typed(step, torch::kInt64, "step");
  TORCH_CHECK(kind >= 0 && kind <= 2, "kind: 0 adam, 1 adagrad, 2 sgd");
  TORCH_CHECK(table.dim() == 2 && table.size(1) == src.size(1) && m.sizes() == table.sizes() &&
                  v.sizes() == table.sizes(),
              "table / m / v must be [rows, D]");
  int64_t n_rows_map = 0;
  const int64_t* rp = map_ptr(rows, n_rows_map, "rows");
  TORCH_CHECK(!rp || n_rows_map == u.n_u, "rows must hold one table row per unique id");
  TORCH_CHECK(rp || u.n_u <= table.size(0), "without rows, unique ids are table rows");
  const c10::DeviceGuard g(src.device());
  ok(eh_sgns_update(static_cast<int>(side), u.n_u, ptr.data_ptr<int64_t>(), list.data_ptr<int32_t>(),
                    coef.data_ptr<float>(), u.P, static_cast<int>(K), static_cast<int>(src.size(1)),
                    src.data_ptr(), src.scalar_type() == torch::kBFloat16 ? 1 : 0, src.size(0), u.smap, u.n_smap,
                    sinv.data_ptr<int64_t>(), nullptr, 0, table.data_ptr<float>(), m.data_ptr<float>(), v.data_ptr<float>(), rp, table.size(0),
                    step.data_ptr<int64_t>(), inc_step ? 1 : 0, static_cast<float>(lr), static_cast<float>(b1),
                    static_cast<float>(b2),
                    static_cast<float>(eps), static_cast<int>(kind), stream()),
     "sgns_apply");
}

// ----------------------------------------------------------------------------- KG scores
struct KgIn {
  int64_t B, K, D, nneg;
};

KgIn kg_check(const torch::Tensor& ent, const torch::Tensor& rel, const torch::Tensor& src, const torch::Tensor& dst,
              const torch::Tensor& ridx, const torch::Tensor& neg, int64_t kind, int64_t corrupt) {
  typed(ent, torch::kFloat32, "ent");
  typed(rel, torch::kFloat32, "rel");
  for (const auto* t : {&src, &dst, &ridx, &neg}) typed(*t, torch::kInt64, "kg index");
  TORCH_CHECK(ent.dim() == 2 && rel.dim() == 2 && ent.size(1) == rel.size(1), "ent [Ne, D], rel [Nr, D]");
  const int64_t B = src.numel(), D = ent.size(1);
  TORCH_CHECK(dst.numel() == B && ridx.numel() == B, "src/dst/rel index must have B entries");
  TORCH_CHECK(B == 0 || neg.numel() % B == 0, "neg must be [B, K]");
  TORCH_CHECK(D % 4 == 0 && D <= 256, "kg kernels need D % 4 == 0 and D <= 256");
  TORCH_CHECK(kind >= 0 && kind <= 2 && corrupt >= 0 && corrupt <= 2, "bad kind / corrupt");
  const int64_t K = B ? neg.numel() / B : 0;
  return KgIn{B, K, D, corrupt == 2 ? 2 * K : K};
}

std::vector<torch::Tensor> kg_fwd(torch::Tensor ent, torch::Tensor rel, torch::Tensor src, torch::Tensor dst,
                                  torch::Tensor ridx, torch::Tensor neg, int64_t kind, int64_t corrupt,
                                  bool normalize) {
  const KgIn k = kg_check(ent, rel, src, dst, ridx, neg, kind, corrupt);
  const c10::DeviceGuard g(ent.device());
  auto pos_s = torch::empty({k.B}, ent.options());
  auto neg_s = torch::empty({k.B, k.nneg}, ent.options());
  ok(eh_kg_fwd(ent.data_ptr<float>(), rel.data_ptr<float>(), src.data_ptr<int64_t>(), dst.data_ptr<int64_t>(),
               ridx.data_ptr<int64_t>(), neg.data_ptr<int64_t>(), k.B, static_cast<int>(k.K), static_cast<int>(k.D),
               static_cast<int>(kind), static_cast<int>(corrupt), normalize ? 1 : 0, pos_s.data_ptr<float>(),
               neg_s.data_ptr<float>(), stream()),
     "kg_fwd");
  return {pos_s, neg_s};
}

// fused TransE margin step (embed.hip K10b): draws B triples from `pool` and K corruptions
// per triple with Philox(seed, step[0], row), scores them on h (the encoder output) and rel,
// writes the mean margin loss to loss[0] and adds its gradients into dent ([N, D], zeroed
// by the caller) and drel ([R, D]); the drawn ids land in o_src / o_dst / o_ridx / o_neg.
// Ids are not range-checked here: the caller validates the triple tables once.
void kg_step(torch::Tensor h, torch::Tensor rel, torch::Tensor pool, torch::Tensor t_src, torch::Tensor t_dst,
             torch::Tensor t_rel, torch::Tensor step, int64_t seed, int64_t kind, bool normalize, double margin,
             torch::Tensor o_src, torch::Tensor o_dst, torch::Tensor o_ridx, torch::Tensor o_neg, torch::Tensor coef,
             torch::Tensor part, torch::Tensor loss, torch::Tensor dent, torch::Tensor drel,
             c10::optional<torch::Tensor> drel_rep, c10::optional<torch::Tensor> occ_e,
             c10::optional<torch::Tensor> occ_r, c10::optional<torch::Tensor> key_e,
             c10::optional<torch::Tensor> key_r) {
  for (auto* t : {&h, &rel, &coef, &part, &loss, &dent, &drel}) typed(*t, torch::kFloat32, "kg_step float buffer");
  for (auto* t : {&pool, &t_src, &t_dst, &t_rel, &step, &o_src, &o_dst, &o_ridx, &o_neg})
    typed(*t, torch::kInt64, "kg_step id buffer");
  TORCH_CHECK(h.dim() == 2 && rel.dim() == 2 && h.size(1) == rel.size(1), "kg_step: h [N, D], rel [R, D]");
  TORCH_CHECK(dent.sizes() == h.sizes() && drel.sizes() == rel.sizes(), "kg_step: grads must match h / rel");
  TORCH_CHECK(t_src.numel() == t_dst.numel() && t_src.numel() == t_rel.numel(), "kg_step: triple tables differ");
  const int64_t B = o_src.numel();
  TORCH_CHECK(B > 0 && o_dst.numel() == B && o_ridx.numel() == B && coef.numel() == B && o_neg.numel() % B == 0,
              "kg_step: per-triple buffers must have B rows");
  const int64_t K = o_neg.numel() / B, D = h.size(1);
  TORCH_CHECK(K >= 1 && K <= 255 && D % 4 == 0 && D <= 256, "kg_step: 1 <= K <= 255, D % 4 == 0, D <= 256");
  int nparts = 0;
  ok(eh_kg_step(nullptr, nullptr, nullptr, 1, nullptr, nullptr, nullptr, 1, nullptr, 0, B, static_cast<int>(K),
                static_cast<int>(D), static_cast<int>(kind), 0, 0.f, nullptr, nullptr, nullptr, nullptr, nullptr,
                nullptr, nullptr, nullptr, nullptr, &nparts, nullptr, 0, 0, stream()),
     "kg_step (grid)");
  float* rep_p = nullptr;
  int rep = 0;
  if (drel_rep.has_value()) {  // [rep, R, D] relation-gradient replicas
    typed(*drel_rep, torch::kFloat32, "drel_rep");
    TORCH_CHECK(drel_rep->dim() == 3 && drel_rep->size(1) == rel.size(0) && drel_rep->size(2) == rel.size(1),
                "kg_step: drel_rep [rep, R, D]");
    rep_p = drel_rep->data_ptr<float>();
    rep = static_cast<int>(drel_rep->size(0));
  }
  // deterministic mode: per-occurrence gradient rows instead of atomics (the caller sums
  // them per entity / relation in a fixed order): occ_e [B * (2 + K), D], occ_r [B, D]
  // and the row keys of those occurrences (-1: a triple without gradient, rows not written)
  float *oe = nullptr, *orr = nullptr;
  int64_t *ke = nullptr, *kr = nullptr;
  if (occ_e.has_value() || occ_r.has_value()) {
    TORCH_CHECK(occ_e.has_value() && occ_r.has_value() && key_e.has_value() && key_r.has_value(),
                "kg_step: occ_e, occ_r, key_e and key_r go together");
    typed(*occ_e, torch::kFloat32, "occ_e");
    typed(*occ_r, torch::kFloat32, "occ_r");
    typed(*key_e, torch::kInt64, "key_e");
    typed(*key_r, torch::kInt64, "key_r");
    TORCH_CHECK(occ_e->numel() == B * (2 + K) * D && occ_r->numel() == B * D, "kg_step: occ_e [B(2+K), D], occ_r [B, D]");
    TORCH_CHECK(key_e->numel() == B * (2 + K) && key_r->numel() == B, "kg_step: key_e [B(2+K)], key_r [B]");
    oe = occ_e->data_ptr<float>();
    orr = occ_r->data_ptr<float>();
    ke = key_e->data_ptr<int64_t>();
    kr = key_r->data_ptr<int64_t>();
  }
  TORCH_CHECK(part.numel() >= nparts, "kg_step: part needs ", nparts, " entries");
  TORCH_CHECK(pool.numel() > 0 && loss.numel() >= 1 && step.numel() >= 1, "kg_step: empty pool / loss / step");
  const c10::DeviceGuard g(h.device());
  ok(eh_kg_step(h.data_ptr<float>(), rel.data_ptr<float>(), pool.data_ptr<int64_t>(), pool.numel(),
                t_src.data_ptr<int64_t>(), t_dst.data_ptr<int64_t>(), t_rel.data_ptr<int64_t>(), h.size(0),
                step.data_ptr<int64_t>(), static_cast<uint64_t>(seed), B, static_cast<int>(K), static_cast<int>(D),
                static_cast<int>(kind), normalize ? 1 : 0, static_cast<float>(margin), o_src.data_ptr<int64_t>(),
                o_dst.data_ptr<int64_t>(), o_ridx.data_ptr<int64_t>(), o_neg.data_ptr<int64_t>(),
                coef.data_ptr<float>(), part.data_ptr<float>(), loss.data_ptr<float>(), dent.data_ptr<float>(),
                drel.data_ptr<float>(), nullptr, rep_p, rep, rel.size(0), stream(), oe, orr, ke, kr),
     "kg_step");
}

int64_t kg_step_parts(int64_t B, int64_t D) {
  int nparts = 0;
  ok(eh_kg_step(nullptr, nullptr, nullptr, 1, nullptr, nullptr, nullptr, 1, nullptr, 0, B, 1, static_cast<int>(D), 1,
                0, 0.f, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, nullptr, &nparts,
                nullptr, 0, 0, nullptr),
     "kg_step_parts");
  return nparts;
}

// x0 = x * keep (per-row Philox keep mask, probability 1 - p), keep [n] fp32 0 / 1
void drop_rows(torch::Tensor x, double p, int64_t seed, torch::Tensor step, int64_t salt, torch::Tensor x0,
               torch::Tensor keep) {
  for (auto* t : {&x, &x0, &keep}) typed(*t, torch::kFloat32, "drop_rows buffer");
  typed(step, torch::kInt64, "step");
  TORCH_CHECK(x.dim() == 2 && x0.sizes() == x.sizes() && keep.numel() == x.size(0) && x.size(1) % 4 == 0,
              "drop_rows: x [n, d] (d % 4 == 0), x0 like x, keep [n]");
  TORCH_CHECK(salt >= 0 && salt < (1 << 24), "drop_rows: 0 <= salt < 2^24");
  const c10::DeviceGuard g(x.device());
  ok(eh_drop_rows(x.data_ptr<float>(), x.size(0), static_cast<int>(x.size(1)), static_cast<float>(p),
                  static_cast<uint64_t>(seed), step.data_ptr<int64_t>(), static_cast<uint64_t>(salt),
                  x0.data_ptr<float>(), keep.data_ptr<float>(), stream()),
     "drop_rows");
}

// fp32 -> bf16 copy (out: bf16, same number of elements, both contiguous)
void cast_bf16(torch::Tensor x, torch::Tensor out) {
  typed(x, torch::kFloat32, "x");
  typed(out, torch::kBFloat16, "out");
  TORCH_CHECK(x.numel() == out.numel() && x.numel() % 4 == 0, "cast_bf16: same size, multiple of 4");
  const c10::DeviceGuard g(x.device());
  ok(eh_cast_bf16(x.data_ptr<float>(), x.numel(), out.data_ptr(), stream()), "cast_bf16");
}

// t = 0: one vector-store kernel (zero_kernel, embed.hip); EULER_AMD_ZERO_MEMSET=1: one
// hipMemsetAsync instead (read per call, so a test can switch it)
void zero_(torch::Tensor t) {
  dev(t, "t");
  const c10::DeviceGuard g(t.device());
  const char* e = std::getenv("EULER_AMD_ZERO_MEMSET");
  const bool use_memset = e && e[0] == '1';
  const int64_t bytes = t.numel() * t.element_size();
  if (use_memset) {
    ok(hipMemsetAsync(t.data_ptr(), 0, static_cast<size_t>(bytes), stream()), "zero_ (memset)");
    return;
  }
  ok(eh_zero(t.data_ptr(), bytes, stream()), "zero_");
}

// t = 0 through hipMemsetAsync, always (diagnostics: tests/test_graph_memset.py)
void memset_zero(torch::Tensor t) {
  dev(t, "t");
  const c10::DeviceGuard g(t.device());
  ok(hipMemsetAsync(t.data_ptr(), 0, static_cast<size_t>(t.numel() * t.element_size()), stream()), "memset_zero");
}

// hipGraphUpload of an instantiated graph (torch.cuda.CUDAGraph.raw_cuda_graph_exec()) on
// torch's current stream: the executable's device-side state is prepared ahead of its first
// launch, so the first replay starts like every later one
void graph_upload(int64_t exec_handle) {
  hipGraphExec_t e = reinterpret_cast<hipGraphExec_t>(static_cast<uintptr_t>(exec_handle));
  TORCH_CHECK(e != nullptr, "graph_upload: null graph exec");
  ok(hipGraphUpload(e, c10::hip::getCurrentHIPStream().stream()), "graph upload");
}

// Nodes and dependency edges of a captured hipGraph (torch.cuda.CUDAGraph(keep_graph=True)
// .raw_cuda_graph()), plus hipGraphDebugDotPrint into dot_path when given.  Every node:
// (index, kind, detail) — kernel name, memset (dst, bytes, value) or memcpy; edges as
// (from, to) index pairs (diagnostics: tests/test_graph_memset.py, tools/graph_dot.py).
py::dict graph_summary(int64_t handle, const std::string& dot_path) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>(static_cast<uintptr_t>(handle));
  TORCH_CHECK(g != nullptr, "graph_summary: null graph");
  if (!dot_path.empty()) ok(hipGraphDebugDotPrint(g, dot_path.c_str(), hipGraphDebugDotFlagsVerbose), "dot print");
  size_t n = 0;
  ok(hipGraphGetNodes(g, nullptr, &n), "graph nodes");
  std::vector<hipGraphNode_t> nodes(n);
  if (n) ok(hipGraphGetNodes(g, nodes.data(), &n), "graph nodes");
  std::map<hipGraphNode_t, int64_t> index;
  py::list out_nodes;
  for (size_t i = 0; i < n; ++i) {
    index[nodes[i]] = static_cast<int64_t>(i);
    hipGraphNodeType t;
    ok(hipGraphNodeGetType(nodes[i], &t), "node type");
    std::string kind, detail;
    switch (t) {
      case hipGraphNodeTypeKernel: {
        kind = "kernel";
        hipKernelNodeParams kp{};
        if (hipGraphKernelNodeGetParams(nodes[i], &kp) == hipSuccess && kp.func) {
          const char* nm = hipKernelNameRefByPtr(kp.func, nullptr);
          detail = nm ? nm : "?";
        }
        break;
      }
      case hipGraphNodeTypeMemset: {
        kind = "memset";
        hipMemsetParams mp{};
        if (hipGraphMemsetNodeGetParams(nodes[i], &mp) == hipSuccess)
          detail = "dst=" + std::to_string(reinterpret_cast<uintptr_t>(mp.dst)) + " bytes=" +
                   std::to_string(static_cast<uint64_t>(mp.width) * mp.height * mp.elementSize) +
                   " value=" + std::to_string(mp.value);
        break;
      }
      case hipGraphNodeTypeMemcpy: kind = "memcpy"; break;
      case hipGraphNodeTypeEmpty: kind = "empty"; break;
      case hipGraphNodeTypeWaitEvent: kind = "wait_event"; break;
      case hipGraphNodeTypeEventRecord: kind = "event_record"; break;
      case hipGraphNodeTypeHost: kind = "host"; break;
      default: kind = "type" + std::to_string(static_cast<int>(t)); break;
    }
    out_nodes.append(py::make_tuple(static_cast<int64_t>(i), kind, detail));
  }
  size_t ne = 0;
  ok(hipGraphGetEdges(g, nullptr, nullptr, &ne), "graph edges");
  std::vector<hipGraphNode_t> from(ne), to(ne);
  if (ne) ok(hipGraphGetEdges(g, from.data(), to.data(), &ne), "graph edges");
  py::list edges;
  for (size_t e = 0; e < ne; ++e) edges.append(py::make_tuple(index[from[e]], index[to[e]]));
  py::dict d;
  d["nodes"] = out_nodes;
  d["edges"] = edges;
  return d;
}

// one hop's block of the device full-neighbourhood flow (flow.hip flow_block_kernel):
// returns (new_n_id [cap_n], res_n_id [cap_prev], edge_index [2, E], perm [E],
// indptr [cap_prev + 1], counts [cap_prev], last_idx [cap_n], n_targets [1] of the next hop)
std::vector<torch::Tensor> flow_block(torch::Tensor src, torch::Tensor offs, torch::Tensor uniq, torch::Tensor inv,
                                      torch::Tensor cnt, torch::Tensor last_idx, torch::Tensor n_targets,
                                      int64_t cap_n, bool self_loops, torch::Tensor overflow) {
  for (auto* t : {&src, &offs, &uniq, &inv, &cnt, &last_idx, &n_targets}) typed(*t, torch::kInt64, "flow_block id");
  typed(overflow, torch::kInt32, "overflow");
  const int64_t cap_e = src.numel(), cap_prev = offs.numel();
  TORCH_CHECK(cap_prev > 0 && cap_n > 0 && last_idx.numel() == cap_prev, "flow_block: last_idx [cap_prev]");
  TORCH_CHECK(uniq.numel() == cap_e + cap_prev && inv.numel() == cap_e + cap_prev,
              "flow_block: uniq / inv over [neighbours, previous set]");
  TORCH_CHECK(cnt.numel() >= 1 && n_targets.numel() >= 1 && overflow.numel() >= 1, "flow_block: scalars");
  const int64_t E = self_loops ? cap_e + cap_prev : cap_e;
  const c10::DeviceGuard g(src.device());
  auto o = src.options();
  auto new_n_id = torch::empty({cap_n}, o), res = torch::empty({cap_prev}, o), ei = torch::empty({2, E}, o);
  auto perm = torch::empty({E}, o), indptr = torch::empty({cap_prev + 1}, o), counts = torch::empty({cap_prev}, o);
  auto last_new = torch::empty({cap_n}, o), cnt_new = torch::empty({1}, o);
  ok(eh_flow_block(src.data_ptr<int64_t>(), offs.data_ptr<int64_t>(), uniq.data_ptr<int64_t>(),
                   inv.data_ptr<int64_t>(), cnt.data_ptr<int64_t>(), last_idx.data_ptr<int64_t>(),
                   n_targets.data_ptr<int64_t>(), cap_e, cap_prev, cap_n, self_loops ? 1 : 0,
                   new_n_id.data_ptr<int64_t>(), res.data_ptr<int64_t>(), ei.data_ptr<int64_t>(),
                   perm.data_ptr<int64_t>(), indptr.data_ptr<int64_t>(), counts.data_ptr<int64_t>(),
                   last_new.data_ptr<int64_t>(), cnt_new.data_ptr<int64_t>(), overflow.data_ptr<int32_t>(), stream()),
     "flow_block");
  return {new_n_id, res, ei, perm, indptr, counts, last_new, cnt_new};
}

// one hop's block of the fixed-fanout device SageDataFlow (flow.hip sage_block / sage_place):
// returns (new_n_id, res_n_id, edge_index [2, E], perm [E], indptr [cap_prev + 1],
// counts [cap_prev], last_idx [cap_n], n_targets [1] of the next hop)
std::vector<torch::Tensor> sage_block(torch::Tensor inv, torch::Tensor uniq, torch::Tensor cnt,
                                      torch::Tensor last_idx, int64_t f, int64_t cap_n, bool self_loops) {
  for (auto* t : {&inv, &uniq, &cnt, &last_idx}) typed(*t, torch::kInt64, "sage_block id");
  const int64_t cap_prev = last_idx.numel();
  TORCH_CHECK(f > 0 && cap_prev > 0 && cap_n > 0 && inv.numel() == cap_prev * (f + 1) && uniq.numel() == inv.numel(),
              "sage_block: inv / uniq over [cap_prev * f neighbours, cap_prev previous]");
  const int64_t E = self_loops ? cap_prev * (f + 1) : cap_prev * f;
  const c10::DeviceGuard g(inv.device());
  auto o = inv.options();
  auto new_n_id = torch::empty({cap_n}, o), res = torch::empty({cap_prev}, o), ei = torch::empty({2, E}, o);
  auto counts = torch::empty({cap_prev}, o), last_new = torch::empty({cap_n}, o), cnt_new = torch::empty({1}, o);
  ok(eh_sage_block(inv.data_ptr<int64_t>(), uniq.data_ptr<int64_t>(), cnt.data_ptr<int64_t>(),
                   last_idx.data_ptr<int64_t>(), cap_prev, f, cap_n, self_loops ? 1 : 0, new_n_id.data_ptr<int64_t>(),
                   res.data_ptr<int64_t>(), ei.data_ptr<int64_t>(), counts.data_ptr<int64_t>(),
                   last_new.data_ptr<int64_t>(), cnt_new.data_ptr<int64_t>(), stream()),
     "sage_block");
  auto indptr = torch::empty({cap_prev + 1}, o);
  ok(eh_zero(indptr.data_ptr(), 8, stream()), "sage_block indptr");
  auto tail = indptr.narrow(0, 1, cap_prev);
  torch::cumsum_out(tail, counts, 0);
  auto perm = torch::empty({E}, o);
  ok(eh_sage_place(inv.data_ptr<int64_t>(), last_idx.data_ptr<int64_t>(), cap_prev, f, self_loops ? 1 : 0,
                   indptr.data_ptr<int64_t>(), perm.data_ptr<int64_t>(), stream()),
     "sage_place");
  return {new_n_id, res, ei, perm, indptr, counts, last_new, cnt_new};
}

// GCN symmetric-norm edge weights from the two endpoint degree vectors (flow.hip)
torch::Tensor gcn_norm_weight(torch::Tensor edge_index, torch::Tensor c0, torch::Tensor c1) {
  typed(edge_index, torch::kInt64, "edge_index");
  typed(c0, torch::kInt64, "c0");
  typed(c1, torch::kInt64, "c1");
  TORCH_CHECK(edge_index.dim() == 2 && edge_index.size(0) == 2, "gcn_norm_weight: edge_index [2, E]");
  const int64_t E = edge_index.size(1);
  const c10::DeviceGuard g(edge_index.device());
  auto w = torch::empty({E}, edge_index.options().dtype(torch::kFloat32));
  ok(eh_gcn_norm_weight(edge_index.data_ptr<int64_t>(), edge_index.data_ptr<int64_t>() + E, E,
                        c0.data_ptr<int64_t>(), c0.numel(), c1.data_ptr<int64_t>(), c1.numel(), w.data_ptr<float>(),
                        stream()),
     "gcn_norm_weight");
  return w;
}

// multi-label sigmoid cross-entropy (mean) of x [B, C] against labels[rows] [N, C] and the
// F1 counts (tp, fp, fn) added into counts [3] int64; returns the 0-d loss
torch::Tensor bce_f1_fwd(torch::Tensor x, torch::Tensor labels, torch::Tensor rows, torch::Tensor counts) {
  typed(x, torch::kFloat32, "x");
  typed(labels, torch::kFloat32, "labels");
  typed(rows, torch::kInt64, "rows");
  typed(counts, torch::kInt64, "counts");
  TORCH_CHECK(x.dim() == 2 && labels.dim() == 2 && labels.size(1) == x.size(1) && rows.numel() == x.size(0) &&
                  counts.numel() >= 3,
              "bce_f1_fwd: x [B, C], labels [N, C], rows [B], counts [3]");
  const c10::DeviceGuard g(x.device());
  auto part = torch::empty({eh_bce_parts(x.numel())}, x.options());
  auto loss = torch::empty({}, x.options());
  ok(eh_bce_f1_fwd(x.data_ptr<float>(), labels.data_ptr<float>(), rows.data_ptr<int64_t>(), x.size(0),
                   static_cast<int>(x.size(1)), part.data_ptr<float>(), loss.data_ptr<float>(),
                   counts.data_ptr<int64_t>(), stream()),
     "bce_f1_fwd");
  return loss;
}

torch::Tensor bce_bwd(torch::Tensor x, torch::Tensor labels, torch::Tensor rows, torch::Tensor g) {
  typed(x, torch::kFloat32, "x");
  typed(labels, torch::kFloat32, "labels");
  typed(rows, torch::kInt64, "rows");
  typed(g, torch::kFloat32, "g");
  TORCH_CHECK(x.dim() == 2 && labels.size(1) == x.size(1) && rows.numel() == x.size(0) && g.numel() == 1,
              "bce_bwd: x [B, C], labels [N, C], rows [B], g scalar");
  const c10::DeviceGuard gd(x.device());
  auto dx = torch::empty_like(x);
  ok(eh_bce_bwd(x.data_ptr<float>(), labels.data_ptr<float>(), rows.data_ptr<int64_t>(), x.size(0),
                static_cast<int>(x.size(1)), g.data_ptr<float>(), dx.data_ptr<float>(), stream()),
     "bce_bwd");
  return dx;
}

// per-segment sizes of an index vector (entries outside [0, size) skipped), int64 [size]
torch::Tensor seg_count(torch::Tensor idx, int64_t size) {
  typed(idx, torch::kInt64, "idx");
  TORCH_CHECK(size >= 0, "seg_count: size >= 0");
  const c10::DeviceGuard g(idx.device());
  auto cnt = torch::empty({size}, idx.options());
  ok(eh_zero(cnt.data_ptr(), size * 8, stream()), "seg_count zero");
  ok(eh_seg_count(idx.data_ptr<int64_t>(), idx.numel(), size, cnt.data_ptr<int64_t>(), stream()), "seg_count");
  return cnt;
}

void kg_bwd(torch::Tensor ent, torch::Tensor rel, torch::Tensor src, torch::Tensor dst, torch::Tensor ridx,
            torch::Tensor neg, int64_t kind, int64_t corrupt, bool normalize, torch::Tensor gpos, torch::Tensor gneg,
            torch::Tensor dent, torch::Tensor drel, bool occ) {
  const KgIn k = kg_check(ent, rel, src, dst, ridx, neg, kind, corrupt);
  typed(gpos, torch::kFloat32, "gpos");
  typed(gneg, torch::kFloat32, "gneg");
  typed(dent, torch::kFloat32, "dent");
  typed(drel, torch::kFloat32, "drel");
  TORCH_CHECK(gpos.numel() == k.B && gneg.numel() == k.B * k.nneg, "score grads must match the scores");
  if (occ) {  // per-occurrence rows: [B * (2 + K), D] entities (h, t, negatives), [B, D] relations
    TORCH_CHECK(dent.dim() == 2 && dent.size(0) == k.B * (2 + k.K) && dent.size(1) == k.D && drel.dim() == 2 &&
                    drel.size(0) == k.B && drel.size(1) == k.D,
                "occurrence grads must be [B*(2+K), D] and [B, D]");
  } else {
    TORCH_CHECK(dent.sizes() == ent.sizes() && drel.sizes() == rel.sizes(), "table grads must match the tables");
  }
  const c10::DeviceGuard g(ent.device());
  ok(eh_kg_bwd(ent.data_ptr<float>(), rel.data_ptr<float>(), src.data_ptr<int64_t>(), dst.data_ptr<int64_t>(),
               ridx.data_ptr<int64_t>(), neg.data_ptr<int64_t>(), k.B, static_cast<int>(k.K), static_cast<int>(k.D),
               static_cast<int>(kind), static_cast<int>(corrupt), normalize ? 1 : 0, gpos.data_ptr<float>(),
               gneg.data_ptr<float>(), dent.data_ptr<float>(), drel.data_ptr<float>(), occ ? 1 : 0, stream()),
     "kg_bwd");
}

// ----------------------------------------------------------------------------- unique
std::vector<torch::Tensor> unique_first(torch::Tensor x) {
  typed(x, torch::kInt64, "x");
  const int64_t n = x.numel();
  TORCH_CHECK(n < (1ll << 30), "unique_first supports < 2^30 elements");
  const c10::DeviceGuard g(x.device());
  auto opts = x.options();
  if (n == 0) return {torch::empty({0}, opts), torch::empty({0}, opts)};
  int64_t cap = 1;
  while (cap < 2 * n) cap <<= 1;
  auto keys = torch::empty({cap}, opts);
  auto minpos = torch::empty({cap}, opts.dtype(torch::kInt32));
  ok(eh_unique_init(keys.data_ptr(), minpos.data_ptr<int32_t>(), cap, stream()), "unique_init");
  auto slot = torch::empty({n}, opts.dtype(torch::kInt32));
  auto flag = torch::empty({n}, opts.dtype(torch::kInt32));
  ok(eh_unique_insert(x.data_ptr<int64_t>(), n, keys.data_ptr(), minpos.data_ptr<int32_t>(), cap,
                      slot.data_ptr<int32_t>(), 0, stream()),
     "unique_insert");
  ok(eh_unique_mark(n, slot.data_ptr<int32_t>(), minpos.data_ptr<int32_t>(), flag.data_ptr<int32_t>(), stream()),
     "unique_mark");
  auto pos = torch::cumsum(flag, 0, torch::kInt32);
  const int64_t u = pos[n - 1].item<int32_t>();
  auto uniq = torch::empty({u}, opts);
  auto inv = torch::empty({n}, opts);
  ok(eh_unique_finalize(x.data_ptr<int64_t>(), n, slot.data_ptr<int32_t>(), minpos.data_ptr<int32_t>(),
                        flag.data_ptr<int32_t>(), pos.data_ptr<int32_t>(), inv.data_ptr<int64_t>(),
                        uniq.data_ptr<int64_t>(), 0, stream()),
     "unique_finalize");
  return {uniq, inv};
}

// Fixed-capacity form for graph-captured steps: no host read of the unique count.
// uniq [n] holds the distinct values in first-occurrence order followed by `fill`,
// count [1] (device) the number of distinct values.
// offset: added to every distinct value (not to the fill), e.g. a table half's base row
std::vector<torch::Tensor> unique_first_padded(torch::Tensor x, int64_t fill, int64_t offset) {
  typed(x, torch::kInt64, "x");
  const int64_t n = x.numel();
  TORCH_CHECK(n < (1ll << 30), "unique_first_padded supports < 2^30 elements");
  const c10::DeviceGuard g(x.device());
  auto opts = x.options();
  if (n == 0) return {torch::empty({0}, opts), torch::empty({0}, opts), torch::zeros({1}, opts)};
  int64_t cap = 1;
  while (cap < 2 * n) cap <<= 1;
  auto keys = torch::empty({cap}, opts);
  auto minpos = torch::empty({cap}, opts.dtype(torch::kInt32));
  ok(eh_unique_init(keys.data_ptr(), minpos.data_ptr<int32_t>(), cap, stream()), "unique_init");
  auto slot = torch::empty({n}, opts.dtype(torch::kInt32));
  auto flag = torch::empty({n}, opts.dtype(torch::kInt32));
  ok(eh_unique_insert(x.data_ptr<int64_t>(), n, keys.data_ptr(), minpos.data_ptr<int32_t>(), cap,
                      slot.data_ptr<int32_t>(), 1, stream()),
     "unique_insert");
  ok(eh_unique_mark(n, slot.data_ptr<int32_t>(), minpos.data_ptr<int32_t>(), flag.data_ptr<int32_t>(), stream()),
     "unique_mark");
  auto pos = torch::cumsum(flag, 0, torch::kInt32);
  auto uniq = torch::full({n}, fill, opts);
  auto inv = torch::empty({n}, opts);
  ok(eh_unique_finalize(x.data_ptr<int64_t>(), n, slot.data_ptr<int32_t>(), minpos.data_ptr<int32_t>(),
                        flag.data_ptr<int32_t>(), pos.data_ptr<int32_t>(), inv.data_ptr<int64_t>(),
                        uniq.data_ptr<int64_t>(), offset, stream()),
     "unique_finalize");
  return {uniq, inv, pos.narrow(0, n - 1, 1).to(torch::kInt64)};
}

// Full neighbours of a capacity-padded row set (flow.hip): (nbr rows, target positions,
// inclusive per-target edge offsets [n]); the first two int64 [cap], -1 past the real edge
// count; overflow[0] |= 1 when the edges exceed cap.
// No allocation beyond the outputs and one scan buffer, no host sync (hipGraph-capturable).
std::vector<torch::Tensor> full_neighbors(torch::Tensor indptr, torch::Tensor nbr, int64_t num_rows,
                                          int64_t num_types, int64_t mask, torch::Tensor rows, int64_t cap,
                                          torch::Tensor overflow) {
  typed(indptr, torch::kInt64, "indptr");
  typed(nbr, torch::kInt32, "nbr");
  typed(rows, torch::kInt64, "rows");
  typed(overflow, torch::kInt32, "overflow");
  TORCH_CHECK(indptr.numel() == num_rows * num_types + 1, "full_neighbors: indptr size mismatch");
  TORCH_CHECK(num_types >= 1 && num_types <= 32 && cap >= 0, "full_neighbors: bad arguments");
  const c10::DeviceGuard g(rows.device());
  const int64_t n = rows.numel();
  auto opts = rows.options();
  auto out_nbr = torch::empty({cap}, opts);
  auto out_src = torch::empty({cap}, opts);
  if (n == 0) {
    out_nbr.fill_(-1);
    out_src.fill_(-1);
    return {out_nbr, out_src, torch::zeros({0}, opts)};
  }
  auto deg = torch::empty({n}, opts);
  ok(eh_flow_degree(indptr.data_ptr<int64_t>(), num_rows, static_cast<int>(num_types), static_cast<uint32_t>(mask),
                    rows.data_ptr<int64_t>(), n, deg.data_ptr<int64_t>(), stream()),
     "flow_degree");
  auto offs = torch::cumsum(deg, 0);
  ok(eh_flow_expand(indptr.data_ptr<int64_t>(), nbr.data_ptr<int32_t>(), num_rows, static_cast<int>(num_types),
                    static_cast<uint32_t>(mask), rows.data_ptr<int64_t>(), n, offs.data_ptr<int64_t>(), cap,
                    out_nbr.data_ptr<int64_t>(), out_src.data_ptr<int64_t>(), overflow.data_ptr<int32_t>(),
                    stream()),
     "flow_expand");
  return {out_nbr, out_src, offs};  // offs: inclusive edge offsets per target
}

// C = op(A) op(B) (+ bias) (relu) (* relu'(rmask)) with the tiled MFMA GEMM (gemm.hip):
// trans_a: A is [K][M]; trans_b: B is [N][K] (else [K][N]); A, B fp32 or bf16 row-major
// (unit inner stride); C fp32 or bf16 [M][N] (row stride >= N) is written in place.
// splits > 1: split-K over the reduction dimension (deterministic slabs + one reduce).
void gemm(torch::Tensor A, torch::Tensor B, torch::Tensor C, bool trans_a, bool trans_b,
          c10::optional<torch::Tensor> bias, c10::optional<torch::Tensor> rmask, bool relu, int64_t splits,
          double alpha, c10::optional<torch::Tensor> addend, c10::optional<torch::Tensor> row_scale) {
  auto fp = [](const torch::Tensor& t, const char* n) {
    TORCH_CHECK(t.is_cuda() && t.dim() == 2 && t.stride(1) == 1 &&
                    (t.scalar_type() == torch::kFloat32 || t.scalar_type() == torch::kBFloat16),
                n, " must be a 2-D fp32/bf16 GPU matrix with unit inner stride");
  };
  fp(A, "A");
  fp(B, "B");
  fp(C, "C");
  const int64_t M = trans_a ? A.size(1) : A.size(0), K = trans_a ? A.size(0) : A.size(1);
  const int64_t N = trans_b ? B.size(0) : B.size(1), KB = trans_b ? B.size(1) : B.size(0);
  TORCH_CHECK(K == KB, "gemm: inner dimensions differ (", K, " vs ", KB, ")");
  TORCH_CHECK(C.size(0) == M && C.size(1) == N, "gemm: C must be [", M, ", ", N, "]");
  TORCH_CHECK(splits >= 1 && splits <= 1024, "gemm: 1 <= splits <= 1024");
  const float* bp = nullptr;
  if (bias.has_value()) {
    typed(*bias, torch::kFloat32, "bias");
    TORCH_CHECK(bias->numel() == N, "gemm: bias must have N elements");
    bp = bias->data_ptr<float>();
  }
  const void* rp = nullptr;
  int64_t ldr = 0;
  int r_bf16 = 0;
  if (rmask.has_value()) {
    fp(*rmask, "rmask");
    TORCH_CHECK(rmask->size(0) == M && rmask->size(1) == N, "gemm: rmask must be [M, N]");
    rp = rmask->data_ptr();
    ldr = rmask->stride(0);
    r_bf16 = rmask->scalar_type() == torch::kBFloat16;
  }
  const void* ap = nullptr;  // residual added in the epilogue (may be C itself)
  int64_t lda_add = 0;
  int add_bf16 = 0;
  if (addend.has_value()) {
    fp(*addend, "addend");
    TORCH_CHECK(addend->size(0) >= M && addend->size(1) >= N, "gemm: addend must cover [M, N]");
    ap = addend->data_ptr();
    lda_add = addend->stride(0);
    add_bf16 = addend->scalar_type() == torch::kBFloat16;
  }
  const float* rs = nullptr;  // per-row scale of the product
  if (row_scale.has_value()) {
    typed(*row_scale, torch::kFloat32, "row_scale");
    TORCH_CHECK(row_scale->numel() == M, "gemm: row_scale must have M elements");
    rs = row_scale->data_ptr<float>();
  }
  const c10::DeviceGuard g(A.device());
  torch::Tensor part;
  if (splits > 1) part = torch::empty({splits * M * N}, A.options().dtype(torch::kFloat32));
  static const bool tn_on = [] {  // EULER_AMD_GEMM_TN=0: the generic kernel's strided path
    const char* e = std::getenv("EULER_AMD_GEMM_TN");
    return !(e && e[0] == '0');
  }();
  if (tn_on && trans_a && !trans_b && !bp && !rp && !relu) {
    // both operands k-major: the transposing-read kernel
    ok(eh_gemm_tn(A.data_ptr(), B.data_ptr(), C.data_ptr(), splits > 1 ? part.data_ptr<float>() : nullptr, M, N, K,
                  A.stride(0), B.stride(0), C.stride(0), A.scalar_type() == torch::kBFloat16,
                  B.scalar_type() == torch::kBFloat16, C.scalar_type() == torch::kBFloat16, static_cast<int>(splits),
                  static_cast<float>(alpha), ap, lda_add, add_bf16, rs, stream()),
       "gemm_tn");
    return;
  }
  ok(eh_gemm(A.data_ptr(), B.data_ptr(), C.data_ptr(), bp, rp, splits > 1 ? part.data_ptr<float>() : nullptr, M, N, K,
             A.stride(0), B.stride(0), C.stride(0), ldr, trans_a ? 1 : 0, trans_b ? 0 : 1,
             A.scalar_type() == torch::kBFloat16, B.scalar_type() == torch::kBFloat16,
             C.scalar_type() == torch::kBFloat16, r_bf16, relu ? 1 : 0, static_cast<int>(splits),
             static_cast<float>(alpha), ap, lda_add, add_bf16, rs, stream()),
     "gemm");
}

// (pos [n] slot of every id in the W*C exchange space, W*C = none / did not fit; send
// [W*C + 1] the id of every slot, -1 = empty); overflow [1] int32 is set to 1 when an id
// did not fit its owner's C slots
std::vector<torch::Tensor> route_by_owner(torch::Tensor ids, int64_t W, int64_t C, torch::Tensor overflow,
                                          int64_t self_rank) {
  typed(ids, torch::kInt64, "ids");
  typed(overflow, torch::kInt32, "overflow");
  TORCH_CHECK(overflow.numel() >= 1 && overflow.device() == ids.device(), "overflow must be [1] int32 on the ids' device");
  TORCH_CHECK(W >= 1 && W <= 63 && C >= 1 && self_rank < W, "route_by_owner: 1 <= W <= 63, C >= 1, self_rank < W");
  const int64_t n = ids.numel();
  const c10::DeviceGuard g(ids.device());
  auto opts = ids.options();
  auto pos = torch::empty({n}, opts);
  auto send = torch::full({W * C + 1}, -1, opts);
  auto cnt = torch::empty({std::max<int64_t>(eh_route_chunks(n), 1) * (W + 1)}, opts.dtype(torch::kInt32));
  ok(eh_route_by_owner(ids.data_ptr<int64_t>(), n, static_cast<int>(W), C, static_cast<int>(self_rank),
                       cnt.data_ptr<int32_t>(),
                       pos.data_ptr<int64_t>(), send.data_ptr<int64_t>(), overflow.data_ptr<int32_t>(), stream()),
     "route_by_owner");
  return {pos, send};
}

}  // namespace

void register_gnn_ops(pybind11::module& m) {
  m.def("route_by_owner", &route_by_owner, py::arg("ids"), py::arg("W"), py::arg("C"), py::arg("overflow"),
        py::arg("self_rank") = -1);
  m.def("gemm", &gemm, py::arg("A"), py::arg("B"), py::arg("C"), py::arg("trans_a") = false,
        py::arg("trans_b") = false, py::arg("bias") = py::none(), py::arg("rmask") = py::none(),
        py::arg("relu") = false, py::arg("splits") = 1, py::arg("alpha") = 1.0, py::arg("addend") = py::none(),
        py::arg("row_scale") = py::none());
  m.def("gat_supported", &gat_supported);
  m.def("gat_fwd", &gat_fwd, py::arg("indptr"), py::arg("col"), py::arg("order"), py::arg("h"), py::arg("al"),
        py::arg("ar"), py::arg("H"), py::arg("C"), py::arg("slope"), py::arg("a_src") = py::none());
  m.def("gat_bwd", &gat_bwd, py::arg("indptr"), py::arg("col"), py::arg("order"), py::arg("cindptr"), py::arg("crow"),
        py::arg("corder"), py::arg("h"), py::arg("al"), py::arg("ar"), py::arg("H"), py::arg("C"), py::arg("slope"),
        py::arg("out"), py::arg("dout"), py::arg("lse"), py::arg("a_src") = py::none());
  m.def("gat_att_fwd", &gat_att_fwd);
  m.def("gat_att_bwd_", &gat_att_bwd_);
  m.def("rel_gemm", &rel_gemm);
  m.def("rel_gemm_dw", &rel_gemm_dw, py::arg("G"), py::arg("g_idx"), py::arg("X"), py::arg("x_idx"), py::arg("scale"),
        py::arg("trel"), py::arg("tstart"), py::arg("tlen"), py::arg("solo"), py::arg("dW"),
        py::arg("accumulate") = false, py::arg("slot") = py::none(), py::arg("part") = py::none(),
        py::arg("mrel") = py::none(), py::arg("mrp") = py::none());
  m.def("rel_weight_bf16", &rel_weight_bf16);
  m.attr("rel_gemm_dw_chunk") = eh_rel_gemm_dw_chunk();
  m.attr("rel_gemm_tile") = eh_rel_gemm_tile();
  m.def("sgns_fwd", &sgns_fwd);
  m.def("sgns_bwd", &sgns_bwd);
  m.def("sgns_fwd_idx", &sgns_fwd_idx);
  m.def("occ_csr", &occ_csr);
  m.def("sgns_grad", &sgns_grad);
  m.def("gather_f32_bf16", &gather_f32_bf16, py::arg("x"), py::arg("idx"), py::arg("out") = py::none());
  m.def("sgns_apply_", &sgns_apply_);
  m.def("kg_fwd", &kg_fwd);
  m.def("kg_step", &kg_step, py::arg("h"), py::arg("rel"), py::arg("pool"), py::arg("t_src"), py::arg("t_dst"),
        py::arg("t_rel"), py::arg("step"), py::arg("seed"), py::arg("kind"), py::arg("normalize"), py::arg("margin"),
        py::arg("o_src"), py::arg("o_dst"), py::arg("o_ridx"), py::arg("o_neg"), py::arg("coef"), py::arg("part"),
        py::arg("loss"), py::arg("dent"), py::arg("drel"), py::arg("drel_rep") = py::none(),
        py::arg("occ_e") = py::none(), py::arg("occ_r") = py::none(), py::arg("key_e") = py::none(),
        py::arg("key_r") = py::none());
  m.def("det_occ", &det_occ, py::arg("keys"), py::arg("S"));
  m.def("det_segment_sum", &det_segment_sum, py::arg("src"), py::arg("ptr"), py::arg("perm"), py::arg("out"));
  m.def("kg_step_parts", &kg_step_parts);
  m.def("cast_bf16", &cast_bf16);
  m.def("drop_rows", &drop_rows);
  m.def("zero_", &zero_);
  m.def("memset_zero", &memset_zero);
  m.def("graph_summary", &graph_summary, py::arg("graph"), py::arg("dot_path") = "");
  m.def("graph_upload", &graph_upload, py::arg("exec"));
  m.def("seg_count", &seg_count);
  m.def("flow_block", &flow_block);
  m.def("gcn_norm_weight", &gcn_norm_weight);
  m.def("sage_block", &sage_block);
  m.def("bce_f1_fwd", &bce_f1_fwd);
  m.def("bce_bwd", &bce_bwd);
  m.def("pair_fwd", &pair_fwd, py::arg("es"), py::arg("ec"), py::arg("B"), py::arg("K"), py::arg("mrr") = py::none());
  m.def("pair_bwd", &pair_bwd);
  m.def("kg_bwd", &kg_bwd, py::arg("ent"), py::arg("rel"), py::arg("src"), py::arg("dst"), py::arg("ridx"),
        py::arg("neg"), py::arg("kind"), py::arg("corrupt"), py::arg("normalize"), py::arg("gpos"), py::arg("gneg"),
        py::arg("dent"), py::arg("drel"), py::arg("occ") = false);
  m.def("unique_first", &unique_first);
  m.def("unique_first_padded", &unique_first_padded, py::arg("x"), py::arg("fill") = -1, py::arg("offset") = 0);
  m.def("full_neighbors", &full_neighbors);
}
