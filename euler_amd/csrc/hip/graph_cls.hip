// Fused graph-classification training step (GIN / GraphGCN): see graph_cls_args.h for the
// launch sequence, models/graph_cls_trainer.py for the model contract.
//
// One block per drawn graph; the graph's nodes (at most kGcMaxRows) never leave LDS:
// activations of every layer, the aggregate Z of the current conv, the backward buffers and
// the graph's CSR / reverse CSR of each edge-type mask.  GEMMs run on the fp32-input MFMA
// (v_mfma_f32_16x16x4_f32, one fp32 fma chain per output: the torch fp32 oracle's
// numerics), 16 x 16 output tiles dealt round-robin to the block's four waves, A operands
// from LDS (rows padded by 4 floats: the 16 rows x 4 k-columns of a fragment read hit
// distinct banks for the 32-wide layers), B operands (weights, a few KB, L2-resident across
// the blocks) straight from global memory.
#include "hip/common.h"
#include "hip/graph_cls_args.h"
#include "hip/optim_math.h"
#include "hip/tile.h"

namespace euler_hip {

namespace {

__device__ __forceinline__ float4_t mfma_f32x4(float a, float b, float4_t c) {
  return __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c, 0, 0, 0);
}

// uniform selection from a per-layer argument array (no dynamic indexing of kernel args)
template <typename T>
__device__ __forceinline__ T gc_pick(const T (&arr)[kGcMaxLayers], int l) {
  T r = arr[0];
#pragma unroll
  for (int i = 1; i < kGcMaxLayers; ++i)
    if (l == i) r = arr[i];
  return r;
}
template <typename T>
__device__ __forceinline__ T gc_pick9(const T (&arr)[kGcMaxLayers + 1], int l) {
  T r = arr[0];
#pragma unroll
  for (int i = 1; i <= kGcMaxLayers; ++i)
    if (l == i) r = arr[i];
  return r;
}

struct GcGraphAdj {  // one mask's adjacency of this block's graph, in LDS
  const int32_t* off;
  const int32_t* nbr;
  const int32_t* roff;
  const int32_t* rnbr;
};

__device__ __forceinline__ GcGraphAdj gc_adj(const GcStepArgs& a, const int32_t* lds, int j) {
  const int stride = 2 * (a.nmax + 1) + 2 * a.emax;
  GcGraphAdj q;
  q.off = lds + j * stride;
  q.nbr = q.off + a.nmax + 1;
  q.roff = q.nbr + a.emax;
  q.rnbr = q.roff + a.nmax + 1;
  return q;
}

// Z = aggregate of X (rows < nrow; rows >= n are zero):
//   GIN        Z[t] = (1 + eps) x_t + sum_{s in N(t)} x_s (+ x_t: self loop)
//   GraphConv  Z[t] = [x_t | mean_{s in N(t) (+ t)} x_s]
__device__ __forceinline__ void gc_aggregate(int kind, int selfl, const float* X, int ldx, int D, float* Z, int ldz,
                                             const GcGraphAdj& q, int n, int nrow, float epsv) {
  for (int it = threadIdx.x; it < nrow * D; it += kGcThreads) {
    const int t = it / D, c = it - t * D;
    float zs = 0.f, zm = 0.f;
    if (t < n) {
      const float xt = X[t * ldx + c];
      const int e0 = q.off[t], e1 = q.off[t + 1];
      float s = 0.f;
      for (int e = e0; e < e1; ++e) s += X[q.nbr[e] * ldx + c];
      if (selfl) s += xt;
      if (kind == 0) {
        zs = (1.f + epsv) * xt + s;
      } else {
        zs = xt;
        const int cnt = e1 - e0 + selfl;
        zm = cnt > 0 ? s / static_cast<float>(cnt) : 0.f;
      }
    }
    Z[t * ldz + c] = zs;
    if (kind == 1) Z[t * ldz + D + c] = zm;
  }
}

// Y[rows < 16 nrt] = relu(Z @ [W | Wf]^T + bias), rows >= n zeroed
__device__ __forceinline__ void gc_fwd_gemm(const float* Z, int ldz, int K, const float* __restrict__ W,
                                            const float* __restrict__ Wf, int Din, const float* __restrict__ bias,
                                            int Dout, float* Y, int ldy, int n, int nrt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int nct = Dout >> 4;
  for (int tile = wave; tile < nrt * nct; tile += kGcThreads / 64) {
    const int rt = tile / nct, ct = tile - rt * nct;
    const int r0 = rt * 16, o = ct * 16 + lr;
    float4_t acc = {0.f, 0.f, 0.f, 0.f};
    const float* arow = Z + (r0 + lr) * ldz + lk;
    // B (weights, global): 16-deep k chunks, the next chunk's loads issued before this
    // chunk's MFMAs (K % 16 == 0; a chunk never straddles W / Wf since Din % 16 == 0)
    auto load = [&](float (&bv)[4], int k0) {
      const float* w = k0 < Din ? W + o * Din + k0 : Wf + o * Din + (k0 - Din);
#pragma unroll
      for (int u = 0; u < 4; ++u) bv[u] = w[4 * u + lk];
    };
    float bc[4];
    load(bc, 0);
    for (int k0 = 0; k0 < K; k0 += 16) {
      float bn[4];
      if (k0 + 16 < K) load(bn, k0 + 16);
#pragma unroll
      for (int u = 0; u < 4; ++u) acc = mfma_f32x4(arow[k0 + 4 * u], bc[u], acc);
#pragma unroll
      for (int u = 0; u < 4; ++u) bc[u] = bn[u];
    }
    const float bo = bias ? bias[o] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + lk * 4 + j;
      Y[r * ldy + o] = r < n ? fmaxf(acc[j] + bo, 0.f) : 0.f;
    }
  }
}

// dW = G^T Z ([Dout][K], into the slab: columns < Din -> o_w, the rest -> o_wf) and
// dZ = G [W | Wf] ([rows][K], into LDS); G rows >= n are zero
__device__ __forceinline__ void gc_bwd_gemms(const float* G, int ldg, const float* Z, int ldz, int K,
                                             const float* __restrict__ W, const float* __restrict__ Wf, int Din,
                                             int Dout, float* DZ, int n, int nrt, float* slab_w, float* slab_wf) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int nkt = K >> 4, not_ = Dout >> 4;
  const int ndw = not_ * nkt;
  const int nv = (n + 3) & ~3;  // k extent of dW (rows n.. of G are zero)
  for (int tile = wave; tile < ndw + nrt * nkt; tile += kGcThreads / 64) {
    float4_t acc = {0.f, 0.f, 0.f, 0.f};
    if (tile < ndw) {
      const int ot = tile / nkt, kt = tile - ot * nkt;
      const int o0 = ot * 16, k = kt * 16 + lr;
      for (int v0 = 0; v0 < nv; v0 += 4) {
        const int v = v0 + lk;
        acc = mfma_f32x4(G[v * ldg + o0 + lr], Z[v * ldz + k], acc);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int o = o0 + lk * 4 + j;
        if (k < Din) slab_w[o * Din + k] = acc[j];
        else slab_wf[o * Din + (k - Din)] = acc[j];
      }
    } else {
      const int t2 = tile - ndw;
      const int rt = t2 / nkt, kt = t2 - rt * nkt;
      const int r0 = rt * 16, k = kt * 16 + lr;
      const float* wcol = (k < Din ? W + k : Wf + (k - Din)) + lk * Din;
      const float* grow = G + (r0 + lr) * ldg + lk;
      auto load = [&](float (&bv)[4], int o0) {
#pragma unroll
        for (int u = 0; u < 4; ++u) bv[u] = wcol[(o0 + 4 * u) * Din];
      };
      float bc[4];
      load(bc, 0);
      for (int o0 = 0; o0 < Dout; o0 += 16) {  // Dout % 16 == 0
        float bn[4];
        if (o0 + 16 < Dout) load(bn, o0 + 16);
#pragma unroll
        for (int u = 0; u < 4; ++u) acc = mfma_f32x4(grow[o0 + 4 * u], bc[u], acc);
#pragma unroll
        for (int u = 0; u < 4; ++u) bc[u] = bn[u];
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) DZ[(r0 + lk * 4 + j) * ldz + k] = acc[j];
    }
  }
}

__device__ __forceinline__ float block_sum(float v, float* red) {
  v = wave_sum(v);
  const int wave = threadIdx.x >> 6;
  __syncthreads();  // red may still be read by a previous reduction
  if ((threadIdx.x & 63) == 0) red[wave] = v;
  __syncthreads();
  float s = 0.f;
#pragma unroll
  for (int w = 0; w < kGcThreads / 64; ++w) s += red[w];
  return s;
}

__global__ __launch_bounds__(kGcThreads) void gc_step_kernel(GcStepArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char gc_smem[];
  __shared__ int s_g, s_n;
  __shared__ float s_red[kGcThreads / 64];
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  const int L = a.L, kind = a.kind, selfl = a.self_loops;
  float* Z = reinterpret_cast<float*>(gc_smem + a.lds_z);
  float* DY = reinterpret_cast<float*>(gc_smem + a.lds_dy);
  float* DZ = reinterpret_cast<float*>(gc_smem + a.lds_dz);
  float* TAB = reinterpret_cast<float*>(gc_smem + a.lds_tab);
  float* VEC = reinterpret_cast<float*>(gc_smem + a.lds_vec);
  int32_t* ADJ = reinterpret_cast<int32_t*>(gc_smem + a.lds_adj);
  const int ldz = a.ldz, ldy = a.ldy;
  float* slab = a.slab + static_cast<int64_t>(b) * a.S;

  // the graph: uniform draw through the alias table, Philox stream 3 at counter + 1 (the
  // generic step's advance-then-alias_sample); the reduce launch advances the counter
  if (tid == 0) {
    const uint4_t r = Philox::gen(static_cast<uint64_t>(a.rng[0]), (static_cast<uint64_t>(a.rng[1] + 1) << 8) ^ 3ull,
                                  static_cast<uint64_t>(b));
    const uint64_t x = (static_cast<uint64_t>(r[0]) << 32) | r[1];
    int64_t k = static_cast<int64_t>(__umul64hi(x, static_cast<uint64_t>(a.G)));
    if (k >= a.G) k = a.G - 1;
    const int g = (u01(r[2]) < a.gprob[k]) ? static_cast<int>(k) : a.galias[k];
    s_g = g;
    s_n = a.gbase[g + 1] - a.gbase[g];
    a.gidx[b] = g;
    if (b == 0 && a.ostep_inc) a.ostep_inc[0] += 1;  // read by this step's reduce launch
  }
  const int D0 = a.D[0];
  const int tab_n = a.tab_rows * D0;
  for (int i = tid; i < tab_n; i += kGcThreads) TAB[i] = 0.f;
  __syncthreads();
  const int g = s_g, n = s_n, base = a.gbase[g];
  const int nrt = (n + 15) >> 4, nrow = nrt * 16;

  // the graph's CSR / reverse CSR of every mask, local offsets
#pragma unroll
  for (int j = 0; j < kGcMaxAdj; ++j) {
    if (j < a.nadj) {
      const GcAdj q = a.adj[j];
      const GcGraphAdj d = gc_adj(a, ADJ, j);
      int32_t* off = const_cast<int32_t*>(d.off);
      int32_t* nbr = const_cast<int32_t*>(d.nbr);
      int32_t* roff = const_cast<int32_t*>(d.roff);
      int32_t* rnbr = const_cast<int32_t*>(d.rnbr);
      const int e0 = q.off[base], r0 = q.roff[base];
      for (int t = tid; t <= n; t += kGcThreads) {
        off[t] = q.off[base + t] - e0;
        roff[t] = q.roff[base + t] - r0;
      }
      const int ne = q.off[base + n] - e0, nr = q.roff[base + n] - r0;
      for (int e = tid; e < ne; e += kGcThreads) nbr[e] = q.nbr[e0 + e];
      for (int e = tid; e < nr; e += kGcThreads) rnbr[e] = q.rnbr[r0 + e];
    }
  }
  // embedding bag of every node's sparse features (sum or mean)
  {
    float* x0 = reinterpret_cast<float*>(gc_smem + a.lds_x[0]);
    const int ld = a.ldx[0];
    for (int it = tid; it < nrow * D0; it += kGcThreads) {
      const int v = it / D0, c = it - v * D0;
      float acc = 0.f;
      if (v < n) {
        const int f0 = a.fo[base + v], f1 = a.fo[base + v + 1];
        for (int f = f0; f < f1; ++f) acc += a.table[static_cast<int64_t>(a.fid[f]) * D0 + c];
        if (a.mean_comb && f1 > f0) acc /= static_cast<float>(f1 - f0);
      }
      x0[v * ld + c] = acc;
    }
  }
  __syncthreads();

  // ---------------------------------------------------------------- forward
  for (int l = 0; l < L; ++l) {
    const int Din = gc_pick9(a.D, l), Dout = gc_pick9(a.D, l + 1);
    const int K = kind == 1 ? 2 * Din : Din;
    const float* X = reinterpret_cast<const float*>(gc_smem + gc_pick9(a.lds_x, l));
    float* Y = reinterpret_cast<float*>(gc_smem + gc_pick9(a.lds_x, l + 1));
    const GcGraphAdj q = gc_adj(a, ADJ, gc_pick(a.adj_of, l));
    const float* ep = gc_pick(a.eps, l);
    gc_aggregate(kind, selfl, X, gc_pick9(a.ldx, l), Din, Z, ldz, q, n, nrow, kind == 0 ? ep[0] : 0.f);
    __syncthreads();
    gc_fwd_gemm(Z, ldz, K, gc_pick(a.W, l), gc_pick(a.Wf, l), Din, kind == 1 ? gc_pick(a.bl, l) : nullptr, Dout, Y,
                gc_pick9(a.ldx, l + 1), n, nrt);
    __syncthreads();
  }

  // ---------------------------------------------------------------- pooled head
  // node_emb = fc(x_L); pooled = sum_v node_emb = Wfc (sum_v x_L[v]) + n bfc; logits = Wout pooled
  const int DL = gc_pick9(a.D, L), E = a.E, C = a.C;
  const float* XL = reinterpret_cast<const float*>(gc_smem + gc_pick9(a.lds_x, L));
  const int ldL = gc_pick9(a.ldx, L);
  float* sv = VEC;                      // [DL] column sums of x_L
  float* uv = sv + kGcMaxWidth;         // [DL] d(x_L[v]) (the same for every node)
  float* pv = uv + kGcMaxWidth;         // [E] pooled
  float* dp = pv + kGcMaxWidth;         // [E] d(pooled)
  float* dl = dp + kGcMaxWidth;         // [C] d(logits)
  float* lt = dl + kGcMaxLabels;        // [C] loss terms, then logits
  float* lg = lt + kGcMaxLabels;        // [C] logits
  for (int k = tid; k < DL; k += kGcThreads) {
    float s = 0.f;
    for (int v = 0; v < n; ++v) s += XL[v * ldL + k];
    sv[k] = s;
  }
  __syncthreads();
  for (int e = tid; e < E; e += kGcThreads) {
    float p = 0.f;
    const float* w = a.Wfc + static_cast<int64_t>(e) * DL;
    for (int k = 0; k < DL; ++k) p += w[k] * sv[k];
    pv[e] = p + static_cast<float>(n) * a.bfc[e];
  }
  __syncthreads();
  if (tid < C) {
    float x = 0.f;
    const float* w = a.Wout + static_cast<int64_t>(tid) * E;
    for (int e = 0; e < E; ++e) x += w[e] * pv[e];
    const float y = a.onehot[static_cast<int64_t>(g) * C + tid];
    lt[tid] = fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
    lg[tid] = x;
    dl[tid] = (1.f / (1.f + __expf(-x)) - y) * a.inv_scale;
  }
  __syncthreads();
  if (tid == 0) {
    float loss = 0.f;
    int am = 0, ay = 0;
    float best = lg[0], besty = a.onehot[static_cast<int64_t>(g) * C];
    for (int c = 0; c < C; ++c) {
      loss += lt[c];
      if (lg[c] > best) {
        best = lg[c];
        am = c;
      }
      const float yc = a.onehot[static_cast<int64_t>(g) * C + c];
      if (yc > besty) {
        besty = yc;
        ay = c;
      }
    }
    a.loss_part[b] = loss * a.inv_scale;
    a.acc_part[b] = am == ay ? 1.f : 0.f;
  }
  for (int it = tid; it < C * E; it += kGcThreads) {
    const int c = it / E, e = it - c * E;
    slab[a.o_out + it] = dl[c] * pv[e];
  }
  for (int e = tid; e < E; e += kGcThreads) {
    float s = 0.f;
    for (int c = 0; c < C; ++c) s += dl[c] * a.Wout[static_cast<int64_t>(c) * E + e];
    dp[e] = s;
  }
  __syncthreads();
  for (int it = tid; it < E * DL; it += kGcThreads) {
    const int e = it / DL, k = it - e * DL;
    slab[a.o_fc + it] = dp[e] * sv[k];
  }
  for (int e = tid; e < E; e += kGcThreads) slab[a.o_bfc + e] = static_cast<float>(n) * dp[e];
  for (int k = tid; k < DL; k += kGcThreads) {
    float s = 0.f;
    for (int e = 0; e < E; ++e) s += dp[e] * a.Wfc[static_cast<int64_t>(e) * DL + k];
    uv[k] = s;
  }
  __syncthreads();

  // ---------------------------------------------------------------- backward
  for (int l = L - 1; l >= 0; --l) {
    const int Din = gc_pick9(a.D, l), Dout = gc_pick9(a.D, l + 1);
    const int K = kind == 1 ? 2 * Din : Din;
    const float* X = reinterpret_cast<const float*>(gc_smem + gc_pick9(a.lds_x, l));
    const int ldx = gc_pick9(a.ldx, l);
    const float* Yo = reinterpret_cast<const float*>(gc_smem + gc_pick9(a.lds_x, l + 1));
    const int ldo = gc_pick9(a.ldx, l + 1);
    const GcGraphAdj q = gc_adj(a, ADJ, gc_pick(a.adj_of, l));
    const float* ep = gc_pick(a.eps, l);
    const float epsv = kind == 0 ? ep[0] : 0.f;
    // G = d(out) * relu'(out), in place in DY (the head's d(x_L) is one row for all nodes)
    for (int it = tid; it < nrow * Dout; it += kGcThreads) {
      const int v = it / Dout, o = it - v * Dout;
      const float d = l == L - 1 ? uv[o] : DY[v * ldy + o];
      DY[v * ldy + o] = (v < n && Yo[v * ldo + o] > 0.f) ? d : 0.f;
    }
    gc_aggregate(kind, selfl, X, ldx, Din, Z, ldz, q, n, nrow, epsv);  // Z of this conv again
    __syncthreads();
    const int64_t ow = gc_pick(a.o_W, l), owf = gc_pick(a.o_Wf, l);
    gc_bwd_gemms(DY, ldy, Z, ldz, K, gc_pick(a.W, l), gc_pick(a.Wf, l), Din, Dout, DZ, n, nrt, slab + ow,
                 slab + (owf >= 0 ? owf : 0));
    if (kind == 1) {  // liner bias
      const int64_t ob = gc_pick(a.o_bl, l);
      for (int o = tid; o < Dout; o += kGcThreads) {
        float s = 0.f;
        for (int v = 0; v < n; ++v) s += DY[v * ldy + o];
        slab[ob + o] = s;
      }
    }
    __syncthreads();
    // d(x_l) = the transposed aggregate of dZ (-> DY; G is dead); GIN: d(eps) = sum dZ . x
    float de = 0.f;
    for (int it = tid; it < nrow * Din; it += kGcThreads) {
      const int s = it / Din, c = it - s * Din;
      float v = 0.f;
      if (s < n) {
        const int e0 = q.roff[s], e1 = q.roff[s + 1];
        if (kind == 0) {
          const float dzs = DZ[s * ldz + c];
          v = (1.f + epsv) * dzs;
          float acc = 0.f;
          for (int e = e0; e < e1; ++e) acc += DZ[q.rnbr[e] * ldz + c];
          if (selfl) acc += dzs;
          v += acc;
          de += dzs * X[s * ldx + c];
        } else {
          v = DZ[s * ldz + c];
          float acc = 0.f;
          for (int e = e0; e < e1; ++e) {
            const int t = q.rnbr[e];
            acc += DZ[t * ldz + Din + c] / static_cast<float>(q.off[t + 1] - q.off[t] + selfl);
          }
          if (selfl) acc += DZ[s * ldz + Din + c] / static_cast<float>(q.off[s + 1] - q.off[s] + 1);
          v += acc;
        }
      }
      DY[s * ldy + c] = v;
    }
    const int64_t oe = gc_pick(a.o_eps, l);
    if (kind == 0 && oe >= 0) {
      const float tot = block_sum(de, s_red);
      if (tid == 0) slab[oe] = tot;
    }
    __syncthreads();
  }

  // ---------------------------------------------------------------- embedding table
  // column c of the table gradient is owned by one thread (deterministic order: nodes,
  // then their features)
  for (int c = tid; c < D0; c += kGcThreads) {
    for (int v = 0; v < n; ++v) {
      const int f0 = a.fo[base + v], f1 = a.fo[base + v + 1];
      if (f1 <= f0) continue;
      const float d = DY[v * ldy + c] * (a.mean_comb ? 1.f / static_cast<float>(f1 - f0) : 1.f);
      for (int f = f0; f < f1; ++f) TAB[a.fid[f] * D0 + c] += d;
    }
  }
  __syncthreads();
  for (int i = tid; i < tab_n; i += kGcThreads) slab[a.o_tab + i] = TAB[i];
}

// the B slab rows summed in block order; the flat optimizer on the sum (fuse_opt) or the
// flat gradient; block 0: loss, accuracy counters, the graph RNG's counter
__global__ __launch_bounds__(256) void gc_reduce_kernel(GcReduceArgs a) {
  const int tid = threadIdx.x;
  if (blockIdx.x == 0 && tid < 64) {
    float ls = 0.f, ac = 0.f;
    for (int b = tid; b < a.B; b += 64) {
      ls += a.loss_part[b];
      ac += a.acc_part[b];
    }
    ls = wave_sum(ls);
    ac = wave_sum(ac);
    if (tid == 0) {
      a.loss_out[0] = ls;
      a.right[0] += static_cast<double>(ac);
      a.right[1] += static_cast<double>(a.B);
      a.rng[1] += 1;
    }
  }
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + tid;
  if (i >= a.S) return;
  const float* src = a.slab + i;
  float g = 0.f;
  int b = 0;
  for (; b + 8 <= a.B; b += 8) {
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) v[u] = src[static_cast<int64_t>(b + u) * a.S];
#pragma unroll
    for (int u = 0; u < 8; ++u) g += v[u];
  }
  for (; b < a.B; ++b) g += src[static_cast<int64_t>(b) * a.S];
  if (a.fuse_opt) {
    float p = a.p[i], m = a.m[i], v = a.v[i];
    optim_one(p, g, m, v, static_cast<float>(a.ostep[0]), a.lr, a.b1, a.b2, a.eps, a.wd, a.grad_scale, a.okind);
    a.p[i] = p;
    a.m[i] = m;
    a.v[i] = v;
  } else {
    a.grad[i] = g;
  }
}

}  // namespace

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

hipError_t eh_gc_step(const GcStepArgs* a, hipStream_t s) {
  if (!a || a->L < 1 || a->L > kGcMaxLayers || a->B < 1 || a->G < 1 || a->nmax < 16 || a->nmax % 16 != 0 ||
      a->nmax > kGcMaxRows || a->nadj < 1 || a->nadj > kGcMaxAdj || a->E < 1 || a->E > kGcMaxWidth || a->C < 1 ||
      a->C > kGcMaxLabels || a->tab_rows * a->D[0] > kGcMaxTable || a->lds_bytes > 160 * 1024 || !a->gprob ||
      !a->galias || !a->rng || !a->gbase || !a->fo || !a->fid || !a->onehot || !a->table || !a->Wfc || !a->bfc ||
      !a->Wout || !a->slab || !a->loss_part || !a->acc_part || !a->gidx || (a->kind != 0 && a->kind != 1))
    return hipErrorInvalidValue;
  for (int l = 0; l <= a->L; ++l)
    if (a->D[l] < 16 || a->D[l] % 16 != 0 || a->D[l] > kGcMaxWidth) return hipErrorInvalidValue;
  for (int l = 0; l < a->L; ++l) {
    if (!a->W[l] || a->adj_of[l] < 0 || a->adj_of[l] >= a->nadj || a->o_W[l] < 0) return hipErrorInvalidValue;
    if (a->kind == 0 && !a->eps[l]) return hipErrorInvalidValue;
    if (a->kind == 1 && (!a->Wf[l] || !a->bl[l] || a->o_Wf[l] < 0 || a->o_bl[l] < 0)) return hipErrorInvalidValue;
  }
  const size_t lds = static_cast<size_t>(a->lds_bytes);
  if (lds > 65536)
    EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(gc_step_kernel),
                                        hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds)));
  hipLaunchKernelGGL(gc_step_kernel, dim3(static_cast<uint32_t>(a->B)), dim3(kGcThreads), lds, s, *a);
  return hipGetLastError();
}

hipError_t eh_gc_reduce(const GcReduceArgs* a, hipStream_t s) {
  if (!a || !a->slab || a->S < 1 || a->B < 1 || !a->loss_part || !a->acc_part || !a->loss_out || !a->right ||
      !a->rng || (!a->fuse_opt && !a->grad) || (a->fuse_opt && (!a->p || !a->m || !a->v || !a->ostep)))
    return hipErrorInvalidValue;
  hipLaunchKernelGGL(gc_reduce_kernel, dim3(static_cast<uint32_t>(ceil_div(a->S, 256))), dim3(256), 0, s, *a);
  return hipGetLastError();
}

}  // extern "C"
