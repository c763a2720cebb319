// Fused graph-classification training step (GIN / GraphGCN): see graph_cls_args.h for the
// launch sequence and the algebra, models/graph_cls_trainer.py for the model contract.
//
// One block (4 waves) per drawn graph; the graph (at most kGcMaxRows nodes) never leaves
// LDS.  Every product — embedding bag, aggregation, linear, their gradients — is a GEMM on
// the fp32-input MFMA (v_mfma_f32_16x16x4_f32: lane l supplies A[i = l & 15][k = l >> 4]
// and B[k = l >> 4][j = l & 15], C/D rows (l >> 4) * 4 + r, column l & 15) over 16 x 16
// output tiles dealt round-robin to the waves; activations, aggregates and gradients are
// LDS operands (rows padded by 4 floats), the weights come from L2 (each XCD's blocks warm
// it at the start; staging them in LDS measured slower).  The graph's sparse structure is
// densified once per step (A, S: n <= 64), so the aggregations are MFMA tiles instead of
// per-edge pointer chasing; the phases are separated by block barriers only.
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

// one 16 x 16 output tile, K-loop over kext (a multiple of 4): fa(k) / fb(k) give this
// lane's A[i][k] / B[k][j] for its (i, j) = (lane & 15, lane & 15) of the A row / B column
template <typename FA, typename FB>
__device__ __forceinline__ float4_t gc_tile(FA fa, FB fb, int kext) {
  const int lk = (threadIdx.x & 63) >> 4;
  float4_t acc = {0.f, 0.f, 0.f, 0.f};
  int k0 = 0;
  for (; k0 + 16 <= kext; k0 += 16) {
    float av[4], bv[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      av[u] = fa(k0 + 4 * u + lk);
      bv[u] = fb(k0 + 4 * u + lk);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) acc = mfma_f32x4(av[u], bv[u], acc);
  }
  for (; k0 < kext; k0 += 4) acc = mfma_f32x4(fa(k0 + lk), fb(k0 + lk), acc);
  return acc;
}

// out[i] = sum_k m(i, k) x(k) for i < N: a power-of-two group of lanes per output (within
// one wave), strided partial sums, butterfly reduction; fin(i, sum) on the group's lane 0
template <typename FM, typename FX, typename FIN>
__device__ __forceinline__ void gc_matvec(int N, int K, FM m, FX x, FIN fin) {
  int G = 1;
  while (G < 64 && 2 * G * N <= kGcThreads) G *= 2;
  const int i = threadIdx.x / G, part = threadIdx.x - i * G;
  float s = 0.f;
  if (i < N)
    for (int k = part; k < K; k += G) s += m(i, k) * x(k);
  for (int o = G >> 1; o >= 1; o >>= 1) s += __shfl_xor(s, o, 64);
  if (i < N && part == 0) fin(i, s);
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

// Z = the conv's aggregate of X (tiles over the rows < 16 nrt and the Din columns):
//   GIN        Z = A X + c X                      (c = 1 + eps + self loop)
//   GraphConv  Z = [X | (A X + self X) / cnt]
__device__ __forceinline__ void gc_agg(int kind, float c, int selfl, const float* A, int lda, const float* invc,
                                       const float* X, int ldx, int D, float* Z, int ldz, int nv, int nrt) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int nct = D >> 4;
  for (int tile = wave; tile < nrt * nct; tile += kGcThreads / 64) {
    const int rt = tile / nct, ct = tile - rt * nct;
    const int t0 = rt * 16, k = ct * 16 + lr;
    const float4_t acc = gc_tile([&](int s) { return A[(t0 + lr) * lda + s]; },
                                 [&](int s) { return X[s * ldx + k]; }, nv);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int t = t0 + lk * 4 + j;
      const float xt = X[t * ldx + k];
      if (kind == 0) {
        Z[t * ldz + k] = acc[j] + c * xt;
      } else {
        Z[t * ldz + k] = xt;
        Z[t * ldz + D + k] = (acc[j] + static_cast<float>(selfl) * xt) * invc[t];
      }
    }
  }
}

// Y = relu(Z [W | Wf]^T + bias) over rows < 16 nrt (rows >= n zeroed); csum (the last
// conv): each tile's column sums of Y at csum[row tile][column] (the pooled head's input)
__device__ __forceinline__ void gc_linear(const float* Z, int ldz, int K, const float* W, const float* Wf, int Din,
                                          int ldw, const float* __restrict__ bias, int Dout, float* Y, int ldy, int n,
                                          int nrt, float* csum) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int nct = Dout >> 4;
  for (int tile = wave; tile < nrt * nct; tile += kGcThreads / 64) {
    const int rt = tile / nct, ct = tile - rt * nct;
    const int r0 = rt * 16, o = ct * 16 + lr;
    const float* zr = Z + (r0 + lr) * ldz;
    const float* wr = W + o * ldw;
    const float* fr = Wf + o * ldw - Din;
    const float4_t acc = gc_tile([&](int k) { return zr[k]; }, [&](int k) { return k < Din ? wr[k] : fr[k]; }, K);
    const float bo = bias ? bias[o] : 0.f;
    float cs = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = r0 + lk * 4 + j;
      const float y = r < n ? fmaxf(acc[j] + bo, 0.f) : 0.f;
      Y[r * ldy + o] = y;
      cs += y;
    }
    if (csum) {  // the tile's 16 rows: the four lane groups of column o (fixed order)
      cs += __shfl_xor(cs, 16, 64);
      cs += __shfl_xor(cs, 32, 64);
      if (lk == 0) csum[rt * kGcMaxWidth + o] = cs;
    }
  }
}

// dW = G^T Z ([Dout][K] -> the slab: columns < Din at slab_w, the rest at slab_wf) and
// dZ = G [W | Wf] ([rows][K] -> LDS; GraphConv: the mean half pre-scaled by 1 / cnt of
// its row, the form the transposed aggregate consumes); G(v, o), rows >= n zero
template <typename FG>
__device__ __forceinline__ void gc_bwd(FG G, const float* Z, int ldz, int K, const float* W, const float* Wf, int Din,
                                       int ldw, int Dout, float* DZ, const float* invc, int kind, int nv, int nrt,
                                       float* slab_w, float* slab_wf) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  const int lr = lane & 15, lk = lane >> 4;
  const int nkt = K >> 4, ndw = (Dout >> 4) * nkt;
  for (int tile = wave; tile < ndw + nrt * nkt; tile += kGcThreads / 64) {
    if (tile < ndw) {
      const int ot = tile / nkt, kt = tile - ot * nkt;
      const int o0 = ot * 16, k = kt * 16 + lr;
      const float4_t acc = gc_tile([&](int v) { return G(v, o0 + lr); }, [&](int v) { return Z[v * ldz + k]; }, nv);
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
      const float* wc = k < Din ? W + k : Wf + (k - Din);
      const float4_t acc = gc_tile([&](int o) { return G(r0 + lr, o); }, [&](int o) { return wc[o * ldw]; }, Dout);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int r = r0 + lk * 4 + j;
        DZ[r * ldz + k] = (kind == 1 && k >= Din) ? acc[j] * invc[r] : acc[j];
      }
    }
  }
}

__global__ __launch_bounds__(kGcThreads) void gc_step_kernel(GcStepArgs a) {
  extern __shared__ __attribute__((aligned(16))) unsigned char gc_smem[];
  __shared__ int s_g;
  __shared__ float s_red[kGcThreads / 64];
  const int tid = threadIdx.x;
  const int b = blockIdx.x;
  const int L = a.L, kind = a.kind, selfl = a.self_loops, nmax = a.nmax;
  auto F = [&](int32_t off) { return reinterpret_cast<float*>(gc_smem + off); };
  float* DY = F(a.lds_dy);
  float* DZ = F(a.lds_dz);
  float* VEC = F(a.lds_vec);
  float* Sm = F(a.lds_s);
  float* Tt = F(a.lds_t);
  const int ldz = a.ldz, ldy = a.ldy, lda = a.lda, ldsm = a.ldsm, ldt = a.ldt;
  float* slab = a.slab + static_cast<int64_t>(b) * a.S;
  int nst = 0;
#define GC_STAMP() \
  if (a.prof && tid == 0 && nst < 32) a.prof[b * 32 + nst++] = static_cast<long long>(wall_clock64())
  GC_STAMP();

  // ---------------------------------------------------------------- P0: draw, staging
  // the graph: uniform draw through the alias table, Philox stream 3 at counter + 1 (the
  // generic step's advance-then-alias_sample); the reduce launch advances the counter
  __shared__ int s_rec[kGcRec];
  if (tid == 0) {
    const uint4_t r = Philox::gen(static_cast<uint64_t>(a.rng[0]), (static_cast<uint64_t>(a.rng[1] + 1) << 8) ^ 3ull,
                                  static_cast<uint64_t>(b));
    const uint64_t x = (static_cast<uint64_t>(r[0]) << 32) | r[1];
    int64_t k = static_cast<int64_t>(__umul64hi(x, static_cast<uint64_t>(a.G)));
    if (k >= a.G) k = a.G - 1;
    const int g = (u01(r[2]) < a.gprob[k]) ? static_cast<int>(k) : a.galias[k];
    s_g = g;
    a.gidx[b] = g;
    if (b == 0 && a.ostep_inc) a.ostep_inc[0] += 1;  // read by this step's reduce launch
#pragma unroll
    for (int q = 0; q < kGcRec; ++q) s_rec[q] = a.rec[static_cast<int64_t>(g) * kGcRec + q];
    for (int c = 0; c < a.C; ++c) VEC[5 * kGcMaxWidth + 3 * kGcMaxLabels + c] = a.onehot[static_cast<int64_t>(g) * a.C + c];
  }
  // the head's fc bias (read after many barriers)
  for (int e = tid; e < a.E; e += kGcThreads) VEC[4 * kGcMaxWidth + 3 * kGcMaxLabels + e] = a.bfc[e];
  const int D0 = a.D[0];
  // warm this XCD's L2 with the parameters the reduce launch just rewrote (from another
  // XCD's L2): the blocks of one XCD (b, b + 8, ...) each touch every 8th 128-byte line, so
  // the GEMMs' weight operands below hit in L2; nothing waits on these loads but the draw's
  float warm = 0.f;
  {
    const int64_t lines = (a.warm_n + 31) / 32;
    for (int64_t q = (b >> 3) + 8 * static_cast<int64_t>(tid); q < lines; q += 8 * kGcThreads) warm += a.warm[q * 32];
  }
  // the table, padding rows zero (S has zero columns there)
  for (int i = tid; i < a.trp * D0; i += kGcThreads) {
    const int r = i / D0, c = i - r * D0;
    Tt[r * ldt + c] = r < a.tab_rows ? a.table[i] : 0.f;
  }
  // A, the in-degrees (later 1 / cnt) and S start from zero
  {
    float* A = F(a.lds_a);
    for (int i = tid; i < a.nadj * nmax * lda; i += kGcThreads) A[i] = 0.f;
    float* ic = F(a.lds_invc);
    for (int i = tid; i < a.nadj * nmax; i += kGcThreads) ic[i] = 0.f;
    for (int i = tid; i < nmax * ldsm; i += kGcThreads) Sm[i] = 0.f;
  }
  __syncthreads();
  GC_STAMP();
  const int g = s_g, n = s_rec[0];
  const int nrt = (n + 15) >> 4, nv = (n + 3) & ~3;

  // ---------------------------------------------------------------- P1: densify the graph
  // A_j[t][s] += 1 per edge t <- s, deg_j[t] += 1; S[v][r] += bag weight per feature
  // occurrence (LDS float atomics of integers / equal weights: exact in any order)
#pragma unroll
  for (int j = 0; j < kGcMaxAdj; ++j) {
    if (j < a.nadj) {
      const int32_t* pr = a.adj[j].pair;
      float* A = F(a.lds_a) + j * nmax * lda;
      float* dg = F(a.lds_invc) + j * nmax;
      for (int e = s_rec[3 + 2 * j] + tid; e < s_rec[4 + 2 * j]; e += kGcThreads) {
        const int p = pr[e];
        const int t = p >> 8, sidx = p & 255;
        atomicAdd(A + t * lda + sidx, 1.f);
        atomicAdd(dg + t, 1.f);
      }
    }
  }
  for (int f = s_rec[1] + tid; f < s_rec[2]; f += kGcThreads) {
    const int p = a.fpair[f];
    atomicAdd(Sm + (p >> 16) * ldsm + (p & 0xffff), a.fw[f]);
  }

  __syncthreads();
  GC_STAMP();
  // 1 / cnt (GraphConv mean: in-degree + self loop; 0 for padding rows)
  for (int i = tid; i < a.nadj * nmax; i += kGcThreads) {
    float* ic = F(a.lds_invc);
    const int t = i % nmax;
    const float cnt = ic[i] + static_cast<float>(selfl);
    ic[i] = (t < n && cnt > 0.f) ? 1.f / cnt : 0.f;
  }
  // X0 = S T (the embedding bag)
  {
    float* X0 = F(a.lds_x[0]);
    const int ld0 = a.ldx[0];
    const int lane = tid & 63, wave = tid >> 6, lr = lane & 15, lk = lane >> 4;
    const int nct = D0 >> 4;
    for (int tile = wave; tile < nrt * nct; tile += kGcThreads / 64) {
      const int rt = tile / nct, ct = tile - rt * nct;
      const int v0 = rt * 16, c = ct * 16 + lr;
      const float4_t acc = gc_tile([&](int r) { return Sm[(v0 + lr) * ldsm + r]; },
                                   [&](int r) { return Tt[r * ldt + c]; }, a.trp);
#pragma unroll
      for (int j = 0; j < 4; ++j) X0[(v0 + lk * 4 + j) * ld0 + c] = acc[j];
    }
  }
  __syncthreads();
  GC_STAMP();

  // ---------------------------------------------------------------- forward
  for (int l = 0; l < L; ++l) {
    const int Din = gc_pick9(a.D, l), Dout = gc_pick9(a.D, l + 1);
    const int K = kind == 1 ? 2 * Din : Din;
    const float* X = F(gc_pick9(a.lds_x, l));
    float* Z = F(a.lds_z) + (a.zst ? l * nmax * ldz : 0);
    const int j = gc_pick(a.adj_of, l);
    const float epsv = kind == 0 ? gc_pick(a.eps, l)[0] : 0.f;
    gc_agg(kind, 1.f + epsv + static_cast<float>(selfl), selfl, F(a.lds_a) + j * nmax * lda, lda,
           F(a.lds_invc) + j * nmax, X, gc_pick9(a.ldx, l), Din, Z, ldz, nv, nrt);
    __syncthreads();
    GC_STAMP();
    gc_linear(Z, ldz, K, gc_pick(a.W, l), gc_pick(a.Wf, l), Din, Din, kind == 1 ? gc_pick(a.bl, l) : nullptr, Dout,
              F(gc_pick9(a.lds_x, l + 1)), gc_pick9(a.ldx, l + 1), n, nrt, l == L - 1 ? F(a.lds_csum) : nullptr);
    __syncthreads();
    GC_STAMP();
  }

  // ---------------------------------------------------------------- pooled head
  // node_emb = fc(x_L); pooled = sum_v node_emb = Wfc (sum_v x_L[v]) + n bfc; logits = Wout pooled
  const int DL = gc_pick9(a.D, L), E = a.E, C = a.C;
  const float* XL = F(gc_pick9(a.lds_x, L));
  const int ldL = gc_pick9(a.ldx, L);
  const float* Wfc = a.Wfc;
  const float* Wout = a.Wout;
  const int ldfc = DL, ldout = E;
  float* sv = VEC;                      // [DL] column sums of x_L
  float* uv = sv + kGcMaxWidth;         // [DL] d(x_L[v]) (the same for every node)
  float* pv = uv + kGcMaxWidth;         // [E] pooled
  float* dp = pv + kGcMaxWidth;         // [E] d(pooled)
  float* dl = dp + kGcMaxWidth;         // [C] d(logits)
  float* lt = dl + kGcMaxLabels;        // [C] loss terms
  float* lg = lt + kGcMaxLabels;        // [C] logits
  const float fn = static_cast<float>(n);
  const float* csum = F(a.lds_csum);
  auto colsum = [&](int k) {  // sum_v x_L[v][k] from the last conv's tile partials
    float s = 0.f;
    for (int rt = 0; rt < nrt; ++rt) s += csum[rt * kGcMaxWidth + k];
    return s;
  };
  for (int k = tid; k < DL; k += kGcThreads) sv[k] = colsum(k);
  const float* hb = VEC + 4 * kGcMaxWidth + 3 * kGcMaxLabels;  // fc bias, label row (staged in P0)
  gc_matvec(E, DL, [&](int e, int k) { return Wfc[e * ldfc + k]; }, colsum,
            [&](int e, float s) { pv[e] = s + fn * hb[e]; });
  __syncthreads();
  const float* yrow = hb + kGcMaxWidth;
  gc_matvec(C, E, [&](int c, int e) { return Wout[c * ldout + e]; }, [&](int e) { return pv[e]; },
            [&](int c, float x) {
              const float y = yrow[c];
              lt[c] = fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
              lg[c] = x;
              dl[c] = (1.f / (1.f + __expf(-x)) - y) * a.inv_scale;
            });
  __syncthreads();
  if (tid == 0) {
    float loss = 0.f;
    int am = 0, ay = 0;
    float best = lg[0], besty = yrow[0];
    for (int c = 0; c < C; ++c) {
      loss += lt[c];
      if (lg[c] > best) {
        best = lg[c];
        am = c;
      }
      if (yrow[c] > besty) {
        besty = yrow[c];
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
  gc_matvec(E, C, [&](int e, int c) { return Wout[c * ldout + e]; }, [&](int c) { return dl[c]; },
            [&](int e, float s) { dp[e] = s; });
  __syncthreads();
  for (int it = tid; it < E * DL; it += kGcThreads) {
    const int e = it / DL, k = it - e * DL;
    slab[a.o_fc + it] = dp[e] * sv[k];
  }
  for (int e = tid; e < E; e += kGcThreads) slab[a.o_bfc + e] = fn * dp[e];
  gc_matvec(DL, E, [&](int k, int e) { return Wfc[e * ldfc + k]; }, [&](int e) { return dp[e]; },
            [&](int k, float s) { uv[k] = s; });
  __syncthreads();
  GC_STAMP();

  // ---------------------------------------------------------------- backward
  for (int l = L - 1; l >= 0; --l) {
    const int Din = gc_pick9(a.D, l), Dout = gc_pick9(a.D, l + 1);
    const int K = kind == 1 ? 2 * Din : Din;
    const float* X = F(gc_pick9(a.lds_x, l));
    const int ldx = gc_pick9(a.ldx, l);
    float* Z = F(a.lds_z) + (a.zst ? l * nmax * ldz : 0);
    const int j = gc_pick(a.adj_of, l);
    const float* A = F(a.lds_a) + j * nmax * lda;
    const float* invc = F(a.lds_invc) + j * nmax;
    const float epsv = kind == 0 ? gc_pick(a.eps, l)[0] : 0.f;
    const float cdiag = 1.f + epsv + static_cast<float>(selfl);
    if (!a.zst) {  // Z of this conv again (only one Z buffer fits)
      gc_agg(kind, cdiag, selfl, A, lda, invc, X, ldx, Din, Z, ldz, nv, nrt);
      __syncthreads();
    }
    const float* Wl = gc_pick(a.W, l);
    const float* Wfl = gc_pick(a.Wf, l);
    const int64_t ow = gc_pick(a.o_W, l), owf = gc_pick(a.o_Wf, l);
    // G: the last conv's is d(x_L) (one row uv for every node) through its ReLU, formed on
    // the fly; the others were written by the conv above (two instantiations)
    auto grads = [&](auto G) {
      gc_bwd(G, Z, ldz, K, Wl, Wfl, Din, Din, Dout, DZ, invc, kind, nv, nrt, slab + ow,
             slab + (owf >= 0 ? owf : 0));
      if (kind == 1) {  // liner bias: column sums of G
        const int64_t ob = gc_pick(a.o_bl, l);
        gc_matvec(Dout, n, [&](int o, int v) { return G(v, o); }, [](int) { return 1.f; },
                  [&](int o, float s) { slab[ob + o] = s; });
      }
    };
    if (l == L - 1) grads([&](int v, int o) { return XL[v * ldL + o] > 0.f ? uv[o] : 0.f; });
    else grads([&](int v, int o) { return DY[v * ldy + o]; });
    __syncthreads();
    GC_STAMP();
    // d(x_l) = A^T dZ' + diagonal terms; below the first conv it is G of the conv below
    // (masked by that conv's ReLU), at l == 0 the input of the table gradient
    {
      const int lane = tid & 63, wave = tid >> 6, lr = lane & 15, lk = lane >> 4;
      const int nct = Din >> 4, zc = kind == 1 ? Din : 0;
      for (int tile = wave; tile < nrt * nct; tile += kGcThreads / 64) {
        const int rt = tile / nct, ct = tile - rt * nct;
        const int s0 = rt * 16, k = ct * 16 + lr;
        const float4_t acc = gc_tile([&](int t) { return A[t * lda + s0 + lr]; },
                                     [&](int t) { return DZ[t * ldz + zc + k]; }, nv);
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) {
          const int s = s0 + lk * 4 + jj;
          const float v = kind == 0 ? acc[jj] + cdiag * DZ[s * ldz + k]
                                    : DZ[s * ldz + k] + acc[jj] + static_cast<float>(selfl) * DZ[s * ldz + Din + k];
          DY[s * ldy + k] = (s < n && (l == 0 || X[s * ldx + k] > 0.f)) ? v : 0.f;
        }
      }
    }
    const int64_t oe = gc_pick(a.o_eps, l);
    if (kind == 0 && oe >= 0) {  // d(eps) = sum dZ . x
      float de = 0.f;
      for (int it = tid; it < n * Din; it += kGcThreads) {
        const int s = it / Din, c = it - s * Din;
        de += DZ[s * ldz + c] * X[s * ldx + c];
      }
      const float tot = block_sum(de, s_red);
      if (tid == 0) slab[oe] = tot;
    }
    __syncthreads();
    GC_STAMP();
  }

  // ---------------------------------------------------------------- embedding table
  // d(T) = S^T d(x_0): every element written once (padding rows skipped)
  {
    const int lane = tid & 63, wave = tid >> 6, lr = lane & 15, lk = lane >> 4;
    const int nct = D0 >> 4, nrt_t = a.trp >> 4;
    for (int tile = wave; tile < nrt_t * nct; tile += kGcThreads / 64) {
      const int rt = tile / nct, ct = tile - rt * nct;
      const int r0 = rt * 16, c = ct * 16 + lr;
      const float4_t acc = gc_tile([&](int v) { return Sm[v * ldsm + r0 + lr]; },
                                   [&](int v) { return DY[v * ldy + c]; }, nv);
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) {
        const int r = r0 + lk * 4 + jj;
        if (r < a.tab_rows) slab[a.o_tab + static_cast<int64_t>(r) * D0 + c] = acc[jj];
      }
    }
  }
  GC_STAMP();
  if (warm == 1.2345e-37f && tid == kGcThreads) slab[0] = warm;  // keeps the warming loads (never true)
#undef GC_STAMP
}

// the B slab rows summed in block order; the flat optimizer on the sum (fuse_opt) or the
// flat gradient; block 0: loss, accuracy counters, the graph RNG's counter
__global__ __launch_bounds__(256) void gc_reduce_kernel(GcReduceArgs a) {
  __shared__ float part[4][64];
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
  // 64 elements per block, wave q sums slab rows q, q + 4, ... (16 loads in flight), the
  // four partial sums then added in wave order (deterministic)
  const int q = tid >> 6, e = tid & 63;
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 64 + e;
  const bool in = i < a.S;
  const float* src = a.slab + (in ? i : 0);
  // the optimizer slots first: independent of the slab sum, their latency overlaps it
  float p = 0.f, m = 0.f, v = 0.f;
  if (a.fuse_opt && q == 0 && in) {
    p = a.p[i];
    m = a.m[i];
    v = a.v[i];
  }
  float g = 0.f;
  for (int b0 = q; b0 < a.B; b0 += 64) {
    float x[16];
#pragma unroll
    for (int u = 0; u < 16; ++u) {
      const int b = b0 + 4 * u;
      x[u] = b < a.B ? src[static_cast<int64_t>(b) * a.S] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 16; ++u) g += x[u];
  }
  part[q][e] = g;
  __syncthreads();
  if (q != 0 || !in) return;
  g = part[0][e] + part[1][e] + part[2][e] + part[3][e];
  if (a.fuse_opt) {
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
      a->C > kGcMaxLabels || a->tab_rows < 1 || a->tab_rows > kGcMaxTableRows || a->trp % 16 != 0 ||
      a->trp < a->tab_rows || a->tab_rows * a->D[0] > kGcMaxTable || a->lds_bytes > 160 * 1024 || !a->gprob ||
      !a->galias || !a->rng || !a->rec || !a->fpair || !a->fw || !a->onehot || !a->table || !a->Wfc || !a->bfc ||
      !a->Wout || !a->slab || !a->loss_part || !a->acc_part || !a->gidx || !a->warm || a->warm_n < 1 ||
      (a->kind != 0 && a->kind != 1))
    return hipErrorInvalidValue;
  for (int l = 0; l <= a->L; ++l)
    if (a->D[l] < 16 || a->D[l] % 16 != 0 || a->D[l] > kGcMaxWidth) return hipErrorInvalidValue;
  for (int l = 0; l < a->L; ++l) {
    if (!a->W[l] || a->adj_of[l] < 0 || a->adj_of[l] >= a->nadj || a->o_W[l] < 0) return hipErrorInvalidValue;
    if (a->kind == 0 && !a->eps[l]) return hipErrorInvalidValue;
    if (a->kind == 1 && (!a->Wf[l] || !a->bl[l] || a->o_Wf[l] < 0 || a->o_bl[l] < 0)) return hipErrorInvalidValue;
  }
  for (int j = 0; j < a->nadj; ++j)
    if (!a->adj[j].pair) return hipErrorInvalidValue;
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
  hipLaunchKernelGGL(gc_reduce_kernel, dim3(static_cast<uint32_t>(ceil_div(a->S, 64))), dim3(256), 0, s, *a);
  return hipGetLastError();
}

}  // extern "C"
