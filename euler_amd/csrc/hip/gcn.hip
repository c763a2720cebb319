// Fused GCN training step on gfx950 (see gcn_args.h for the launch sequence) — the kernels
// behind euler_amd.models.gcn_trainer.GcnTrainer, which NodeEstimator(device_graph=True)
// runs for SupervisedGCN-shaped models.
//
// Reference semantics: tf_euler/python/dataflow/gcn_dataflow.py:26-48 (full neighbourhoods,
// unique per hop, self loops), tf_euler/python/convolution/gcn_conv.py:26-54 (symmetric
// deg^-1/2 normalisation over the block's own edge list), mp_utils/base.py:24-47 (fc, out_fc,
// sigmoid cross-entropy on dense labels).
//
// Design notes (MI355X):
//  * node sets without sorting or clearing: one returning atomicAdd per edge on a per-node
//    counter (random-address device atomics cost one memory-side request each, ~20-30 G/s
//    chip-wide, so the flow spends exactly one per edge): the edge that sees 0 claims the
//    node — its set position when unplaced, and later its final count (the GCN source
//    degree, one atomic per distinct source) and the counter's reset; positions live in a
//    per-node (epoch, position) table, so a new epoch per step makes older entries stale;
//  * prefix sums inside the producing launch: a decoupled look-back over 8-byte
//    {tag, flag, value} granules written with relaxed agent-scope atomics (the data is the
//    flag: no fences), tagged with the step epoch so no status word is ever cleared;
//  * aggregation is edge-parallel: each worker (one lane per 8 columns) walks a contiguous
//    slice of its tile's edge list with 8 rows in flight and flushes a running sum to an LDS
//    accumulator when the target changes, so a hub's edges spread over every worker of
//    the block instead of serialising one thread;
//  * every GEMM is bf16 MFMA (16x16x32) on LDS images; k-major products (A^T B: the weight
//    gradients, and the backward through a weight stored [out][in]) read the image rows
//    with the transposing ds_read_b64_tr_b16 (tile.h tl_tr_frag), the other operand with
//    the same k permutation, so no transposed copy of any weight or activation exists;
//  * the whole row-local part of the backward (loss, d logits, d emb, d h, d aggregate) runs
//    in the head launch, which writes d(agg) of the roots; the ReLU mask of h1 is per source
//    row, so d(W0) is linear over hop 0's edges and the dW launch runs its GEMM over those
//    edges directly: d(h1) is never formed (no scatter, no atomics, nothing to clear).
#include <hip/hip_runtime.h>

#include "hip/gcn_args.h"
#include "hip/sampling_math.h"
#include "hip/optim_math.h"
#include "hip/tile.h"

namespace euler_hip {

// ----------------------------------------------------------------------------
// look-back scan (R2 granules: {tag:24 | flag:2 | value:38}, relaxed agent-scope atomics)
// ----------------------------------------------------------------------------
constexpr uint64_t kLbAgg = 1, kLbPre = 2;
constexpr uint64_t kLbMask = (uint64_t{1} << 38) - 1;

__device__ __forceinline__ uint64_t lb_word(uint32_t tag, uint64_t flag, int64_t v) {
  return (static_cast<uint64_t>(tag & 0xFFFFFFu) << 40) | (flag << 38) | (static_cast<uint64_t>(v) & kLbMask);
}

__device__ __forceinline__ void lb_store(uint64_t* p, uint64_t w) {
  __hip_atomic_store(p, w, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Exclusive prefix of block b's aggregate over blocks 0..b-1.  Called by every lane of wave
// 0 (the result is returned on every lane).  Each wave-pass reads the 64 nearest
// predecessors at once, waits until all are published, adds up to and including the
// closest inclusive prefix.  Bounded: a wait longer than ~0.2 s sets err bit 1 and gives up
// (the step's overflow / error word makes the caller discard the batch).
__device__ int64_t lb_prefix(uint64_t* st, int b, int64_t agg, uint32_t tag, int* err) {
  const int lane = threadIdx.x & 63;
  const uint32_t t24 = tag & 0xFFFFFFu;
  if (b == 0) {
    if (lane == 0) lb_store(&st[0], lb_word(tag, kLbPre, agg));
    return 0;
  }
  if (lane == 0) lb_store(&st[b], lb_word(tag, kLbAgg, agg));
  int64_t excl = 0;
  int base = b - 1;
  const long long t0 = wall_clock64();
  while (base >= 0) {
    const int j = base - lane;
    uint64_t w = 0;
    bool ready = false;
    while (true) {
      if (j >= 0) {
        w = __hip_atomic_load(&st[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        ready = (static_cast<uint32_t>(w >> 40) == t24) && ((w >> 38) & 3u) != 0;
      } else {
        w = lb_word(tag, kLbPre, 0);
        ready = true;
      }
      if (__all(ready)) break;
      if (wall_clock64() - t0 > 20000000ll) {  // 100 MHz clock: 0.2 s
        if (lane == 0) atomicOr(err, 2);
        return excl;
      }
      __builtin_amdgcn_s_sleep(1);
    }
    const bool pre = ((w >> 38) & 3u) == kLbPre;
    const uint64_t pm = __ballot(pre);
    const int first = pm ? __ffsll(static_cast<long long>(pm)) - 1 : 64;
    int64_t v = lane <= first ? static_cast<int64_t>(w & kLbMask) : 0;
#pragma unroll
    for (int o = 32; o >= 1; o >>= 1) v += __shfl_xor(v, o, 64);
    excl += v;
    if (pm) break;
    base -= 64;
  }
  if (lane == 0) lb_store(&st[b], lb_word(tag, kLbPre, excl + agg));
  return excl;
}

// inclusive block scan of one int per thread (256 threads); returns the inclusive value,
// *total = the block sum
__device__ __forceinline__ int block_scan_incl(int x, int* lds4, int* total) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  int v = x;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(v, o, 64);
    if (lane >= o) v += y;
  }
  if (lane == 63) lds4[wave] = v;
  __syncthreads();
  int add = 0;
  for (int w = 0; w < wave; ++w) add += lds4[w];
  *total = lds4[0] + lds4[1] + lds4[2] + lds4[3];
  __syncthreads();
  return v + add;
}

__device__ __forceinline__ uint64_t gcn_key(int32_t stamp, int h, int64_t occ) {
  const uint32_t hi = 0xFFFFFFFFu - (static_cast<uint32_t>(stamp) * 4u + static_cast<uint32_t>(h));
  return (static_cast<uint64_t>(hi) << 32) | static_cast<uint32_t>(occ);
}

__device__ __forceinline__ int masked_degree(const GcnGraph& g, int32_t row, uint32_t mask, int64_t* start,
                                             bool* contiguous) {
  const int64_t base = static_cast<int64_t>(row) * g.num_types;
  const uint32_t all = g.num_types >= 32 ? 0xFFFFFFFFu : ((1u << g.num_types) - 1u);
  if ((mask & all) == all) {
    *start = g.indptr[base];
    *contiguous = true;
    return static_cast<int>(g.indptr[base + g.num_types] - *start);
  }
  *contiguous = false;
  *start = 0;
  int d = 0;
  for (int t = 0; t < g.num_types; ++t)
    if ((mask >> t) & 1u) d += static_cast<int>(g.indptr[base + t + 1] - g.indptr[base + t]);
  return d;
}

// the k-th masked neighbour of row (segments in ascending type order)
__device__ __forceinline__ int32_t masked_nbr(const GcnGraph& g, int32_t row, uint32_t mask, int k) {
  const int64_t base = static_cast<int64_t>(row) * g.num_types;
  for (int t = 0; t < g.num_types; ++t) {
    if (!((mask >> t) & 1u)) continue;
    const int64_t a = g.indptr[base + t], n = g.indptr[base + t + 1] - a;
    if (k < n) return g.nbr[a + k];
    k -= static_cast<int>(n);
  }
  return -1;
}

// ----------------------------------------------------------------------------
// expand: targets' degrees -> offsets (look-back) -> edge list + first-occurrence claims.
// te = gcn_expand_tile(cap_t) <= kGcnExpandT targets per block (small hops get small tiles,
// so a hop of a few hundred targets still spreads over ~128 blocks and its hubs' edge
// lists over many CUs); the block's edges are spread over all 256 threads, 8 per
// thread per pass with every load of a pass in flight.  Hop 0's launch also carries the
// weight-staging blocks (GcnHop.st: fp32 masters -> padded bf16 images for the layer and
// head launches, which then copy them to LDS with 16-byte loads).
// ----------------------------------------------------------------------------
__device__ void gcn_stage_blocks(const GcnHop& a, int sb, int nsb) {
  for (int k = 0; k < a.nst; ++k) {
    const GcnStageW& w = a.st[k];
    const int64_t n = static_cast<int64_t>(w.rowsp) * (w.ld >> 1);
    for (int64_t i = static_cast<int64_t>(sb) * 256 + threadIdx.x; i < n; i += static_cast<int64_t>(nsb) * 256) {
      const int r = static_cast<int>(i / (w.ld >> 1)), c = static_cast<int>(i - static_cast<int64_t>(r) * (w.ld >> 1)) * 2;
      const float x = (r < w.rows && c < w.cols) ? w.w[static_cast<int64_t>(r) * w.cols + c] : 0.f;
      const float y = (r < w.rows && c + 1 < w.cols) ? w.w[static_cast<int64_t>(r) * w.cols + c + 1] : 0.f;
      reinterpret_cast<uint32_t*>(w.img)[i] = pack_bf16x2(x, y);
    }
  }
}

// alias draw of sampling.hip alias_sample_kernel (Philox (rng0, rng1 << 8 ^ stream, i))
__device__ __forceinline__ int32_t gcn_alias_draw(const float* prob, const int32_t* alias, const int32_t* rows,
                                                  int64_t pop, const int64_t* rng, uint64_t stream, int64_t i) {
  const uint4_t r = Philox::gen(static_cast<uint64_t>(rng[0]), (static_cast<uint64_t>(rng[1]) << 8) ^ stream,
                                static_cast<uint64_t>(i));
  const uint64_t x = (static_cast<uint64_t>(r[0]) << 32) | r[1];
  int64_t k = static_cast<int64_t>(__umul64hi(x, static_cast<uint64_t>(pop)));
  if (k >= pop) k = pop - 1;
  const int64_t pick = (u01(r[2]) < prob[k]) ? k : static_cast<int64_t>(alias[k]);
  return rows ? rows[pick] : static_cast<int32_t>(pick);
}

// AdaptiveGCN's layer (GcnLayerDraw kind 1): one block
__device__ void gcn_layerwise_draw(const GcnLayerDraw& a) {
  __shared__ double cum[kGcnLayerMaxRoots];
  __shared__ double s_tot[4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int B = a.B;
  const int per = (B + 255) / 256;  // consecutive roots per thread (scan order = root order)
  double run = 0.0;
  for (int j = 0; j < per; ++j) {
    const int i = tid * per + j;
    if (i >= B) break;
    const int32_t row = gcn_alias_draw(a.prob, a.alias, a.root_rows, a.pop, a.rng, 1ull, i);
    a.roots[i] = row;
    // out-weight under the mask: the types' segment totals in type order (float, as the
    // generic _out_weight)
    float w = 0.f;
    if (row >= 0 && row < a.g.num_rows) {
      const int64_t base = static_cast<int64_t>(row) * a.g.num_types;
      for (int t = 0; t < a.g.num_types; ++t) {
        if (!((a.mask >> t) & 1u)) continue;
        const int64_t lo = a.g.indptr[base + t], hi = a.g.indptr[base + t + 1];
        w = w + (hi > lo ? a.g.cumw[hi - 1] : 0.f);
      }
    }
    run += static_cast<double>(w);
    cum[i] = run;  // thread-local inclusive prefix, offset below
  }
  // exclusive offsets of the threads' runs (doubles of float weights: exact sums)
  double incl = run;
  for (int o = 1; o < 64; o <<= 1) {
    const double v = __shfl_up(incl, o, 64);
    if (lane >= o) incl += v;
  }
  if (lane == 63) s_tot[wave] = incl;
  __syncthreads();
  double woff = 0.0;
  for (int w2 = 0; w2 < wave; ++w2) woff += s_tot[w2];
  const double off = woff + incl - run;
  for (int j = 0; j < per; ++j) {
    const int i = tid * per + j;
    if (i < B) cum[i] += off;
  }
  __syncthreads();
  const double total = cum[B - 1];
  for (int64_t m = tid; m < a.count; m += 256) {
    int32_t root = -1;
    if (total > 0.0) {
      // the generic _uniform: two 16-bit draws of a flat 65536-entry alias table
      const uint4_t rh = Philox::gen(static_cast<uint64_t>(a.rng[0]),
                                     (static_cast<uint64_t>(a.rng[1]) << 8) ^ a.stream_u, static_cast<uint64_t>(m));
      const uint4_t rl = Philox::gen(static_cast<uint64_t>(a.rng[0]),
                                     (static_cast<uint64_t>(a.rng[1]) << 8) ^ (a.stream_u + 100), static_cast<uint64_t>(m));
      const uint64_t xh = (static_cast<uint64_t>(rh[0]) << 32) | rh[1];
      const uint64_t xl = (static_cast<uint64_t>(rl[0]) << 32) | rl[1];
      const double hi = static_cast<double>(__umul64hi(xh, 65536ull)), lo = static_cast<double>(__umul64hi(xl, 65536ull));
      const double u = (hi * 65536.0 + lo + 0.5) / 4294967296.0 * total;
      int a0 = 0, b0 = B;  // first index with cum > u (searchsorted right), clamped
      while (a0 < b0) {
        const int mid = (a0 + b0) >> 1;
        if (cum[mid] > u) b0 = mid;
        else a0 = mid + 1;
      }
      root = a.roots[a0 < B ? a0 : B - 1];
    }
    int32_t v = -1;
    if (root >= 0 && root < a.g.num_rows) {
      const uint4_t r = Philox::gen(static_cast<uint64_t>(a.rng[0]), (static_cast<uint64_t>(a.rng[1]) << 8) ^ a.stream,
                                    static_cast<uint64_t>(m));
      v = sample_one_neighbor(a.g.indptr, a.g.nbr, a.g.cumw, a.g.num_types, a.mask, root, r, -1, nullptr, nullptr);
    }
    if (v >= 0) a.lflag[v] = a.stamp[0];
  }
}

// stamp this step's layer (GcnLayerDraw); a row drawn twice is stamped twice
__global__ __launch_bounds__(256) void gcn_layer_draw_kernel(GcnLayerDraw a) {
  if (a.kind == 1) {
    gcn_layerwise_draw(a);
    return;
  }
  const int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x;
  if (i >= a.count) return;
  const uint4_t r = Philox::gen(static_cast<uint64_t>(a.rng[0]), (static_cast<uint64_t>(a.rng[1]) << 8) ^ a.stream,
                                static_cast<uint64_t>(i));
  const uint64_t x = (static_cast<uint64_t>(r[0]) << 32) | r[1];
  int64_t k = static_cast<int64_t>(__umul64hi(x, static_cast<uint64_t>(a.pop)));
  if (k >= a.pop) k = a.pop - 1;
  const int64_t pick = (u01(r[2]) < a.prob[k]) ? k : static_cast<int64_t>(a.alias[k]);
  const int32_t row = a.root_rows ? a.root_rows[pick] : static_cast<int32_t>(pick);
  if (row >= 0) a.lflag[row] = a.stamp[0];
}

__global__ __launch_bounds__(256) void gcn_expand_kernel(GcnHop a) {
  const int TE = gcn_expand_tile(a.cap_t);
  const int nexp = static_cast<int>(ceil_div(a.cap_t, TE));
  if (static_cast<int>(blockIdx.x) >= nexp) {  // weight staging (hop 0 only)
    gcn_stage_blocks(a, blockIdx.x - nexp, gridDim.x - nexp);
    return;
  }
  __shared__ int lds4[4];
  __shared__ int s_incl[kGcnExpandT];
  __shared__ int32_t s_row[kGcnExpandT];
  __shared__ int64_t s_start[kGcnExpandT];
  __shared__ int64_t s_prefix;
  const int tid = threadIdx.x;
  const int32_t stamp = a.stamp[0];
  const int64_t tb = static_cast<int64_t>(blockIdx.x) * TE;
  const int64_t t = tb + tid;
  const int nt = a.h == 0 ? a.B : a.cnt[a.h];
  // this hop's source counts start from zero (place adds)
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + tid; i < a.cap_n; i += static_cast<int64_t>(nexp) * 256)
    a.deg_s[i] = 0;
  // blocks past the last real target have nothing to publish: no later block reads them
  const int lastb = (nt - 1) / TE;
  if (static_cast<int>(blockIdx.x) > lastb) return;
  int32_t row = -1;
  int deg = 0;
  int64_t start = 0;
  bool contig = true;
  if (tid < TE && t < nt && t < a.cap_t) {
    if (a.h == 0 && a.roots_given) {  // drawn by the layer-wise draw launch
      row = a.roots[t];
    } else if (a.h == 0) {  // this block's roots: the alias draw of sampling.hip, stream 1
      const uint4_t r = Philox::gen(static_cast<uint64_t>(a.rng[0]), (static_cast<uint64_t>(a.rng[1]) << 8) ^ 1ull,
                                    static_cast<uint64_t>(t));
      const uint64_t x = (static_cast<uint64_t>(r[0]) << 32) | r[1];
      int64_t k = static_cast<int64_t>(__umul64hi(x, static_cast<uint64_t>(a.pop)));
      if (k >= a.pop) k = a.pop - 1;
      const int64_t pick = (u01(r[2]) < a.prob[k]) ? k : static_cast<int64_t>(a.alias[k]);
      row = a.root_rows ? a.root_rows[pick] : static_cast<int32_t>(pick);
      a.roots[t] = row;
    } else {
      row = a.set[t];
    }
    if (row >= 0 && row < a.g.num_rows) deg = masked_degree(a.g, row, a.mask, &start, &contig);
    else row = -1;
  }
  if (!contig) start = -1;  // per-type walk (masked_nbr) for this target
  const int raw = deg;
  if (a.lflag && row >= 0) {  // FastGCN layer: only the neighbours in this step's layer
    int kept = 0;
    for (int k0 = 0; k0 < raw; k0 += 8) {
      int32_t v[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int k = k0 + u;
        v[u] = k < raw ? (start >= 0 ? a.g.nbr[start + k] : masked_nbr(a.g, row, a.mask, k)) : -1;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) kept += (v[u] >= 0 && a.lflag[v[u]] == stamp) ? 1 : 0;
    }
    deg = kept;
  }
  int total = 0;
  const int incl = block_scan_incl(deg, lds4, &total);
  __shared__ int s_raw[kGcnExpandT];
  if (tid < TE) {
    s_incl[tid] = incl;
    s_row[tid] = row;
    s_start[tid] = start;
    s_raw[tid] = raw;
  }
  if (tid < 64) {
    const int64_t p = lb_prefix(a.scan_deg, blockIdx.x, total, static_cast<uint32_t>(stamp) * 8u + 2u * a.h, a.err);
    if (tid == 0) s_prefix = p;
  }
  __syncthreads();
  const int64_t prefix = s_prefix;
  if (tid < TE && t < a.cap_t) {
    const int64_t excl = prefix + incl - deg;
    a.off[t] = static_cast<int32_t>(excl < a.cap_e ? excl : a.cap_e);
  }
  if (static_cast<int>(blockIdx.x) == lastb && tid < 64) {
    // the end offset, read as the hop's total (off[cap_t]) and as the end of the last
    // aggregation tile (16 targets, which may reach past this block when te < 16): every
    // entry up to the next multiple of 64 beyond the block
    const int64_t tot = prefix + total;
    const int32_t v = static_cast<int32_t>(tot < a.cap_e ? tot : a.cap_e);
    const int64_t te_end = tb + TE + tid;
    if (te_end < a.cap_t && te_end <= ((tb + TE + 63) & ~int64_t{63})) a.off[te_end] = v;
    if (tid == 0) {
      a.off[a.cap_t] = v;
      if (tot > a.cap_e) atomicOr(a.overflow, 1);
    }
  }
  // hop 0: the roots are occurrences 0..B-1 (S_1 begins with the distinct roots)
  if (a.h == 0 && row >= 0) atomicMin(reinterpret_cast<unsigned long long*>(&a.first[row]), gcn_key(stamp, 0, t));
  if (a.lflag) {
    // filtered: one wave per target walks its neighbour list 64 at a time; the kept ones
    // (ballot + prefix popcount) take consecutive edge slots in neighbour order
    const int lane = tid & 63, wave = tid >> 6;
    const uint64_t below = lane == 0 ? 0ull : (~0ull >> (64 - lane));
    for (int tl = wave; tl < TE; tl += 4) {
      const int32_t r = s_row[tl];
      if (r < 0) continue;
      const int n = s_raw[tl];
      const int64_t st = s_start[tl];
      int64_t e_at = prefix + (tl > 0 ? s_incl[tl - 1] : 0);
      for (int c0 = 0; c0 < n; c0 += 64) {
        const int k = c0 + lane;
        const int32_t v = k < n ? (st >= 0 ? a.g.nbr[st + k] : masked_nbr(a.g, r, a.mask, k)) : -1;
        const bool keep = v >= 0 && a.lflag[v] == stamp;
        const uint64_t bal = __ballot(keep);
        if (keep) {
          const int64_t e = e_at + __popcll(bal & below);
          if (e < a.cap_e) {
            const int32_t tg = a.tag[v];
            const int32_t old = atomicAdd(&a.cntw[v], 1);
            a.enode[e] = v;
            a.etgt[e] = static_cast<int32_t>(tb + tl);
            a.eflag[e] = static_cast<uint8_t>(old == 0 ? (tg != stamp ? 3 : 1) : 0);
          }
        }
        e_at += __popcll(bal);
      }
    }
    return;
  }
  // the block's edges [prefix, prefix + total): target by a binary search of the block's
  // inclusive offsets; 8 edges per thread per pass, loads and counter atomics of a pass
  // issued together
  constexpr int U = 8;
  for (int i0 = tid; i0 < total; i0 += 256 * U) {
    int32_t v[U], tl[U];
    int64_t e[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int i = i0 + u * 256;
      v[u] = -1;
      tl[u] = 0;
      e[u] = -1;
      if (i < total && prefix + i < a.cap_e) {
        int lo = 0, hi = TE - 1;
        while (lo < hi) {
          const int m = (lo + hi) >> 1;
          if (s_incl[m] > i) hi = m;
          else lo = m + 1;
        }
        const int kk = i - (lo > 0 ? s_incl[lo - 1] : 0);  // neighbour index within target lo
        const int64_t st = s_start[lo];
        v[u] = st >= 0 ? a.g.nbr[st + kk] : masked_nbr(a.g, s_row[lo], a.mask, kk);
        tl[u] = lo;
        e[u] = prefix + i;
      }
    }
    int32_t tg[U], old[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      tg[u] = stamp;
      old[u] = 1;
      if (v[u] >= 0) {
        tg[u] = a.tag[v[u]];
        old[u] = atomicAdd(&a.cntw[v[u]], 1);
      }
    }
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (e[u] < 0) continue;
      a.enode[e[u]] = v[u];
      a.etgt[e[u]] = static_cast<int32_t>(tb + tl[u]);
      a.eflag[e[u]] = static_cast<uint8_t>(old[u] == 0 ? (tg[u] != stamp ? 3 : 1) : 0);
    }
  }
}

// ----------------------------------------------------------------------------
// mark: first occurrences -> positions in S_{h+1}
// ----------------------------------------------------------------------------
constexpr int kGcnMarkPer = 4;  // occurrences per thread (1024 per block: a quarter of the look-back chain)

__global__ __launch_bounds__(256) void gcn_mark_kernel(GcnHop a) {
  __shared__ int lds4[4];
  __shared__ int64_t s_prefix;
  const int tid = threadIdx.x;
  const int32_t stamp = a.stamp[0];
  const int64_t o0 = static_cast<int64_t>(blockIdx.x) * 256 * kGcnMarkPer + tid * kGcnMarkPer;
  const int64_t base_occ = a.h == 0 ? a.B : 0;
  const int64_t n_occ = base_occ + a.off[a.cap_t];
  // the grid covers the capacity; blocks past the last occurrence exit (nothing reads them)
  const int64_t lastb = n_occ > 0 ? (n_occ - 1) / (256 * kGcnMarkPer) : 0;
  if (static_cast<int64_t>(blockIdx.x) > lastb) return;
  int32_t v[kGcnMarkPer];
  bool isf[kGcnMarkPer];
  uint8_t fl[kGcnMarkPer];
#pragma unroll
  for (int j = 0; j < kGcnMarkPer; ++j) {  // every flag load in flight first
    const int64_t o = o0 + j;
    fl[j] = (o >= base_occ && o < n_occ) ? a.eflag[o - base_occ] : 0;
  }
  int c = 0;
#pragma unroll
  for (int j = 0; j < kGcnMarkPer; ++j) {
    const int64_t o = o0 + j;
    v[j] = -1;
    isf[j] = false;
    if (o < base_occ) {
      const int32_t r = a.roots[o];
      v[j] = (r >= 0 && r < a.g.num_rows) ? r : -1;
      isf[j] = v[j] >= 0 && a.first[v[j]] == gcn_key(stamp, 0, o);
    } else if (fl[j] & 2) {
      v[j] = a.enode[o - base_occ];
      // hop 0: a root reached as a neighbour is already S_1's (the roots come first); a
      // root's key this step is (stamp, hop 0, occurrence < B) — the all-ones initial key
      // shares stamp 0's high word but not the occurrence
      if (a.h == 0) {
        const uint64_t k = a.first[v[j]];
        isf[j] = (k >> 32) != (gcn_key(stamp, 0, 0) >> 32) || (k & 0xFFFFFFFFu) >= static_cast<uint64_t>(a.B);
      } else {
        isf[j] = true;
      }
    }
    c += isf[j] ? 1 : 0;
  }
  int total = 0;
  const int incl = block_scan_incl(c, lds4, &total);
  if (tid < 64) {
    const int64_t p = lb_prefix(a.scan_flag, blockIdx.x, total, static_cast<uint32_t>(stamp) * 8u + 2u * a.h + 1u,
                                a.err);
    if (tid == 0) s_prefix = p;
  }
  __syncthreads();
  const int64_t base_pos = a.h == 0 ? 0 : a.cnt[a.h];
  int64_t p = base_pos + s_prefix + incl - c;
#pragma unroll
  for (int j = 0; j < kGcnMarkPer; ++j) {
    if (!isf[j]) continue;
    if (p < a.cap_n) {
      a.set[p] = v[j];
      a.pos[v[j]] = static_cast<int32_t>(p);
      a.tag[v[j]] = stamp;
    } else {
      atomicOr(a.overflow, 1);
    }
    ++p;
  }
  if (static_cast<int64_t>(blockIdx.x) == lastb && tid == 255) {
    const int64_t n = base_pos + s_prefix + incl;
    a.cnt[a.h + 1] = static_cast<int32_t>(n < a.cap_n ? n : a.cap_n);
  }
}

// ----------------------------------------------------------------------------
// place: edge sources, self loops, per-source in-block counts (one atomic per distinct
// source, from its counter claimer, + one per self loop)
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gcn_place_kernel(GcnHop a) {
  const int32_t stamp = a.stamp[0];
  const int64_t total_e = a.off[a.cap_t];
  const int nt = a.h == 0 ? a.B : a.cnt[a.h];
  const int64_t n = a.cap_e + a.cap_t;
  for (int64_t i = static_cast<int64_t>(blockIdx.x) * 256 + threadIdx.x; i < n;
       i += static_cast<int64_t>(gridDim.x) * 256) {
    if (i < a.cap_e) {
      if (i >= total_e) continue;
      const int32_t v = a.enode[i];
      const uint8_t f = a.eflag[i];
      const int32_t s = (v >= 0 && a.tag[v] == stamp) ? a.pos[v] : -1;
      a.esrc[i] = s;
      if (f & 1) {  // the counter claimer: the node's edges of this hop, then reset
        const int32_t c = a.cntw[v];
        a.cntw[v] = 0;
        if (s >= 0) atomicAdd(&a.deg_s[s], c);
      }
    } else {
      const int64_t t = i - a.cap_e;
      if (t >= nt || !a.self_loops) continue;
      int32_t s;
      if (a.h == 0) {
        const int32_t r = a.roots[t];
        s = (r >= 0 && r < a.g.num_rows && a.tag[r] == stamp) ? a.pos[r] : -1;
        a.rself[t] = s;
      } else {
        s = static_cast<int32_t>(t);
      }
      if (s >= 0) atomicAdd(&a.deg_s[s], 1);
    }
  }
}

// ----------------------------------------------------------------------------
// edge-parallel weighted aggregation of a 16-target tile into an LDS fp32 accumulator
// acc[16][KP + 1]:  acc[t] = sum_e rsqrt(deg_t) rsqrt(deg_s[src_e]) x[src_e]  (+ self loop)
// ----------------------------------------------------------------------------
constexpr int kGT = 16;  // targets per tile

template <int KP, int NT = 256>
struct AggTile {
  static constexpr int NCH = KP / 8;     // column chunks of 8 (one lane each)
  static constexpr int NW = NT / NCH;    // workers per block of NT threads
  static constexpr int LDA = KP + 1;     // fp32 accumulator row stride (bank spread)
};

// one row chunk (8 columns) as loaded: bf16 rows stay packed (4 dwords) until they are
// accumulated, so a worker keeps twice as many rows in flight in the same registers
template <bool F32>
struct RowRaw {
  uint32_t w[F32 ? 8 : 4];
};

template <bool F32>
__device__ __forceinline__ void row_load(const GcnAggSrc& s, int32_t row, int c, RowRaw<F32>& r) {
  if (row < 0 || c * 8 >= s.cols) {
#pragma unroll
    for (int j = 0; j < (F32 ? 8 : 4); ++j) r.w[j] = 0u;
    return;
  }
  if constexpr (F32) {
    const float* p = static_cast<const float*>(s.x) + static_cast<int64_t>(row) * s.ld + c * 8;
    const uint4_t lo = *reinterpret_cast<const uint4_t*>(p);
    const uint4_t hi = *reinterpret_cast<const uint4_t*>(p + 4);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      r.w[j] = lo[j];
      r.w[4 + j] = hi[j];
    }
  } else {
    const uint4_t v =
        *reinterpret_cast<const uint4_t*>(static_cast<const bf16_t*>(s.x) + static_cast<int64_t>(row) * s.ld + c * 8);
#pragma unroll
    for (int j = 0; j < 4; ++j) r.w[j] = v[j];
  }
}

template <bool F32>
__device__ __forceinline__ void row_axpy(const RowRaw<F32>& r, float w, float* run) {
  if constexpr (F32) {
#pragma unroll
    for (int j = 0; j < 8; ++j) run[j] += w * __uint_as_float(r.w[j]);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      run[2 * j] += w * __uint_as_float(r.w[j] << 16);
      run[2 * j + 1] += w * __uint_as_float(r.w[j] & 0xffff0000u);
    }
  }
}

// enode: neighbour node ids of the hop (by-id sources read row = enode[e]); self_src:
// nullable (target t's self-loop source is t) ; nt: real targets
// per-target prelude (threads < 16, once per tile): rsqrt of the target degree, the self
// loop's source and source row, so the self items of the main loop need no extra round.
// Each worker (NCH lanes, one per 8 columns) walks a contiguous slice of the tile's edges,
// U per batch, software-pipelined: the next batch's index loads are in flight while the
// current batch's rows are accumulated, and its rows (+ source degrees) are issued before
// the loop comes back — one memory round trip per batch instead of two.
template <int KP, bool F32, int NT>
__device__ void gcn_aggregate_t(const GcnAggSrc& src, const int32_t* off, const int32_t* etgt, const int32_t* esrc,
                                const int32_t* enode, const int32_t* deg_s, const int32_t* self_src, int self_loops,
                                int64_t t0, int nt, float* acc, float* rdt, int* sself) {
  using AT = AggTile<KP, NT>;
  const int tid = threadIdx.x;
  for (int i = tid; i < kGT * AT::LDA; i += NT) acc[i] = 0.f;
  __shared__ int64_t s_e[2];
  __shared__ int s_row[kGT];
  if (tid == 0) {
    s_e[0] = off[t0];
    s_e[1] = off[t0 + kGT];
  }
  if (tid < kGT) {
    const int64_t t = t0 + tid;
    const int dt = t < nt ? static_cast<int>(off[t + 1] - off[t]) + self_loops : 0;
    rdt[tid] = dt > 0 ? rsqrtf(static_cast<float>(dt)) : 0.f;
    const int ss = t < nt ? (self_src ? self_src[t] : static_cast<int>(t)) : -1;
    sself[tid] = ss;
    s_row[tid] = ss < 0 ? -1 : (src.by_id ? src.set[ss] : ss);
  }
  __syncthreads();
  const int64_t e0 = s_e[0], E = s_e[1] - s_e[0];
  const int nself = self_loops ? static_cast<int>(nt - t0 < kGT ? (nt - t0 > 0 ? nt - t0 : 0) : kGT) : 0;
  const int64_t W = E + nself;
  const int g = tid / AT::NCH, c = tid % AT::NCH;
  const int64_t per = (W + AT::NW - 1) / AT::NW;
  const int64_t i0 = g * per, i1 = (i0 + per) < W ? (i0 + per) : W;
  constexpr int U = F32 ? 4 : 8;  // the same 32 dwords of rows in flight per batch
  float run[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  int cur = -1;
  auto flush = [&]() {
    if (cur >= 0) {
#pragma unroll
      for (int j = 0; j < 8; ++j) atomicAdd(&acc[cur * AT::LDA + c * 8 + j], run[j]);
    }
#pragma unroll
    for (int j = 0; j < 8; ++j) run[j] = 0.f;
  };
  auto load_idx = [&](int64_t i, int* tl, int* sv, int* row) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const int64_t ii = i + u;
      tl[u] = -1;
      sv[u] = -1;
      row[u] = -1;
      if (ii < i1) {
        if (ii < E) {
          const int64_t e = e0 + ii;
          tl[u] = static_cast<int>(etgt[e] - t0);
          sv[u] = esrc[e];
          row[u] = src.by_id ? enode[e] : sv[u];
        } else {
          tl[u] = static_cast<int>(ii - E);
          sv[u] = sself[tl[u]];
          row[u] = s_row[tl[u]];
        }
      }
    }
  };
  auto load_rows = [&](const int* sv, const int* row, float* ds, RowRaw<F32>* x) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      ds[u] = sv[u] >= 0 ? static_cast<float>(deg_s[sv[u]]) : 1.f;
      row_load<F32>(src, sv[u] >= 0 ? row[u] : -1, c, x[u]);
    }
  };
  int tl0[U], s0[U], r0[U];
  float ds0[U];
  RowRaw<F32> x0[U];
  if (i0 < i1) {
    load_idx(i0, tl0, s0, r0);
    load_rows(s0, r0, ds0, x0);
  }
  for (int64_t i = i0; i < i1; i += U) {
    int tl1[U], s1[U], r1[U];
    const bool more = i + U < i1;
    if (more) load_idx(i + U, tl1, s1, r1);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      if (tl0[u] < 0 || s0[u] < 0) continue;
      if (tl0[u] != cur) {
        flush();
        cur = tl0[u];
      }
      row_axpy<F32>(x0[u], rdt[tl0[u]] * rsqrtf(ds0[u]), run);
    }
    if (!more) break;
    load_rows(s1, r1, ds0, x0);
#pragma unroll
    for (int u = 0; u < U; ++u) {
      tl0[u] = tl1[u];
      s0[u] = s1[u];
    }
  }
  flush();
  __syncthreads();
}

template <int KP, int NT = 256>
__device__ void gcn_aggregate(const GcnAggSrc& src, const int32_t* off, const int32_t* etgt, const int32_t* esrc,
                              const int32_t* enode, const int32_t* deg_s, const int32_t* self_src, int self_loops,
                              int64_t t0, int nt, float* acc, float* rdt, int* sself) {
  if (src.x_fp32)
    gcn_aggregate_t<KP, true, NT>(src, off, etgt, esrc, enode, deg_s, self_src, self_loops, t0, nt, acc, rdt, sself);
  else
    gcn_aggregate_t<KP, false, NT>(src, off, etgt, esrc, enode, deg_s, self_src, self_loops, t0, nt, acc, rdt, sself);
}

// ----------------------------------------------------------------------------
// MFMA operand reads from row-major bf16 LDS images
// ----------------------------------------------------------------------------
__device__ __forceinline__ uint4_t lds16(const bf16_t* p) { return *reinterpret_cast<const uint4_t*>(p); }

// standard fragment: row r0 + (lane & 15), k = k0 + 8 (lane >> 4) .. +7
__device__ __forceinline__ uint4_t frag_std(const bf16_t* img, int ld, int r0, int k0, int lane) {
  return lds16(img + (r0 + (lane & 15)) * ld + k0 + (lane >> 4) * 8);
}
// the k permutation of tl_tr_frag: lane group g holds k0 + 4g .. +3 and k0 + 16 + 4g .. +3
__device__ __forceinline__ uint4_t frag_perm(const bf16_t* img, int ld, int r0, int k0, int lane) {
  const bf16_t* p = img + (r0 + (lane & 15)) * ld + k0 + (lane >> 4) * 4;
  const tl_uint2 lo = *reinterpret_cast<const tl_uint2*>(p);
  const tl_uint2 hi = *reinterpret_cast<const tl_uint2*>(p + 16);
  return uint4_t{lo[0], lo[1], hi[0], hi[1]};
}
template <int LD>
__device__ __forceinline__ uint4_t frag_tr(const bf16_t* img, int e0, int c0, int lane) {
  return tl_tr_frag<LD>(img, e0, c0, lane);
}

// stage an fp32 [rows][cols] matrix into a bf16 LDS image [rowsp][ld] (zero padding)
__device__ __forceinline__ void stage_w(const float* w, int rows, int cols, int rowsp, int colsp, bf16_t* img,
                                        int ld) {
  for (int i = threadIdx.x; i < rowsp * (colsp >> 1); i += 256) {
    const int r = i / (colsp >> 1), c = (i - r * (colsp >> 1)) * 2;
    const float a = (r < rows && c < cols) ? w[static_cast<int64_t>(r) * cols + c] : 0.f;
    const float b = (r < rows && c + 1 < cols) ? w[static_cast<int64_t>(r) * cols + c + 1] : 0.f;
    *reinterpret_cast<uint32_t*>(img + r * ld + c) = pack_bf16x2(a, b);
  }
}

// copy a staged bf16 image (global, 16-byte multiples) into LDS: every load in flight
template <int NT = 256>
__device__ __forceinline__ void copy_img(const uint16_t* src, bf16_t* dst, int n) {
  const uint4_t* s = reinterpret_cast<const uint4_t*>(src);
  uint4_t* d = reinterpret_cast<uint4_t*>(dst);
  const int n16 = n >> 3;
  constexpr int U = 8;
  for (int i0 = threadIdx.x; i0 < n16; i0 += NT * U) {
    uint4_t v[U];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * NT < n16) v[u] = s[i0 + u * NT];
#pragma unroll
    for (int u = 0; u < U; ++u)
      if (i0 + u * NT < n16) d[i0 + u * NT] = v[u];
  }
}

__device__ __forceinline__ void zero_img(bf16_t* img, int n) {
  for (int i = threadIdx.x; i < (n >> 1); i += 256) reinterpret_cast<uint32_t*>(img)[i] = 0u;
}

// LDS image stride for a width: the tl_tr_frag bank-spreading strides (tile.h)
__host__ __device__ constexpr int img_ld(int w) { return w <= 64 ? 80 : 144; }

// ----------------------------------------------------------------------------
// layer (L = 2): targets S_1 in tiles of 16, sources S_2 (feature rows by node id)
// ----------------------------------------------------------------------------
// threads per 16-target tile of the layer launch (512 measured slower on PPI: 33.4 vs
// 25.2 us, profiles/r5_gcn/fused_v3/ — the tile's LDS flushes contend and fewer tiles
// are resident)
constexpr int kGcnLayerThreads = 256;

template <int KP, int HP>
__global__ __launch_bounds__(kGcnLayerThreads) void gcn_layer_kernel(GcnLayerArgs a) {
  constexpr int NT = kGcnLayerThreads;
  constexpr int LDK = img_ld(KP), LDAcc = AggTile<KP, NT>::LDA;
  __shared__ __attribute__((aligned(16))) bf16_t wimg[HP * LDK];
  __shared__ __attribute__((aligned(16))) bf16_t aimg[kGT * LDK];
  __shared__ float acc[kGT * LDAcc];
  __shared__ float rdt[kGT];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int nt = a.cnt[1];
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kGT;
  if (t0 >= nt) return;  // uniform: rows past the set are never read
  copy_img<NT>(a.wimg, wimg, HP * LDK);
  __shared__ int sself[kGT];
  gcn_aggregate<KP, NT>(a.src, a.off, a.etgt, a.esrc, a.enode, a.deg_s, nullptr, a.self_loops, t0, nt, acc, rdt,
                        sself);
  // aggregate -> bf16 image + the dW operand rows
  for (int i = tid; i < kGT * (KP / 2); i += NT) {
    const int r = i / (KP / 2), c = (i - r * (KP / 2)) * 2;
    const uint32_t pk = pack_bf16x2(acc[r * LDAcc + c], acc[r * LDAcc + c + 1]);
    *reinterpret_cast<uint32_t*>(aimg + r * LDK + c) = pk;
    *reinterpret_cast<uint32_t*>(a.agg_out + (t0 + r) * KP + c) = pk;
  }
  __syncthreads();
  // z = agg W^T, h = relu(z): wave w -> 16-column tiles w, w + NT / 64, ...
  for (int ct = wave; ct < HP / 16; ct += NT / 64) {
    float4_t z = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < KP; k0 += 32)
      z = mfma16(frag_std(aimg, LDK, 0, k0, lane), frag_std(wimg, LDK, ct * 16, k0, lane), z);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = (lane >> 4) * 4 + j;
      a.h_out[(t0 + r) * HP + ct * 16 + (lane & 15)] = f2bf(fmaxf(z[j], 0.f));
    }
  }
}

// ----------------------------------------------------------------------------
// head: 16 roots per block; the last conv, fc, out_fc, loss and the row-local backward.
// Images: weights [out][in] bf16 (the fc / out_fc images at stride 144: E, C <= 128),
// activations [32 rows][width] with rows 16..31 zero (the k = 32 of the row-reduction
// MFMAs of the weight gradients).
// ----------------------------------------------------------------------------
constexpr int kWide = 144;  // LDS stride of the E- and C-wide images

__host__ __device__ inline size_t gcn_head_lds_bytes(int KP, int HP, int EP, int CP) {
  const int LK = img_ld(KP), LH = img_ld(HP);
  const size_t bf = static_cast<size_t>(HP) * LK + static_cast<size_t>(EP) * LH + static_cast<size_t>(CP) * kWide +
                    32 * LK + 32 * LH + 32 * kWide * 3 + 32 * LH;
  return bf * 2 + static_cast<size_t>(kGT) * (KP + 1) * 4 + kGT * 4 + static_cast<size_t>(kGT) * CP * 4 + 64;
}

template <int KP, int HP>
__global__ __launch_bounds__(256) void gcn_head_kernel(GcnHeadArgs a) {
  constexpr int LK = img_ld(KP), LH = img_ld(HP), LE = kWide, LC = kWide;
  const int EP = a.Ep, CP = a.Cp;
  extern __shared__ __attribute__((aligned(16))) bf16_t lds[];
  bf16_t* Wl = lds;                 // [HP][LK] last conv W [out][in]
  bf16_t* Wf = Wl + HP * LK;        // [EP][LH] fc W [E][H]
  bf16_t* Wo = Wf + EP * LH;        // [CP][LE] out W [C][E]
  bf16_t* Ag = Wo + CP * LE;        // [32][LK] aggregate
  bf16_t* H0 = Ag + 32 * LK;        // [32][LH] relu(z)
  bf16_t* Em = H0 + 32 * LH;        // [32][LE] emb
  bf16_t* Dl = Em + 32 * LE;        // [32][LC] d logits
  bf16_t* De = Dl + 32 * LC;        // [32][LE] d emb
  bf16_t* Dz = De + 32 * LE;        // [32][LH] d z (ReLU mask applied)
  float* acc = reinterpret_cast<float*>(Dz + 32 * LH);  // [16][KP + 1]
  float* rdt = acc + kGT * AggTile<KP>::LDA;
  __shared__ float red[4][4];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int lr = lane & 15, lg = lane >> 4;
  const int64_t t0 = static_cast<int64_t>(blockIdx.x) * kGT;
  const int blk = blockIdx.x;
  // the weights (fp32 masters -> bf16) and cleared activation images
  __shared__ int sself[kGT];
  __shared__ int s_root[kGT];
  float* lab = rdt + kGT;  // [16][CP] the tile's dense labels
#define GH_STAMP(k) \
  if (a.prof && threadIdx.x == 0) a.prof[static_cast<int64_t>(blockIdx.x) * 16 + (k)] = wall_clock64()
  GH_STAMP(0);
  if (a.ostep_inc && blk == 0 && tid == 0) a.ostep_inc[0] += 1;  // read by this step's reduce launch
  if (tid < kGT) s_root[tid] = t0 + tid < a.B ? a.roots[t0 + tid] : -1;
  copy_img(a.wl_img, Wl, HP * LK);
  copy_img(a.wfc_img, Wf, EP * LH);
  copy_img(a.wout_img, Wo, CP * LE);
  zero_img(Ag, 32 * LK + 32 * LH + 32 * LE * 3 + 32 * LH);
  __syncthreads();
  GH_STAMP(1);
  {  // every label load in flight at once (16 x CP <= 2048 values: 8 per thread)
    float v[8];
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      const int i = tid + u * 256;
      const int r = i / CP, c = i - r * CP;
      const int32_t root = i < kGT * CP ? s_root[r] : -1;
      v[u] = (root >= 0 && c < a.C) ? a.labels[static_cast<int64_t>(root) * a.C + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < 8; ++u)
      if (tid + u * 256 < kGT * CP) lab[tid + u * 256] = v[u];
  }
  gcn_aggregate<KP>(a.src, a.off, a.etgt, a.esrc, a.enode, a.deg_s, a.rself, a.self_loops, t0, a.B, acc, rdt,
                    sself);
  for (int i = tid; i < kGT * (KP / 2); i += 256) {
    const int r = i / (KP / 2), c = (i - r * (KP / 2)) * 2;
    *reinterpret_cast<uint32_t*>(Ag + r * LK + c) = pack_bf16x2(acc[r * AggTile<KP>::LDA + c],
                                                                acc[r * AggTile<KP>::LDA + c + 1]);
    if (a.dbg_agg && t0 + r < a.B) {
      a.dbg_agg[(t0 + r) * KP + c] = acc[r * AggTile<KP>::LDA + c];
      a.dbg_agg[(t0 + r) * KP + c + 1] = acc[r * AggTile<KP>::LDA + c + 1];
    }
  }
  __syncthreads();
  GH_STAMP(2);
  // z = Ag Wl^T -> H0 = relu(z)
  for (int ct = wave; ct < HP / 16; ct += 4) {
    float4_t z = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < KP; k0 += 32)
      z = mfma16(frag_std(Ag, LK, 0, k0, lane), frag_std(Wl, LK, ct * 16, k0, lane), z);
#pragma unroll
    for (int j = 0; j < 4; ++j) H0[(lg * 4 + j) * LH + ct * 16 + lr] = f2bf(fmaxf(z[j], 0.f));
  }
  __syncthreads();
  GH_STAMP(3);
  // emb = H0 Wf^T + bfc
  for (int ct = wave; ct < EP / 16; ct += 4) {
    float4_t z = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < HP; k0 += 32)
      z = mfma16(frag_std(H0, LH, 0, k0, lane), frag_std(Wf, LH, ct * 16, k0, lane), z);
    const int col = ct * 16 + lr;
    const float b = col < a.E ? a.bfc[col] : 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) Em[(lg * 4 + j) * LE + col] = f2bf(col < a.E ? z[j] + b : 0.f);
  }
  __syncthreads();
  GH_STAMP(4);
  // logits = emb Wo^T -> loss, F1 counts, d logits
  float lsum = 0.f, tp = 0.f, fp = 0.f, fn = 0.f;
  for (int ct = wave; ct < CP / 16; ct += 4) {
    float4_t z = float4_t{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < EP; k0 += 32)
      z = mfma16(frag_std(Em, LE, 0, k0, lane), frag_std(Wo, LE, ct * 16, k0, lane), z);
    const int col = ct * 16 + lr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = lg * 4 + j;
      const int64_t t = t0 + r;
      float d = 0.f;
      if (t < a.B && col < a.C) {
        const float y = lab[r * CP + col];
        const float x = z[j];
        lsum += fmaxf(x, 0.f) - x * y + log1pf(__expf(-fabsf(x)));
        const bool pred = x >= 0.f, pos = y > 0.5f;
        tp += (pred && pos) ? 1.f : 0.f;
        fp += (pred && !pos) ? 1.f : 0.f;
        fn += (!pred && pos) ? 1.f : 0.f;
        d = (1.f / (1.f + __expf(-x)) - y) * a.inv_scale;
      }
      Dl[r * LC + col] = f2bf(d);
    }
  }
  lsum = wave_sum(lsum);
  tp = wave_sum(tp);
  fp = wave_sum(fp);
  fn = wave_sum(fn);
  if (lane == 0) {
    red[wave][0] = lsum;
    red[wave][1] = tp;
    red[wave][2] = fp;
    red[wave][3] = fn;
  }
  __syncthreads();
  GH_STAMP(5);
  if (tid < 4) {  // the mean loss's share of this block; raw F1 counts
    const float v = red[0][tid] + red[1][tid] + red[2][tid] + red[3][tid];
    a.part_stat[blk * 4 + tid] = tid == 0 ? v * a.inv_scale : v;
  }
  // d emb = d logits Wo (K = C: the rows of Wo are the reduction index); d bfc partial
  for (int ct = wave; ct < EP / 16; ct += 4) {
    float4_t z = float4_t{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < CP; k0 += 32)
      z = mfma16(frag_perm(Dl, LC, 0, k0, lane), frag_tr<LE>(Wo, k0, ct * 16, lane), z);
    const int col = ct * 16 + lr;
    float cs = 0.f;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      De[(lg * 4 + j) * LE + col] = f2bf(z[j]);
      cs += z[j];
    }
    cs += __shfl_xor(cs, 16, 64);
    cs += __shfl_xor(cs, 32, 64);
    if (lg == 0) a.part_bfc[static_cast<int64_t>(blk) * EP + col] = cs;
  }
  __syncthreads();
  GH_STAMP(6);
  // d z = (d emb Wf) * relu'(z)   (K = E: the rows of Wf are the reduction index)
  for (int ct = wave; ct < HP / 16; ct += 4) {
    float4_t z = float4_t{0.f, 0.f, 0.f, 0.f};
    for (int k0 = 0; k0 < EP; k0 += 32)
      z = mfma16(frag_perm(De, LE, 0, k0, lane), frag_tr<LH>(Wf, k0, ct * 16, lane), z);
    const int col = ct * 16 + lr;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int r = lg * 4 + j;
      Dz[r * LH + col] = f2bf(bf_pos(H0[r * LH + col]) ? z[j] : 0.f);
    }
  }
  __syncthreads();
  GH_STAMP(7);
  // weight-gradient partials of this block's rows (k = the 32 image rows, 16..31 zero):
  // d out W = Dl^T Em [CP][EP], d fc W = De^T H0 [EP][HP], d conv W = Dz^T Ag [HP][KP]
  {
    const int n1 = (CP / 16) * (EP / 16), n2 = (EP / 16) * (HP / 16);
    constexpr int n3 = (HP / 16) * (KP / 16);
    for (int j = wave; j < n1 + n2 + n3; j += 4) {
      float4_t z = float4_t{0.f, 0.f, 0.f, 0.f};
      float* out;
      int ld, r0, c0;
      if (j < n1) {
        r0 = (j / (EP / 16)) * 16;
        c0 = (j % (EP / 16)) * 16;
        z = mfma16(frag_tr<LC>(Dl, 0, r0, lane), frag_tr<LE>(Em, 0, c0, lane), z);
        out = a.part_out + static_cast<int64_t>(blk) * CP * EP;
        ld = EP;
      } else if (j < n1 + n2) {
        const int q = j - n1;
        r0 = (q / (HP / 16)) * 16;
        c0 = (q % (HP / 16)) * 16;
        z = mfma16(frag_tr<LE>(De, 0, r0, lane), frag_tr<LH>(H0, 0, c0, lane), z);
        out = a.part_fc + static_cast<int64_t>(blk) * EP * HP;
        ld = HP;
      } else {
        const int q = j - n1 - n2;
        r0 = (q / (KP / 16)) * 16;
        c0 = (q % (KP / 16)) * 16;
        z = mfma16(frag_tr<LH>(Dz, 0, r0, lane), frag_tr<LK>(Ag, 0, c0, lane), z);
        out = a.part_w + static_cast<int64_t>(blk) * HP * KP;
        ld = KP;
      }
#pragma unroll
      for (int q = 0; q < 4; ++q) out[static_cast<int64_t>(r0 + lg * 4 + q) * ld + c0 + lr] = z[q];
    }
  }
  if (a.dagg == nullptr) {  // L = 1: no layer below
    GH_STAMP(15);
    return;
  }
  // d agg = Dz Wl (K = H: the rows of Wl are the reduction index) -> the fp32 accumulator
  __syncthreads();
  GH_STAMP(8);
  for (int ct = wave; ct < KP / 16; ct += 4) {
    float4_t z = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int k0 = 0; k0 < HP; k0 += 32)
      z = mfma16(frag_perm(Dz, LH, 0, k0, lane), frag_tr<LK>(Wl, k0, ct * 16, lane), z);
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[(lg * 4 + j) * AggTile<KP>::LDA + ct * 16 + lr] = z[j];
  }
  __syncthreads();
  GH_STAMP(9);
  // d agg rows to global: gcn_dw_kernel reads them per hop-0 edge (no d h1 scatter)
  for (int i = tid; i < kGT * KP; i += 256) {
    const int r = i / KP, c = i - r * KP;
    if (t0 + r < a.B) a.dagg[(t0 + r) * KP + c] = acc[r * AggTile<KP>::LDA + c];
  }
  GH_STAMP(15);
#undef GH_STAMP
}

// ----------------------------------------------------------------------------
// dw (L = 2): d W0 partial = (d h1 * relu'(h1))^T agg over 128 rows of S_1; clears d h1
// ----------------------------------------------------------------------------
template <int KP, int HP>
__global__ __launch_bounds__(256) void gcn_dw_kernel(GcnDwArgs a) {
  // the ReLU mask of h1 is per source row, so
  //   d W0 = sum_s agg[s]^T (mask[s] . sum_{e: src s} w_e d agg[t_e])
  //        = sum_e w_e agg[s_e]^T (mask[s_e] . d agg[t_e])
  // and the rows of this GEMM are hop 0's edges (+ self loops): no d h1 scatter, no atomics
  constexpr int LK = img_ld(KP), LH = img_ld(HP), CH = kGcnDwRows / 32;
  __shared__ __attribute__((aligned(16))) bf16_t dz[CH][32 * LH];
  __shared__ __attribute__((aligned(16))) bf16_t ag[CH][32 * LK];
  __shared__ int32_t s_src[kGcnDwRows], s_tgt[kGcnDwRows];
  __shared__ float s_w[kGcnDwRows];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int64_t total = a.off[a.cap_t];
  const int64_t W = total + (a.self_loops ? a.B : 0);
  const int64_t r0 = static_cast<int64_t>(blockIdx.x) * kGcnDwRows;
  if (tid < kGcnDwRows) {
    const int64_t e = r0 + tid;
    int32_t sv = -1, tv = 0;
    if (e < total) {
      tv = a.etgt[e];
      sv = a.esrc[e];
    } else if (e < W) {
      tv = static_cast<int32_t>(e - total);
      sv = a.rself[tv];
    }
    float w = 0.f;
    if (sv >= 0) {
      const float dt = static_cast<float>(a.off[tv + 1] - a.off[tv] + a.self_loops);
      w = rsqrtf(dt) * rsqrtf(static_cast<float>(a.deg_s[sv]));
    }
    s_src[tid] = sv;
    s_tgt[tid] = tv;
    s_w[tid] = w;
  }
  __syncthreads();
  // every row load of the block in flight at once: dz = w (mask . d agg[t]), ag = agg[s]
  constexpr int NZ = kGcnDwRows * (HP / 8) / 256, NA = kGcnDwRows * (KP / 8) / 256;
  static_assert(NZ >= 1 && NA >= 1, "dw tile");
  uint4_t hv[NZ], av[NA];
  float4_t dlo[NZ], dhi[NZ];
#pragma unroll
  for (int u = 0; u < NZ; ++u) {
    const int i = tid + u * 256, r = i / (HP / 8), c = (i - r * (HP / 8)) * 8;
    const int32_t sv = s_src[r];
    hv[u] = uint4_t{0u, 0u, 0u, 0u};
    dlo[u] = dhi[u] = float4_t{0.f, 0.f, 0.f, 0.f};
    if (sv >= 0) {
      const int64_t t = s_tgt[r];
      hv[u] = *reinterpret_cast<const uint4_t*>(a.h + static_cast<int64_t>(sv) * HP + c);
      dlo[u] = *reinterpret_cast<const float4_t*>(a.dagg + t * HP + c);
      dhi[u] = *reinterpret_cast<const float4_t*>(a.dagg + t * HP + c + 4);
    }
  }
#pragma unroll
  for (int u = 0; u < NA; ++u) {
    const int i = tid + u * 256, r = i / (KP / 8), c = (i - r * (KP / 8)) * 8;
    const int32_t sv = s_src[r];
    av[u] = sv >= 0 ? *reinterpret_cast<const uint4_t*>(a.agg + static_cast<int64_t>(sv) * KP + c)
                    : uint4_t{0u, 0u, 0u, 0u};
  }
#pragma unroll
  for (int u = 0; u < NZ; ++u) {
    const int i = tid + u * 256, r = i / (HP / 8), c = (i - r * (HP / 8)) * 8;
    const float w = s_w[r];
    uint4_t o;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const uint32_t hw = hv[u][q];
      const float x0 = q < 2 ? dlo[u][2 * q] : dhi[u][2 * q - 4];
      const float x1 = q < 2 ? dlo[u][2 * q + 1] : dhi[u][2 * q - 3];
      o[q] = pack_bf16x2(bf_pos(static_cast<bf16_t>(hw & 0xffffu)) ? w * x0 : 0.f,
                         bf_pos(static_cast<bf16_t>(hw >> 16)) ? w * x1 : 0.f);
    }
    *reinterpret_cast<uint4_t*>(&dz[r >> 5][(r & 31) * LH + c]) = o;
  }
#pragma unroll
  for (int u = 0; u < NA; ++u) {
    const int i = tid + u * 256, r = i / (KP / 8), c = (i - r * (KP / 8)) * 8;
    *reinterpret_cast<uint4_t*>(&ag[r >> 5][(r & 31) * LK + c]) = av[u];
  }
  __syncthreads();
  constexpr int nt = (HP / 16) * (KP / 16);
  for (int j = wave; j < nt; j += 4) {
    const int p0 = (j / (KP / 16)) * 16, q0 = (j % (KP / 16)) * 16;
    float4_t z = float4_t{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int ch = 0; ch < CH; ++ch) z = mfma16(frag_tr<LH>(dz[ch], 0, p0, lane), frag_tr<LK>(ag[ch], 0, q0, lane), z);
    float* out = a.part + static_cast<int64_t>(blockIdx.x) * HP * KP;
#pragma unroll
    for (int q = 0; q < 4; ++q) out[static_cast<int64_t>(p0 + (lane >> 4) * 4 + q) * KP + q0 + (lane & 15)] = z[q];
  }
}

// ----------------------------------------------------------------------------
// reduce: partial slabs -> flat gradient; loss / counts; epoch + 1
// 256 threads = 16 elements x 16 slab groups
// ----------------------------------------------------------------------------
__global__ __launch_bounds__(256) void gcn_reduce_kernel(GcnReduceArgs a) {
  __shared__ float red[16][17];
  const int tid = threadIdx.x, b = blockIdx.x;
  GcnRedSeg sg = a.seg[0];
#pragma unroll
  for (int k = 1; k < kGcnMaxSegs; ++k)
    if (k < a.nseg && b >= a.seg[k].blk0) sg = a.seg[k];
  const int el = tid & 15, grp = tid >> 4;
  const int64_t i = static_cast<int64_t>(b - sg.blk0) * 16 + el;
  const int64_t n = static_cast<int64_t>(sg.rows) * sg.cols;
  float s = 0.f;
  if (i < n) {
    const int64_t r = i / sg.cols, c = i - r * sg.cols;
    const float* p = sg.part + r * sg.prs + c;
    float v[8];
    for (int s0 = grp; s0 < sg.S; s0 += 128) {
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int sl = s0 + 16 * u;
        v[u] = sl < sg.S ? p[static_cast<int64_t>(sl) * sg.slab] : 0.f;
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) s += v[u];
    }
  }
  red[grp][el] = s;
  __syncthreads();
  if (grp == 0 && i < n) {
    float t = 0.f;
#pragma unroll
    for (int q = 0; q < 16; ++q) t += red[q][el];
    sg.grad[i] = t;
    if (a.fuse_opt) {
      float p = sg.p[i], m = sg.m[i], v = sg.v[i];
      optim_one(p, t, m, v, static_cast<float>(a.ostep[0]), a.lr, a.b1, a.b2, a.eps, a.wd, a.grad_scale, a.okind);
      sg.p[i] = p;
      if (a.okind == 0 || a.okind == 3) sg.m[i] = m;
      if (a.okind == 0 || a.okind == 1) sg.v[i] = v;
    }
  }

  if (b == 0 && tid < 64) {
    float st[4] = {0.f, 0.f, 0.f, 0.f};
    for (int k = tid; k < a.nstat; k += 64)
#pragma unroll
      for (int q = 0; q < 4; ++q) st[q] += a.part_stat[k * 4 + q];
#pragma unroll
    for (int q = 0; q < 4; ++q) st[q] = wave_sum(st[q]);
    if (tid == 0) {
      a.loss_out[0] = st[0];
      a.counts[0] += static_cast<int64_t>(st[1] + 0.5f);
      a.counts[1] += static_cast<int64_t>(st[2] + 0.5f);
      a.counts[2] += static_cast<int64_t>(st[3] + 0.5f);
      a.stamp[0] += 1;
      a.rng[1] += 1;
    }
  }
}

}  // namespace euler_hip

using namespace euler_hip;

extern "C" {

int64_t eh_gcn_expand_blocks(int64_t cap_t) { return ceil_div(cap_t, gcn_expand_tile(cap_t)); }
int64_t eh_gcn_mark_blocks(const GcnHop* a) {
  return ceil_div((a->h == 0 ? a->B : 0) + a->cap_e, 256 * kGcnMarkPer);
}

static bool gcn_hop_ok(const GcnHop* a) {
  return a && a->g.indptr && a->g.nbr && a->set && a->cnt && a->off && a->enode && a->etgt && a->esrc && a->deg_s &&
         a->first && a->cntw && a->eflag && a->tag && a->pos && a->scan_deg && a->scan_flag && a->stamp && a->overflow && a->err &&
         a->cap_t > 0 && a->cap_t % 256 == 0 && a->cap_e > 0 && a->cap_n > 0 && a->g.num_types >= 1 &&
         (a->h > 0 || (a->prob && a->alias && a->rng && a->pop > 0)) &&
         a->g.num_types <= 32 && (a->h > 0 || (a->roots && a->rself && a->B > 0 && a->B <= a->cap_t)) &&
         a->cap_e + a->B < (1ll << 31) && a->cap_n < (1ll << 31);
}

hipError_t eh_gcn_layer_draw(const GcnLayerDraw* a, hipStream_t s) {
  if (!a || !a->prob || !a->alias || a->pop < 1 || !a->rng || a->count < 1 || !a->lflag || !a->stamp)
    return hipErrorInvalidValue;
  if (a->kind == 1 && (a->B < 1 || a->B > kGcnLayerMaxRoots || !a->roots || !a->g.indptr || !a->g.nbr || !a->g.cumw))
    return hipErrorInvalidValue;
  const dim3 grid(a->kind == 1 ? 1u : static_cast<uint32_t>(ceil_div(a->count, 256)));
  hipLaunchKernelGGL(gcn_layer_draw_kernel, grid, dim3(256), 0, s, *a);
  return hipGetLastError();
}

hipError_t eh_gcn_expand(const GcnHop* a, hipStream_t s) {
  if (!gcn_hop_ok(a)) return hipErrorInvalidValue;
  if (a->nst < 0 || a->nst > kGcnMaxStage) return hipErrorInvalidValue;
  for (int k = 0; k < a->nst; ++k)
    if (!a->st[k].w || !a->st[k].img || a->st[k].rows > a->st[k].rowsp || a->st[k].cols > a->st[k].ld ||
        a->st[k].ld % 8 != 0)
      return hipErrorInvalidValue;
  const int64_t nb = eh_gcn_expand_blocks(a->cap_t) + (a->nst > 0 ? kGcnStageBlocks : 0);
  hipLaunchKernelGGL(gcn_expand_kernel, dim3(static_cast<uint32_t>(nb)), dim3(256), 0, s, *a);
  return hipGetLastError();
}

hipError_t eh_gcn_mark(const GcnHop* a, hipStream_t s) {
  if (!gcn_hop_ok(a)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gcn_mark_kernel, dim3(static_cast<uint32_t>(eh_gcn_mark_blocks(a))), dim3(256), 0, s, *a);
  return hipGetLastError();
}

hipError_t eh_gcn_place(const GcnHop* a, hipStream_t s) {
  if (!gcn_hop_ok(a)) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gcn_place_kernel, grid_for(a->cap_e + a->cap_t), dim3(256), 0, s, *a);
  return hipGetLastError();
}

static bool gcn_kp_ok(int k) { return k == 32 || k == 64 || k == 128; }
static bool gcn_hp_ok(int h) { return h == 32 || h == 64; }
static bool gcn_src_ok(const GcnAggSrc& s, int kp) {
  return s.x && s.ld >= s.cols && s.cols <= kp && s.ld % 8 == 0 && (!s.by_id || s.set);
}

#define GCN_DISPATCH(KP, HP, KERNEL, ...)                                            \
  do {                                                                              \
    if ((KP) == 32 && (HP) == 32) KERNEL(32, 32, __VA_ARGS__);                      \
    else if ((KP) == 32 && (HP) == 64) KERNEL(32, 64, __VA_ARGS__);                 \
    else if ((KP) == 64 && (HP) == 32) KERNEL(64, 32, __VA_ARGS__);                 \
    else if ((KP) == 64 && (HP) == 64) KERNEL(64, 64, __VA_ARGS__);                 \
    else if ((KP) == 128 && (HP) == 32) KERNEL(128, 32, __VA_ARGS__);               \
    else KERNEL(128, 64, __VA_ARGS__);                                              \
  } while (0)

#define GCN_LAYER(K, H, grid, s, A) \
  hipLaunchKernelGGL((gcn_layer_kernel<K, H>), grid, dim3(kGcnLayerThreads), 0, s, A)

hipError_t eh_gcn_layer(const GcnLayerArgs* a, hipStream_t s) {
  if (!a || !a->enode || !a->off || !a->etgt || !a->esrc || !a->deg_s || !a->cnt || !a->h_out || !a->agg_out ||
      !a->wimg || a->cap_t % kGT != 0 || !gcn_kp_ok(a->lin.inp) || !gcn_hp_ok(a->lin.outp) ||
      !gcn_src_ok(a->src, a->lin.inp) || a->lin.in > a->lin.inp || a->lin.out > a->lin.outp)
    return hipErrorInvalidValue;
  const dim3 grid(static_cast<uint32_t>(a->cap_t / kGT));
  GCN_DISPATCH(a->lin.inp, a->lin.outp, GCN_LAYER, grid, s, *a);
  return hipGetLastError();
}

size_t eh_gcn_head_lds(const GcnHeadArgs* a) { return gcn_head_lds_bytes(a->lin.inp, a->lin.outp, a->Ep, a->Cp); }

#define GCN_HEAD(K, H, grid, lds, s, A)                                                                     \
  do {                                                                                                     \
    if ((lds) > 65536)                                                                                     \
      EULER_HIP_CHECK(hipFuncSetAttribute(reinterpret_cast<const void*>(gcn_head_kernel<K, H>),           \
                                          hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(lds))); \
    hipLaunchKernelGGL((gcn_head_kernel<K, H>), grid, dim3(256), lds, s, A);                              \
  } while (0)

hipError_t eh_gcn_head(const GcnHeadArgs* a, hipStream_t s) {
  if (!a || !a->off || !a->etgt || !a->esrc || !a->deg_s || !a->rself || !a->roots || a->B < 1 || !a->wl_img ||
      !a->wfc_img || !a->bfc || !a->wout_img || !a->labels || !a->part_w || !a->part_fc || !a->part_bfc || !a->part_out ||
      !a->part_stat || !gcn_kp_ok(a->lin.inp) || !gcn_hp_ok(a->lin.outp) || !gcn_src_ok(a->src, a->lin.inp) ||
      a->Ep % 32 != 0 || a->Cp % 32 != 0 || a->Ep > 128 || a->Cp > 128 || a->E > a->Ep || a->C > a->Cp ||
      (a->src.by_id && !a->enode) || a->lin.in > a->lin.inp || a->lin.out > a->lin.outp)
    return hipErrorInvalidValue;
  const size_t lds = eh_gcn_head_lds(a);
  if (lds > 160 * 1024) return hipErrorInvalidValue;
  const dim3 grid(static_cast<uint32_t>(ceil_div(a->B, kGT)));
  GCN_DISPATCH(a->lin.inp, a->lin.outp, GCN_HEAD, grid, lds, s, *a);
  return hipGetLastError();
}

#define GCN_DW(K, H, grid, s, A) hipLaunchKernelGGL((gcn_dw_kernel<K, H>), grid, dim3(256), 0, s, A)

hipError_t eh_gcn_dw(const GcnDwArgs* a, int64_t nblk, hipStream_t s) {
  if (!a || !a->dagg || !a->h || !a->agg || !a->off || !a->etgt || !a->esrc || !a->rself || !a->deg_s || !a->part ||
      a->B < 1 || nblk < 1 || nblk * kGcnDwRows < a->cap_e + a->B ||
      !gcn_kp_ok(a->lin.inp) || !gcn_hp_ok(a->lin.outp))
    return hipErrorInvalidValue;
  const dim3 grid(static_cast<uint32_t>(nblk));
  GCN_DISPATCH(a->lin.inp, a->lin.outp, GCN_DW, grid, s, *a);
  return hipGetLastError();
}

hipError_t eh_gcn_reduce(const GcnReduceArgs* a, hipStream_t s) {
  if (!a || a->nseg < 1 || a->nseg > kGcnMaxSegs || a->nblk < 1 || !a->part_stat || a->nstat < 1 || !a->loss_out ||
      !a->counts || !a->stamp || !a->rng)
    return hipErrorInvalidValue;
  for (int k = 0; k < a->nseg; ++k) {
    const GcnRedSeg& g = a->seg[k];
    if (!g.grad || !g.part || g.rows < 1 || g.cols < 1 || g.S < 1 || g.prs < g.cols) return hipErrorInvalidValue;
    if (a->fuse_opt && (!g.p || !g.m || !g.v)) return hipErrorInvalidValue;
  }
  if (a->fuse_opt && !a->ostep) return hipErrorInvalidValue;
  hipLaunchKernelGGL(gcn_reduce_kernel, dim3(static_cast<uint32_t>(a->nblk)), dim3(256), 0, s, *a);
  return hipGetLastError();
}

}  // extern "C"
