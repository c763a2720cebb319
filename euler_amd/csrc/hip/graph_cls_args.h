// Argument blocks of the fused graph-classification training step (graph_cls.hip), shared
// by the kernels and the host binding (binding_graph_cls.cpp).  Plain C++ (no device code).
//
// The step (models/graph_cls_trainer.py) trains the pooled graph-classification models of
// the reference whose convolutions are linear in an aggregate — GIN (reference
// tf_euler/python/convolution/gin_conv.py:26-57, examples/gin/gin.py) and GraphGCN
// (convolution/graph_conv.py:26-46, examples/graphgcn/graphgcn.py) — over the induced
// full-neighbourhood subgraph of each drawn graph, with sparse-feature embedding-bag
// inputs, ReLU after every conv, fc, add pooling, out_fc and the sigmoid cross-entropy of
// mp_utils/base_graph.py:24-47.  Two launches per step:
//
//   gc_step    one block per drawn graph (the draw is the alias table on the graph RNG's
//              Philox stream 3, as alias_sample): every node of the graph stays in LDS for
//              the whole step, and every product is an fp32 MFMA GEMM on LDS operands
//              (v_mfma_f32_16x16x4_f32: exact fp32, the torch oracle's numerics).  The
//              graph's adjacency becomes a dense [n][n] count matrix A per edge-type mask
//              (n <= 64), the node features a dense [n][rows] bag matrix S, so
//                embedding     X0 = S T
//                aggregate     GIN  Z = A X + (1 + eps + self) X
//                              GraphConv  Z = [X | diag(1 / cnt) (A + self I) X]
//                linear        X' = relu(Z [W | Wf]^T + b)
//              then fc, add pooling and out_fc as mat-vecs of the pooled ReLU output, the
//              loss; backward: the pooled head's rank-1 gradients, per conv dW = G^T Z and
//              dZ = G W, the transposed aggregate A^T dZ (masked by the layer below's ReLU
//              in its epilogue), the table gradient S^T dX0.  Every gradient element is
//              written once into the block's slab row (no atomics on global memory).
//   gc_reduce  the B slab rows summed in block order into the flat gradient, or straight
//              into the flat optimizer's update (one process); loss, accuracy, RNG counter.
#pragma once
#include <hip/hip_runtime_api.h>
#include <stdint.h>

namespace euler_hip {

constexpr int kGcMaxLayers = 8;
constexpr int kGcMaxAdj = 4;        // distinct edge-type masks among the layers
constexpr int kGcThreads = 256;
constexpr int kGcMaxRows = 64;      // nodes per graph
constexpr int kGcMaxWidth = 128;    // conv / fc widths
constexpr int kGcMaxLabels = 64;
constexpr int kGcMaxTable = 8192;   // embedding-table elements (staged in LDS)
constexpr int kGcMaxTableRows = 64; // rows of the dense bag matrix S

constexpr int kGcRec = 12;          // ints per graph record: n, feature pairs [f0, f1), per mask edge pairs [e0, e1)

// one edge-type mask's edges of every graph, graph by graph (static, built once): each
// edge t <- s (the flow's full-neighbour expansion of t, repeats kept) as (t << 8) | s in
// local node indices
struct GcAdj {
  const int32_t* pair;
};

struct GcStepArgs {
  int32_t L, B, kind;   // kind 0: GIN, 1: GraphConv
  int32_t self_loops;
  int32_t nmax;         // LDS rows (max nodes per graph, rounded up to 16)
  int32_t D[kGcMaxLayers + 1];  // D[0]: embedding width; D[l + 1]: conv l's width
  int32_t E, C;         // fc width, labels
  int32_t adj_of[kGcMaxLayers];
  int32_t nadj;
  GcAdj adj[kGcMaxAdj];
  // graphs
  int32_t G;
  const float* gprob;   // [G] alias table of the uniform graph draw
  const int32_t* galias;
  const int64_t* rng;   // (seed, counter): this launch draws with counter + 1
  const int32_t* rec;   // [G][kGcRec] graph records
  const int32_t* fpair; // (node << 16) | table row of every feature occurrence, graph by graph
  const float* fw;      // its bag weight (1; 1 / features of the node for the mean combiner)
  const float* onehot;  // [G][C]
  // parameters (flat fp32 views)
  const float* table;   // [tab_rows][D0]
  int32_t tab_rows;
  const float* W[kGcMaxLayers];   // GIN mlp / GraphConv liner weight [D[l+1]][D[l]]
  const float* Wf[kGcMaxLayers];  // GraphConv fc weight [D[l+1]][D[l]]
  const float* bl[kGcMaxLayers];  // GraphConv liner bias [D[l+1]]
  const float* eps[kGcMaxLayers]; // GIN eps (parameter or buffer), one float
  const float* Wfc;     // [E][D[L]]
  const float* bfc;     // [E]
  const float* Wout;    // [C][E]
  // slab offsets (elements of the flat parameter buffer) of every gradient; -1: none
  int64_t o_W[kGcMaxLayers], o_Wf[kGcMaxLayers], o_bl[kGcMaxLayers], o_eps[kGcMaxLayers];
  int64_t o_fc, o_bfc, o_out, o_tab;
  // outputs
  float* slab;          // [B][S]
  int64_t S;
  float* loss_part;     // [B]
  float* acc_part;      // [B] 1 when the arg-max class is the label's
  int32_t* gidx;        // [B] the drawn graphs
  int64_t* ostep_inc;   // block 0 advances the optimizer's step (the fused update reads it)
  float inv_scale;      // 1 / (B C)
  // LDS layout (bytes), computed by the host: activations X_l [nmax][ldx], Z [nmax][ldz]
  // (one per conv when zst, else one recomputed in the backward), dZ, d(out) / G [nmax][ldy],
  // A [nadj][nmax][lda], 1 / cnt [nadj][nmax], S [nmax][lds], the table [trp][ldt]
  int32_t lds_x[kGcMaxLayers + 1], lds_z, lds_dy, lds_dz, lds_vec, lds_a, lds_invc, lds_s, lds_t, lds_csum, lds_bytes;
  int32_t ldx[kGcMaxLayers + 1], ldz, ldy, lda, ldsm, ldt, trp;
  int32_t zst;
  // the flat parameter buffer: each XCD's blocks touch it once at the start (L2 warm-up)
  const float* warm;
  int64_t warm_n;
  long long* prof;      // [B][32] phase wall-clock stamps (diagnostics; null in training)
};

struct GcReduceArgs {
  const float* slab;
  int64_t S;
  int32_t B;
  float* grad;          // [S] flat gradient (fuse_opt 0)
  const float* loss_part;
  const float* acc_part;
  float* loss_out;
  double* right;        // (correct, total)
  int64_t* rng;         // counter advanced by one
  // fused flat optimizer
  int32_t fuse_opt, okind;
  float* p;
  float* m;
  float* v;
  const int64_t* ostep;
  float lr, b1, b2, eps, wd, grad_scale;
};

}  // namespace euler_hip

extern "C" {
hipError_t eh_gc_step(const euler_hip::GcStepArgs* a, hipStream_t s);
hipError_t eh_gc_reduce(const euler_hip::GcReduceArgs* a, hipStream_t s);
}
