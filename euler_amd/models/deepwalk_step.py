"""DeepWalk / node2vec(p = q = 1) skip-gram training step on the GPU with row-sharded
embedding tables (BASELINE config 4: 128-d embeddings, 100M nodes, DP over RCCL with an
embedding all-to-all).

Reference model: examples/deepwalk/deepwalk.py:27-99 — ``random_walk`` (walk_len, p, q)
-> ``gen_pair`` (left/right window) -> negatives from ``sample_node`` (batch x pairs x
num_negs) -> target embedding of the centre, context embedding of the positive and the
negatives -> sigmoid CE (mp_utils/base.py:80-91) -> Adam on the (PS-partitioned) tables.

One step here, per rank (no autograd, no dense table gradient):

  1. walks    : ``random_walk_kernel`` from ``batch`` alias-sampled start nodes
  2. pairs    : skip-gram (centre, context) pairs of every walk; negatives per pair
  3. unique   : hash-table unique of the centre ids and of the context+negative ids,
                plus the occurrence lists of every unique id (occ_csr)
     (one row-sharded table holds target rows [0, N] and context rows [N+1, 2N+1])
  4. loss     : ``sgns_fwd_idx`` — logits straight from the table rows through the two-level
                (occurrence -> unique id -> row) index; emits only coef = dloss/dlogit
  5. update   : per unique row, the gradient is rebuilt from its occurrence list and
                applied in place (``sgns_update``: row-sparse Adam/Adagrad/SGD) — no
                per-pair gradient rows, no zero-filled accumulator, no float atomics.
                Target rows are updated first from the (not yet updated) context table;
                the context update reads a copy of the pre-update target rows.
     world > 1: rows come from ShardedTable.lookup (RCCL all-to-all), ``sgns_grad`` builds
                the per-unique-row gradients from the looked-up rows and
                ShardedTable.apply sends them to the owners.

Padding: a walk that hits a node without out-edges continues with the pad row
``num_nodes`` (the reference's ``max_id + 1`` default node).

Static mode (``static=True``): the unique id sets are fixed-capacity (padded with -1 by
``unique_first_padded``, count kept on the device), occurrence lists are built over the
capacities, and with collectives the table exchange is ShardedTable.lookup_static /
apply_static (equal-split all-to-alls of W x C slots).  No step size is read back to the
host, so :meth:`capture` records the whole step — sampling, unique, (all-to-all), loss,
row-sparse update — into one hipGraph that :meth:`step` replays.
"""
from __future__ import annotations

import torch

import euler_amd.ops.graph_api as ge
from euler_amd.ops import gnn_ops
from euler_amd.ops._native import hip, use_hip
from euler_amd.parallel.sparse_table import ShardedTable
from euler_amd.models.captured import new_graph

__all__ = ["DeepWalkTrainer", "DeepWalkEstimatorTrainer"]


def _pair_positions(walk_len, left, right):
    pairs = ge.gen_pair(torch.arange(walk_len + 1).view(1, -1), left, right)[0]
    return pairs[:, 0].clone(), pairs[:, 1].clone()


def _row_sum(x):
    """Sum of a 1-D loss vector in two passes when it splits into 256-wide rows: torch's
    one-shot reduction of the ~98 K per-pair losses runs in a single 512-lane block (27 us
    per step on the 100M-node bench, profiles/r5_zoo/occ_csr_fused/README.txt)."""
    n = x.numel()
    if n >= 4096 and n % 256 == 0:
        return x.view(-1, 256).sum(1).sum()
    return x.sum()


class DeepWalkTrainer:
    def __init__(self, graph, num_nodes, dim=128, walk_len=3, left_win_size=1, right_win_size=1, num_negs=5,
                 batch_size=1024, lr=0.01, optimizer="adam", group=None, seed=0, force_comm=False, static=False,
                 wire_dtype="bf16", overflow_check_every=200, micro_batches=1, edge_types=None, p=1.0, q=1.0,
                 row_map=None, table_init="normal", table_slots=True):
        import torch.distributed as dist

        self.graph = graph
        self.edge_types, self.p, self.q = edge_types, float(p), float(q)
        self.num_nodes = int(num_nodes)
        self.pad = self.num_nodes  # rows: num_nodes + 1 (pad row like the reference's max_id + 1)
        self.dim, self.walk_len, self.num_negs, self.batch = int(dim), int(walk_len), int(num_negs), int(batch_size)
        dev = graph.device
        self.device = dev
        # row_map [graph rows + 1]: table row of every graph row (the last entry: the walk's
        # pad, graph row num_rows) when the table rows are not the graph rows (model ids)
        self.row_map = None if row_map is None else torch.as_tensor(row_map, dtype=torch.int64).to(dev)
        # ONE row-sharded table holds both embeddings: target row of node i is row i, its
        # context row is row off + i.  A step then needs one id exchange, one row exchange,
        # one gradient exchange and one host sync (world > 1) instead of two of each.  off is
        # a multiple of the world size, so each half is itself mod-sharded: this rank's target
        # rows and context rows are two contiguous blocks of its shard with the same layout as
        # a ShardedEmbedding of the half (model tables can be views of them, checkpoints
        # write each half as the model's table)
        world = dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1
        self.off = -(-(self.num_nodes + 1) // world) * world
        self.table = ShardedTable(2 * self.off, dim, dev, group, optimizer, lr, seed=seed, force_comm=force_comm,
                                  wire_dtype=wire_dtype, init=table_init, slots=table_slots)
        pi, pj = _pair_positions(walk_len, left_win_size, right_win_size)
        self.pi, self.pj = pi.to(dev), pj.to(dev)
        self.pairs_per_walk = int(pi.numel())
        self.loss = torch.zeros((), device=dev)
        self.static = bool(static)
        self.hip_graph = None
        # static mode: read the exchange's device overflow flag every N steps (one host
        # sync) so a dropped id fails loudly instead of silently training less
        self.overflow_check_every = int(overflow_check_every)
        self.steps_done = 0
        # static mode with collectives: 2 = two micro-batches per step whose exchanges run
        # on a comm stream under the other micro-batch's sampling / SGNS compute
        if micro_batches not in (1, 2) or (micro_batches == 2 and self.batch % 2):
            raise ValueError("micro_batches must be 1 or 2 (2 needs an even batch)")
        self.micro_batches = int(micro_batches)
        self._xstream = None
        self._keep = None

    def _gather(self, rows, inv):
        if use_hip(rows, inv):
            return hip().gather_rows(rows, inv.contiguous())
        return rows[inv]

    def sample(self, batch=None):
        """(centre [P], positive [P], negatives [P, K]) global ids of one step."""
        g = self.graph
        g.advance()
        starts = g.sample_node(self.batch if batch is None else int(batch), stream_id=1)
        # a pad at or past the graph's rows ends a walk like -1 does (no row to step from), so
        # the walk kernel writes it directly: no compare / fill / where per step
        pad = g.num_rows if self.row_map is not None else self.pad
        direct = pad >= g.num_rows
        walks = g.random_walk(starts, self.walk_len, edge_types=self.edge_types, default=pad if direct else -1,
                              stream_id=3, p=self.p, q=self.q).long()
        if not direct:
            walks = torch.where(walks < 0, torch.full_like(walks, pad), walks)
        src = walks[:, self.pi].reshape(-1)
        pos = walks[:, self.pj].reshape(-1)
        negs = g.sample_node(src.numel() * self.num_negs, stream_id=4).long().view(-1, self.num_negs)
        if self.row_map is not None:  # graph rows -> table rows (model ids)
            src, pos, negs = self.row_map[src], self.row_map[pos], self.row_map[negs]
        return src, pos, negs

    def step(self):
        self.steps_done += 1
        if self.static and self.overflow_check_every > 0 and self.steps_done % self.overflow_check_every == 0:
            self.table.check_overflow()
        if self.hip_graph is not None:
            self.hip_graph.replay()
            return self.loss
        return self._step_static() if self.static else self._step_dynamic()

    def capture(self, warm=2):
        """Record one static step into a hipGraph (after ``warm`` real eager steps on a side
        stream, which allocate the kernels' workspaces; ``warm_loss`` is the last one's
        loss); later :meth:`step` calls replay it.  Capturing executes nothing, so
        ``self.loss`` (the graph's output) is valid after the first replay."""
        if not (self.static and self.device.type == "cuda"):
            raise ValueError("capture needs static=True on a GPU")
        cur = torch.cuda.current_stream()
        side = torch.cuda.Stream()
        side.wait_stream(cur)
        with torch.cuda.stream(side):
            for _ in range(int(warm)):
                self.warm_loss = self._step_static()
        cur.wait_stream(side)
        g = new_graph()
        with torch.cuda.graph(g, capture_error_mode="thread_local"):
            self._step_static()
        self.hip_graph = g
        return g

    def release(self):
        """Drop the captured graph (do this before destroying a process group whose
        collectives it recorded: a live graph keeps the communicator's work pending)."""
        if self.hip_graph is not None:
            torch.cuda.synchronize()
            self.hip_graph.reset()
            self.hip_graph = None

    def _step_static(self):
        if self.micro_batches == 2 and self.table.comm:
            return self._step_static_overlapped()
        src, pos, negs = self.sample()
        P, K = src.numel(), self.num_negs
        gscale = 1.0 / (P * (1 + K))
        u_t, inv_t, _ = gnn_ops.unique_first_padded(src)
        # context ids straight as their table rows (off + id; padding stays -1)
        rows_c_id, inv_c, _ = gnn_ops.unique_first_padded(torch.cat([pos, negs.reshape(-1)]), offset=self.off)
        tab = self.table
        if tab.fused_sgns_ok(u_t):
            ptr_t, lst_t = gnn_ops.occ_csr(inv_t, u_t.numel())
            ptr_c, lst_c = gnn_ops.occ_csr(inv_c, rows_c_id.numel())
            W = tab.weight
            coef, loss_rows = gnn_ops.sgns_fwd_idx(W, u_t, inv_t, W, rows_c_id, inv_c, K, gscale)
            rt = self._gather(W, u_t)                       # pre-update target rows (pad: zero)
            tab.apply_sgns(0, ptr_t, lst_t, coef, K, W, rows_c_id, inv_c, u_t)
            tab.apply_sgns(1, ptr_c, lst_c, coef, K, rt, None, inv_t, rows_c_id, inc_step=False)
        else:
            ids = torch.cat([u_t, rows_c_id])
            # rows [W*C + 1, D]: the extra zero row is the trash slot of ids dropped by a
            # capacity overflow (pos = W*C), so they never alias a live slot
            rows, h = tab.lookup_static(ids, trash_row=True, keep_wire=True)
            n = rows.shape[0]
            tinv = h.pos[inv_t]
            cinv = h.pos[u_t.numel() + inv_c]
            coef, loss_rows = gnn_ops.sgns_fwd_idx(rows, None, tinv, rows, None, cinv, K, gscale)
            ptr_t, lst_t = gnn_ops.occ_csr(tinv, n)
            ptr_c, lst_c = gnn_ops.occ_csr(cinv, n)
            # every occupied live slot is written by exactly one side (target and context ids
            # live in different table halves); empty slots (local row -1) are skipped by the
            # update, so no 4*D*W*C-byte zero fill per step; the trash row is not applied
            g = torch.empty_like(rows)
            gnn_ops.sgns_grad(0, ptr_t, lst_t, coef, K, rows, None, cinv, inv_self=tinv, out=g)
            gnn_ops.sgns_grad(1, ptr_c, lst_c, coef, K, rows, None, tinv, inv_self=cinv, out=g)
            tab.apply_static(h, g[: n - 1])
        self.loss = _row_sum(loss_rows) * gscale
        return self.loss

    # ------------------------------------------------------------------ overlapped static step
    def _mb_front(self, nb):
        """sample + unique + owner routing of one micro-batch (no collective)"""
        src, pos, negs = self.sample(nb)
        u_t, inv_t, _ = gnn_ops.unique_first_padded(src)
        # context ids straight as their table rows (off + id; padding stays -1)
        rows_c_id, inv_c, _ = gnn_ops.unique_first_padded(torch.cat([pos, negs.reshape(-1)]), offset=self.off)
        routed = self.table.route_static(torch.cat([u_t, rows_c_id]))
        return {"P": src.numel(), "inv_t": inv_t, "inv_c": inv_c, "nt": u_t.numel(), "routed": routed}

    def _mb_compute(self, mb, rows, h):
        """SGNS loss + per-slot gradients of one micro-batch from its exchanged rows"""
        K = self.num_negs
        gscale = 1.0 / (mb["P"] * (1 + K))
        n = rows.shape[0]
        tinv = h.pos[mb["inv_t"]]
        cinv = h.pos[mb["nt"] + mb["inv_c"]]
        coef, loss_rows = gnn_ops.sgns_fwd_idx(rows, None, tinv, rows, None, cinv, K, gscale)
        ptr_t, lst_t = gnn_ops.occ_csr(tinv, n)
        ptr_c, lst_c = gnn_ops.occ_csr(cinv, n)
        g = torch.empty_like(rows)
        gnn_ops.sgns_grad(0, ptr_t, lst_t, coef, K, rows, None, cinv, inv_self=tinv, out=g)
        gnn_ops.sgns_grad(1, ptr_c, lst_c, coef, K, rows, None, tinv, inv_self=cinv, out=g)
        return g[: n - 1], _row_sum(loss_rows) * gscale, (coef, ptr_t, lst_t, ptr_c, lst_c, g)

    def _step_static_overlapped(self):
        """Two micro-batches of batch/2 walks.  The calling stream S runs every collective
        and table access in order: front0, exchange0, exchange1, apply0, apply1; a forked
        compute stream X runs front1 (under exchange0), compute0 (under exchange1) and
        compute1 (under apply0).  Micro-batch 1 reads its rows before micro-batch 0's
        update lands (the full-batch step reads every row before its single update); every
        rank issues the collectives in the same order.  Each micro-batch applies its own
        row-sparse optimizer update."""
        tab = self.table
        S = torch.cuda.current_stream(self.device) if self.device.type == "cuda" else None
        if S is None:  # CPU (gloo): the same phases in order on one stream
            m0 = self._mb_front(self.batch // 2)
            r0 = tab.exchange_static(m0["routed"], trash_row=True, keep_wire=True)
            m1 = self._mb_front(self.batch // 2)
            r1 = tab.exchange_static(m1["routed"], trash_row=True, keep_wire=True)
            g0, l0, _ = self._mb_compute(m0, *r0)
            tab.apply_static(r0[1], g0)
            g1, l1, _ = self._mb_compute(m1, *r1)
            tab.apply_static(r1[1], g1)
            self.loss = 0.5 * (l0 + l1)
            return self.loss
        if self._xstream is None:
            self._xstream = torch.cuda.Stream(device=self.device)
            # per micro-batch exchange buffers: allocated by the first (eager) step, reused
            # by every later step and by the capture
            self._bufs = ({}, {})
        # collectives stay on the calling (capture-origin) stream S; the micro-batches'
        # sampling / SGNS compute forks onto X (a capture with RCCL all-to-alls issued on a
        # side stream crashed in capture_end on this ROCm: profiles/r3_deepwalk/)
        X = self._xstream
        ev = [torch.cuda.Event() for _ in range(5)]
        m0 = self._mb_front(self.batch // 2)                                   # S
        ev[0].record(S)
        with torch.cuda.stream(X):
            X.wait_event(ev[0])
            m1 = self._mb_front(self.batch // 2)                               # X, under exchange 0
            ev[1].record(X)
        r0 = tab.exchange_static(m0["routed"], trash_row=True, bufs=self._bufs[0],
                                keep_wire=True)  # S
        ev[2].record(S)
        with torch.cuda.stream(X):
            X.wait_event(ev[2])
            g0, l0, k0 = self._mb_compute(m0, *r0)                            # X, under exchange 1
            ev[3].record(X)
        S.wait_event(ev[1])
        r1 = tab.exchange_static(m1["routed"], trash_row=True, bufs=self._bufs[1],
                                keep_wire=True)  # S
        S.wait_event(ev[3])
        ev[4].record(S)
        with torch.cuda.stream(X):
            X.wait_event(ev[4])
            g1, l1, k1 = self._mb_compute(m1, *r1)                            # X, under apply 0
        tab.apply_static(r0[1], g0, bufs=self._bufs[0])                        # S
        S.wait_stream(X)
        tab.apply_static(r1[1], g1, bufs=self._bufs[1])                        # S
        # every intermediate stays referenced until the next step: tensors made on one
        # stream and read on the other are never handed back to the allocator mid-step
        self._keep = (m0, m1, r0, r1, g0, g1, k0, k1)
        self.loss = 0.5 * (l0 + l1)
        return self.loss

    def _step_dynamic(self):
        src, pos, negs = self.sample()
        P, K = src.numel(), self.num_negs
        gscale = 1.0 / (P * (1 + K))
        # unique ids per role (first-occurrence order; hash kernel on the GPU)
        u_t, inv_t = gnn_ops.unique_first(src)
        u_c, inv_c = gnn_ops.unique_first(torch.cat([pos, negs.reshape(-1)]))
        n_t = u_t.numel()
        tab = self.table
        rows_c_id = u_c + self.off
        if tab.fused_sgns_ok(u_t):
            # one rank owns every row: local row == table row
            ptr_t, lst_t = gnn_ops.occ_csr(inv_t, n_t)
            ptr_c, lst_c = gnn_ops.occ_csr(inv_c, u_c.numel())
            W = tab.weight
            coef, loss_rows = gnn_ops.sgns_fwd_idx(W, u_t, inv_t, W, rows_c_id, inv_c, K, gscale)
            rt = self._gather(W, u_t)                       # pre-update target rows
            tab.apply_sgns(0, ptr_t, lst_t, coef, K, W, rows_c_id, inv_c, u_t)
            tab.apply_sgns(1, ptr_c, lst_c, coef, K, rt, None, inv_t, rows_c_id, inc_step=False)
        else:
            # target and context rows in one exchange (the id sets are disjoint); rows stay
            # in the owner-sorted order they arrive in and the index arrays are remapped, so
            # the gradients come out in send order (no [n, D] permutations)
            rows, h = tab.lookup(torch.cat([u_t, rows_c_id]), sorted_out=True)
            n = rows.shape[0]
            tinv = h.rank[inv_t]
            cinv = h.rank[n_t + inv_c]
            coef, loss_rows = gnn_ops.sgns_fwd_idx(rows, None, tinv, rows, None, cinv, K, gscale)
            ptr_t, lst_t = gnn_ops.occ_csr(tinv, n)
            ptr_c, lst_c = gnn_ops.occ_csr(cinv, n)
            g = torch.empty_like(rows)   # every row is a target row or a context row
            gnn_ops.sgns_grad(0, ptr_t, lst_t, coef, K, rows, None, cinv, inv_self=tinv, out=g)
            gnn_ops.sgns_grad(1, ptr_c, lst_c, coef, K, rows, None, tinv, inv_self=cinv, out=g)
            tab.apply(h, g, sorted_in=True)
        self.loss = _row_sum(loss_rows) * gscale
        return self.loss

    def pairs_per_step(self):
        return self.batch * self.pairs_per_walk

    def embedding(self, ids):
        """target embeddings of global ids (inference)."""
        u, inv = gnn_ops.unique_first(ids.reshape(-1).long())
        rows, _ = self.table.lookup(u)
        return rows[inv].view(*ids.shape, self.dim)

    def context_embedding(self, ids):
        u, inv = gnn_ops.unique_first(ids.reshape(-1).long())
        rows, _ = self.table.lookup(u + self.off)
        return rows[inv].view(*ids.shape, self.dim)


def _id_table(enc):
    """(table module, sharded) of a pure id encoder: an IdEncoder (ShardedEmbedding when
    sharded) or a ShallowEncoder with only an id embedding and combiner 'add'; None if the
    encoder has features"""
    from euler_amd.models.unsupervised import IdEncoder

    if isinstance(enc, IdEncoder):
        if enc.table is not None:
            return enc.table, True
        enc = enc.enc
    if enc is None or not getattr(enc, "use_id", False) or getattr(enc, "use_feature", True) or \
            getattr(enc, "use_sparse_feature", True) or enc.combiner != "add":
        return None
    return enc.embedding, False


class DeepWalkEstimatorTrainer:
    """``NodeEstimator(device_graph=True)`` for DeepWalk / Node2Vec and second-order LINE
    models with id embeddings (reference examples/deepwalk/deepwalk.py:27-99,
    examples/line/line.py:27-71 through
    euler_estimator/python/node_estimator.py): the walks, pairs, negatives and the
    row-sparse SGNS update of :class:`DeepWalkTrainer` on the HBM graph, several static
    steps per hipGraph replay.

    Table ownership: the trainer's row-sharded table holds target rows [0, off) and context
    rows [off, 2 off) in MODEL row space (model id i; the pad row is the model's
    ``max_id + 1``; graph rows are mapped to model ids on the device when they differ).
    ``off`` is a multiple of the world size, so this rank's rows of each half are a
    contiguous block laid out exactly like a ``mod``-sharded table of the half.  Whenever the
    model's table has that layout — a ``sharded=True`` model (ShardedEmbedding, any world
    size) or any model on one rank — the model's weight becomes a VIEW of that block: no
    second copy of a table exists while the trainer trains it (a 100M x 128 table pair is
    102 GB).  Only a dense (non-sharded) model under 2+ ranks keeps its own full table,
    written from the shards when training ends.

    Data parallel (the reference's ``mod``-partitioned PS embedding variables,
    tf_euler/python/utils/embedding.py:24-68): every step's rows travel over fixed-capacity
    all-to-alls and only the touched rows are updated; each rank draws its own walks (its
    own Philox key).  Checkpoints are per-rank shards (parallel/shard_io.py): every rank
    writes its rows of each table and their sparse-optimizer slots, and a restore under any
    world size reads exactly its own rows from them — no all-gather anywhere."""

    metric_name = "loss"
    self_synced = True  # no dense gradient for the estimator to all-reduce

    def __init__(self, model, graph, batch_size, optimizer="adam", learning_rate=0.01, seed=0):
        import numpy as np

        import euler_amd.ops.graph_api as ge

        enc_t, enc_c = getattr(model, "_target_encoder", None), getattr(model, "_context_encoder", None)
        tabs = [_id_table(e) for e in (enc_t, enc_c)]
        if any(t is None for t in tabs):
            raise ValueError("the DeepWalk device path trains pure id embeddings (no features, combiner 'add')")
        if enc_t is enc_c or tabs[0][0] is tabs[1][0]:
            raise ValueError("the DeepWalk device path needs separate target and context tables "
                             "(LINE: order='second')")
        self.model = model
        self.graph = graph
        self.device = graph.device
        self.on_gpu = self.device.type == "cuda"
        self._mods = [t for t, _ in tabs]
        self._sharded = tabs[0][1]
        self.num = int(self._mods[0].num)  # model rows per table: max_id + 2 (pad row max_id + 1)
        if int(self._mods[1].num) != self.num or self.num != int(model.max_id) + 2:
            raise ValueError("DeepWalk tables must have max_id + 2 rows (the pad row is max_id + 1)")
        names = {id(p): k for k, p in model.named_parameters()}
        self._keys = tuple(names[id(m.weight)] for m in self._mods)
        et = model.edge_type
        ets = None if et in (None, -1, "-1") else [int(t) for t in np.asarray(ge.get_edge_type_id(et)).reshape(-1)]
        # graph row -> model row, unless graph row r is node id r for every row
        ids = graph.ids
        row_map = None
        if ids is not None:
            ids = np.asarray(ids).astype(np.int64)
            if ids.size and (ids.max() > model.max_id or ids.min() < 0):
                raise ValueError("graph node ids beyond the model's max_id")
            if not np.array_equal(ids, np.arange(ids.size)):
                row_map = np.concatenate([ids, [self.num - 1]])
        elif graph.num_rows > self.num - 1:
            raise ValueError("graph rows beyond the model's max_id")
        # LINE (second order, examples/line/line.py:27-71): the positive of a root is one
        # weighted neighbour sample (UnsuperviseModel.to_sample) = the second node of a
        # one-step walk, paired (root, neighbour) only: walk_len 1, window (0, 1)
        walk_len = getattr(model, "walk_len", 1)
        win = (getattr(model, "left_win_size", 0), getattr(model, "right_win_size", 1))
        self.inner = DeepWalkTrainer(graph, self.num - 1, dim=model.dim, walk_len=walk_len,
                                     left_win_size=win[0], right_win_size=win[1],
                                     num_negs=model.num_negs, batch_size=batch_size, lr=learning_rate,
                                     optimizer=optimizer, seed=seed, static=self.on_gpu, edge_types=ets,
                                     p=getattr(model, "walk_p", 1), q=getattr(model, "walk_q", 1),
                                     row_map=row_map, table_init=None, table_slots=False)
        t = self.inner.table
        self._offw = self.inner.off // t.world  # local rows per half
        self._pad_rows()
        # the model's tables become views of the trainer's halves (same layout) — or, for a
        # dense model under 2+ ranks, this rank's rows are copied in
        self._bound = self._sharded or t.world == 1
        with torch.no_grad():
            for h, mod in enumerate(self._mods):
                w = mod.weight
                if self._bound:
                    n = int(w.shape[0])
                    view = t.weight[h * self._offw: h * self._offw + n]
                    view.copy_(w.detach().to(view))
                    w.data = view
                else:
                    rows = self._half_rows()
                    ok = rows < self.num
                    t.weight[h * self._offw: (h + 1) * self._offw][ok] = w.detach()[rows[ok].to(w.device)].to(t.weight)
        # slots only now: the model's own table storage is gone when the tables are views
        t.alloc_slots()
        self.loss_sum = torch.zeros(2, dtype=torch.float64, device=self.device)
        self._graphs, self._graph_loss, self._graph_exec = {}, {}, None
        self._loss = torch.zeros((), device=self.device)
        self.step_count = 0
        self.captures = 0

    # ------------------------------------------------------------------ table <-> model
    def _half_rows(self):
        """model row of each of this rank's local rows of one half"""
        t = self.inner.table
        return torch.arange(self._offw, device=self.device) * t.world + t.rank

    def _pad_rows(self):
        """zero the alignment rows [num, off) of both halves (never drawn, never trained)"""
        t = self.inner.table
        rows = self._half_rows()
        dead = torch.nonzero(rows >= self.num).reshape(-1)
        with torch.no_grad():
            for h in range(2):
                t.weight[h * self._offw + dead] = 0.0

    def logical_keys(self):
        return set(self._keys)

    def load_logical(self, sd):
        """model-named tables: this rank's rows (a ShardedEmbedding's shard) or the whole
        table (a dense model's, or one saved by a single rank)"""
        t = self.inner.table
        rows = self._half_rows()
        ok = rows < self.num
        with torch.no_grad():
            for h, key in enumerate(self._keys):
                if key not in sd:
                    continue
                w = torch.as_tensor(sd[key])
                dst = t.weight[h * self._offw: (h + 1) * self._offw]
                if int(w.shape[0]) == self.num:
                    dst[ok] = w[rows[ok].cpu()].to(dst)
                elif int(w.shape[0]) == int(ok.sum()):
                    dst[: w.shape[0]] = w.to(dst)
                else:
                    raise ValueError(f"{key}: {tuple(w.shape)} is neither the table nor this rank's shard")

    def _full_table(self, h):
        """the whole table ``h`` (dense model under 2+ ranks: an all-gather)"""
        t = self.inner.table
        half = t.weight[h * self._offw: (h + 1) * self._offw]
        if t.world == 1:
            return half[: self.num]
        import torch.distributed as dist

        parts = [torch.empty_like(half) for _ in range(t.world)]
        dist.all_gather(parts, half.contiguous(), group=t.group)
        return torch.stack(parts, 1).reshape(-1, t.dim)[: self.num]

    def write_to_model(self, model):
        """views: nothing to copy; a dense model under 2+ ranks gets the gathered tables
        (a collective — at the end of training, never per checkpoint)"""
        if self._bound and model is self.model:
            return
        own = model.state_dict()
        with torch.no_grad():
            for h, key in enumerate(self._keys):
                full = self._full_table(h)
                own[key].copy_(full.to(own[key]) if own[key].shape[0] == full.shape[0] else
                               self.inner.table.weight[h * self._offw: h * self._offw + own[key].shape[0]])

    def finish(self):
        self.write_to_model(self.model)

    def state_dict(self):
        self.write_to_model(self.model)
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items()}

    def logical_params(self):
        return self.state_dict()

    # ------------------------------------------------------------------ per-rank checkpoints
    def checkpoint_model_state(self):
        """the model's state without its id tables (they go to the per-rank shard files)"""
        return {k: v.detach().cpu() for k, v in self.model.state_dict().items() if k not in self._keys}

    def checkpoint_shards(self, ckpt_path):
        """write this rank's rows of both tables and their optimizer slots next to
        ``ckpt_path``; returns the per-table metadata for the checkpoint file"""
        t = self.inner.table
        return {key: t.save_shard(ckpt_path, key, num=self.num, lo=h * self._offw)
                for h, key in enumerate(self._keys)}

    def load_shards(self, dirname, metas):
        """this rank's rows of both tables (and slots) from a checkpoint of any world size"""
        t = self.inner.table
        for h, key in enumerate(self._keys):
            if key in metas:
                t.load_shard(dirname, metas[key], lo=h * self._offw, n_local=self._offw, name=key)
        self._pad_rows()

    # ------------------------------------------------------------------ steps
    def _one(self):
        loss = self.inner._step_static() if self.inner.static else self.inner._step_dynamic()
        self.loss_sum += torch.stack([loss.detach().double(), torch.ones((), dtype=torch.float64,
                                                                         device=self.device)])
        return loss

    def step(self, grad_sync=None):
        self.step_count += 1
        if self._graph_exec is not None:
            self._graph_exec.replay()
            self._loss = self._graph_loss[1]
            return self._loss
        self._loss = self._one()
        return self._loss

    def capture(self, grad_sync=None, warmup=2, steps=1, extra_sizes=()):
        if not self.on_gpu:
            return None
        s = torch.cuda.Stream(device=self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self.step_count += 1
                self._loss = self._one()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        self._graphs, self._graph_loss = {}, {}
        for k in sorted({1, int(steps)} | {int(e) for e in extra_sizes if int(e) > 0}, reverse=True):
            gr = new_graph()
            with torch.cuda.graph(gr, capture_error_mode="thread_local"):
                for _ in range(k):
                    out = self._one()
            self._graphs[k], self._graph_loss[k] = gr, out
        self._graph_exec = self._graphs[1]
        self.captures += 1
        return self._graphs[int(steps)]

    def replay(self, n=1):
        for _ in range(int(n)):
            self._graph_exec.replay()
        self._loss = self._graph_loss[1]
        self.step_count += int(n)

    def replay_steps(self, n):
        left = int(n)
        for k in sorted(self._graphs, reverse=True):
            while left >= k:
                self._graphs[k].replay()
                self._loss = self._graph_loss[k]
                left -= k
        self.step_count += int(n)

    def release_graphs(self):
        for g in self._graphs.values():
            g.reset()
        self._graphs, self._graph_loss, self._graph_exec = {}, {}, None

    # ------------------------------------------------------------------ state
    @property
    def loss(self):
        return self._loss

    def metric(self) -> float:
        s, n = self.loss_sum.tolist()
        return s / max(n, 1.0)

    def reset_metric(self):
        self.loss_sum.zero_()

    def samples(self):
        return None

    def trainer_state(self):
        """step and sampler counter (the tables and their slots are in the shard files)"""
        t = self.inner.table
        return {"step": int(t.step.item()), "rng": self.graph.rng.detach().cpu().clone()}

    def load_trainer_state(self, st):
        t = self.inner.table
        t.step.fill_(int(st["step"]))
        self.graph.rng.copy_(torch.as_tensor(st["rng"]).to(self.graph.rng))
        self.step_count = int(st["step"])

    def dp_state_tensors(self):
        t = self.inner.table
        return [t.weight, t.m, t.v, t.step]

    def set_learning_rate(self, lr):
        self.inner.table.lr = float(lr)
