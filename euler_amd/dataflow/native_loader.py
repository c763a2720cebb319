"""Native mini-batch pipeline for the engine (CPU-sampling) GraphSAGE path.

C++ worker threads (``_engine.SagePipeline``, csrc/pipeline/pipeline.cc; no GIL) build
complete batches — roots, every SageDataFlow hop (sampling, unique, edge list), the
outermost node set's dense input features and the roots' labels — into pinned slot
buffers that are allocated once and reused.  The consumer side here only wraps a ready
slot in tensor views, issues the H2D copies on a side stream (``non_blocking``), makes
the compute stream wait on that copy's event, and returns the slot to the workers once
the copy has completed (event polled, never a host sync on the compute stream).  Slots:
``workers + 3`` by default (every worker filling one, two copies in flight, one being
handed out).

Reference mechanics replaced: the reference builds the same batch inside the TF graph
with one GQL op per hop plus one per feature (tf_euler/kernels/
sample_fanout_with_feature_op.cc:43-69, get_dense_feature_op.cc:89-116) serially with
the step; the round-1 Python prefetcher called ``pin_memory()`` on every batch.

Batch b is drawn with the keyed samplers (Philox key (seed, b, hop); roots through virtual
node buckets, neighbours keyed by (id, occurrence); csrc/graph/keyed.cc) and delivered in
order, so the batch stream is reproducible for any worker count and identical whether the
graph is in-process or on shard servers.

Remote sessions (``initialize_shared_graph``; also ``local_sharded``): the same workers
build the batch through the session's distribute-mode GQL plans — one roots (+ labels)
query, one ``sampleNB`` query per hop over the hop's unique frontier and one ``values``
query for the outermost nodes, each one RPC per shard (csrc/pipeline/pipeline.cc
RemoteSource; reference tf_euler/kernels/sample_fanout_with_feature_op.cc:43-69 +
euler/core/kernels/remote_op.cc:60-146) — so W workers keep W batches of RPCs in flight
and the step still only consumes ready slots.  The servers draw with the batch's keys
(``sampleNodeAt`` / keyed ``sampleNB``), so a remote batch equals the local one.

Static mode (``static=True``, GPU only) serves every batch through ONE set of
fixed-capacity device tensors, the inputs of a graph-captured training step
(estimator/graph_step.py): the slot's ``res`` / ``nbr`` are padded with -1 up to the
level capacities by the C++ writer, the H2D copy lands in one of two device staging
sets on the side stream, and a device-to-device copy on the compute stream moves it into
the static set right before the replay (the staging set is reused only after that copy
has run, tracked by an event).  ``get()`` then returns the same ``Prepared`` every time.
"""
from __future__ import annotations

import numpy as np
import torch

from euler_amd.dataflow.dataflows import Block, DataFlow
from euler_amd.mp_utils.models import Prepared
from euler_amd.ops.base import get_engine

__all__ = ["NativeSageLoader", "native_spec"]


def _names(x):
    if x is None:
        return []
    return [x] if isinstance(x, str) else list(x)


def native_spec(model, params):
    """(flow, dense names, dims, label, label_dim, node_type) for models the native
    pipeline serves (SupervisedGNN with a SageDataFlow); None otherwise."""
    from euler_amd.dataflow.dataflows import SageDataFlow

    gnn = getattr(model, "gnn", None)
    flow = getattr(gnn, "sampler", None)
    if not isinstance(flow, SageDataFlow) or not hasattr(model, "label_idx"):
        return None
    names, dims = _names(getattr(gnn, "feature_idx", None)), getattr(gnn, "feature_dim", None)
    dims = [int(dims)] * len(names) if isinstance(dims, int) else [int(d) for d in (dims or [])]
    if not names or len(names) != len(dims):
        return None
    return flow, names, dims, model.label_idx, int(model.label_dim), params.get("train_node_type", -1)


class NativeSageLoader:
    def __init__(self, flow, dense_names, dense_dims, label, label_dim, batch_size, node_type, device, workers=8,
                 slots=None, seed=0, static=False):
        import euler_amd._engine as E
        import euler_amd.ops.graph_api as ge

        eng = get_engine()
        self.mode = eng.meta()["mode"]
        if self.mode not in ("local", "remote", "local_sharded"):
            # graph_partition: the keyed root draw assumes bucket (id % B) lives on shard
            # (bucket % P) % S, which holds only for id-hash partitions (csrc/graph/keyed.cc)
            raise ValueError("the native pipeline serves local, local_sharded and remote sessions "
                             "(id-hash partitions); %s sessions train on the per-op engine path" % self.mode)
        self.device = torch.device(device)
        self.cuda = self.device.type == "cuda"
        self.B = int(batch_size)
        self.fanouts = [int(f) for f in flow.fanouts]
        self.self_loops = bool(flow.add_self_loops)
        self.label_dim = int(label_dim)
        ets = [[int(x) for x in np.asarray(ge.get_edge_type_id(m)).reshape(-1) if int(x) >= 0] if m is not None else []
               for m in flow.metapath]
        nt = -1 if node_type in (None, -1, "-1") else int(np.asarray(ge.get_node_type_id(node_type)).reshape(-1)[0])
        self.lay = E.sage_pipeline_layout(self.B, self.fanouts, self.self_loops, [int(d) for d in dense_dims],
                                          self.label_dim)
        n_slots = int(slots or (int(workers) + 3))
        self.n_slots = n_slots
        self.workers = int(workers)
        pin = self.cuda
        self.ints = [torch.zeros(self.lay["ints"], dtype=torch.int64, pin_memory=pin) for _ in range(n_slots)]
        self.floats = [torch.zeros(max(1, self.lay["floats"]), dtype=torch.float32, pin_memory=pin)
                       for _ in range(n_slots)]
        self.pipe = E.SagePipeline(eng, self.B, nt, ets, self.fanouts, int(flow.max_id) + 1, self.self_loops,
                                   ["dense_" + str(nm) for nm in dense_names], [int(d) for d in dense_dims],
                                   ("dense_" + str(label)) if label else "",
                                   self.label_dim, [t.data_ptr() for t in self.ints],
                                   [t.data_ptr() for t in self.floats], int(workers), int(seed))
        self.stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self._inflight = []  # (slot, event) copies not yet known complete
        self.static = bool(static) and self.cuda
        if self.static:
            self._setup_static(dense_dims)

    # ------------------------------------------------------------------ static mode
    def _setup_static(self, dense_dims):
        lay, L = self.lay, len(self.fanouts)
        self.cap = [int(c) for c in lay["cap"]]
        self.w = [f + (1 if self.self_loops else 0) for f in self.fanouts]
        self.fd = int(lay["feat_dim"])
        # every int word any static view reads lies below the end of hop L's nbr block
        self.static_ints = int(lay["off_nbr"][L]) + (self.cap[L - 1] * self.w[L - 1] + 1) // 2
        dev = self.device

        def bufs():
            return (torch.zeros(self.static_ints, dtype=torch.int64, device=dev),
                    torch.zeros(self.cap[L] * self.fd, dtype=torch.float32, device=dev),
                    torch.zeros(self.B * self.label_dim, dtype=torch.float32, device=dev))

        self._stage = [bufs(), bufs()]
        self._stage_free = [None, None]  # compute-stream event after the D2D out of stage j
        self._j = 0
        ints, x, lab = self._static_bufs = bufs()
        df = DataFlow(ints[16:16 + self.B])
        for h in range(1, L + 1):
            nid = ints[lay["off_nid"][h]:lay["off_nid"][h] + self.cap[h]]
            res = ints[lay["off_res"][h]:lay["off_res"][h] + self.cap[h - 1]]
            t, w, o = self.cap[h - 1], self.w[h - 1], int(lay["off_nbr"][h])
            nbr = ints[o:o + (t * w + 1) // 2].view(torch.int32)[: t * w].view(t, w)
            df.blocks.append(Block(nid, res, None, None, [t, self.cap[h]], nbr))
            df._last = nid
        self.static_prepared = Prepared(inputs=ints[16:16 + self.B], label=lab.view(self.B, self.label_dim),
                                        embed_in=Prepared(flow=df, x=x.view(self.cap[L], self.fd)))

    def _get_static(self, slot, n):
        L = len(self.fanouts)
        I, Fl, lay = self.ints[slot], self.floats[slot], self.lay
        nx = n[L] * self.fd
        j = self._j
        self._j ^= 1
        st = self._stage[j]
        cur = torch.cuda.current_stream(self.device)
        with torch.cuda.stream(self.stream):
            if self._stage_free[j] is not None:
                self.stream.wait_event(self._stage_free[j])
            st[0].copy_(I[:self.static_ints], non_blocking=True)
            st[1][:nx].copy_(Fl[:nx], non_blocking=True)
            st[2].copy_(Fl[lay["off_labels"]:lay["off_labels"] + self.B * self.label_dim], non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        self._inflight.append((slot, ev))
        cur.wait_event(ev)
        ints, x, lab = self._static_bufs
        ints.copy_(st[0])
        x[:nx].copy_(st[1][:nx])
        lab.copy_(st[2])
        free = torch.cuda.Event()
        free.record(cur)
        self._stage_free[j] = free
        return self.static_prepared

    # ------------------------------------------------------------------ consumer
    def _recycle(self, block=False):
        keep = []
        for slot, ev in self._inflight:
            if ev is None or ev.query() or block:
                if ev is not None and block:
                    ev.synchronize()
                self.pipe.release(slot)
            else:
                keep.append((slot, ev))
        self._inflight = keep

    def _extent(self, slot):
        """(header sizes, used int64 prefix length) of a filled slot"""
        I, lay = self.ints[slot], self.lay
        hdr = I[:16].tolist()
        L = int(hdr[0])
        n = [int(hdr[1 + h]) for h in range(L + 1)]
        e = [0] + [int(hdr[8 + h]) for h in range(1, L + 1)]
        f = self.fanouts[L - 1] + (1 if self.self_loops else 0)
        return L, n, e, int(lay["off_nbr"][L]) + (n[L - 1] * f + 1) // 2

    def _backpressure(self):
        """Slots held by copies still in flight must leave the workers something to fill:
        ``next()`` blocks in C++ and nothing releases a slot meanwhile, so if the host ran
        far ahead of the GPU (asynchronous graph replays) and every slot waited on a copy,
        ``next()`` would wait forever.  Wait on the oldest copies instead (bounded: the GPU
        completes them), keeping at least ``workers`` slots free or filled."""
        while self._inflight and len(self._inflight) > self.n_slots - self.workers - 1:
            slot, ev = self._inflight.pop(0)
            if ev is not None:
                ev.synchronize()
            self.pipe.release(slot)

    def get(self):
        """Prepared(inputs=roots, label, embed_in=Prepared(flow, x)) on the device.  Three
        H2D copies per batch (used int prefix, feature rows, labels), device-side views."""
        self._recycle()
        self._backpressure()
        slot = self.pipe.next()
        if slot < 0:
            raise StopIteration
        L, n, e, used = self._extent(slot)
        if self.static:
            return self._get_static(slot, n)
        I, Fl, lay = self.ints[slot], self.floats[slot], self.lay
        fd = int(lay["feat_dim"])
        src = (I[:used], Fl[:n[L] * fd], Fl[lay["off_labels"]:lay["off_labels"] + self.B * self.label_dim])
        if self.cuda:
            cur = torch.cuda.current_stream(self.device)
            with torch.cuda.stream(self.stream):
                ints_d, x_d, lab_d = (t.to(self.device, non_blocking=True) for t in src)
                ev = torch.cuda.Event()
                ev.record(self.stream)
            cur.wait_event(ev)
            for t in (ints_d, x_d, lab_d):
                t.record_stream(cur)
            self._inflight.append((slot, ev))
        else:
            ints_d, x_d, lab_d = (t.clone() for t in src)
            self._inflight.append((slot, None))
        # views (compute stream, after the copy event)
        roots = ints_d[16:16 + self.B]
        df = DataFlow(roots)
        for h in range(1, L + 1):
            nid = ints_d[lay["off_nid"][h]:lay["off_nid"][h] + n[h]]
            res = ints_d[lay["off_res"][h]:lay["off_res"][h] + n[h - 1]]
            ei = ints_d[lay["off_src"][h]:lay["off_src"][h] + 2 * e[h]].view(2, e[h])
            t, w = n[h - 1], self.fanouts[h - 1] + (1 if self.self_loops else 0)
            o = lay["off_nbr"][h]
            nbr = ints_d[o:o + (t * w + 1) // 2].view(torch.int32)[: t * w].view(t, w)
            df.blocks.append(Block(nid, res, None, ei, [t, n[h]], nbr))
            df._last = nid
        x = x_d.view(n[L], fd)
        lab = lab_d.view(self.B, self.label_dim)
        return Prepared(inputs=roots, label=lab, embed_in=Prepared(flow=df, x=x))

    def close(self):
        if self.pipe is not None:
            self.pipe.stop()
            self._recycle(block=True)
            self.pipe = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
