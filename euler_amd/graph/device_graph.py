"""HBM-resident graph shard with GPU-side sampling.

An MI355X has 288 GB of HBM: a 100M-node / 1B-edge weighted graph (CSR with int32
neighbor rows + fp32 cumulative weights ~ 8.8 GB) plus 100M x 128 bf16 features
(25.6 GB) fits on every GPU with room to spare.  Keeping the shard resident lets
neighbor sampling run as gfx950 kernels next to the model instead of streaming
sampled ids over PCIe each step (SURVEY §7.4 "possibly GPU-side sampling from an
HBM-resident CSR ... decide by measurement").

Semantics are the engine's (``csrc/graph``): per (row, edge type) segments with
inclusive prefix-sum weights; a neighbor draw picks an edge-type group by its
weight sum, then binary-searches the group (reference ``node.cc:98-161``); empty
rows yield ``default`` (reference ``sample_neighbor_op.cc:37-145``).  Rows are
dense 0..N-1; ``ids`` (optional) maps rows back to raw uint64 node ids.

Randomness: Philox counter-based, keyed by a device-resident ``(seed, counter)``
pair.  Each call site passes a distinct ``stream_id`` and ``advance()`` bumps the
counter on the GPU, so a captured hipGraph replays with fresh samples.
"""
from __future__ import annotations

import time

import numpy as np
import torch

from euler_amd.ops._native import hip, use_hip

__all__ = ["DeviceGraph", "build_alias_table"]


def _export_local(eng, names, dims, label, label_dim):
    """an in-process engine's graph as host arrays (CSR in engine row order, node table,
    the dense feature / label columns)"""
    indptr, nbr, w, T, ids, _ = eng.export_csr()
    _, types, nw = eng.export_nodes()
    out = {"indptr": indptr, "nbr": nbr, "w": w, "T": np.asarray([int(T)], np.int64), "ids": ids, "types": types,
           "nw": nw}
    if names:
        out["features"] = np.concatenate([np.asarray(eng.dense_feature(ids, "dense_" + str(n), int(d)), np.float32)
                                          for n, d in zip(names, dims)], 1)
    if label is not None:
        out["labels"] = np.asarray(eng.dense_feature(ids, "dense_" + str(label), int(label_dim)), np.float32)
    return out


def shared_export(fn):
    """``(arrays, done)``: ``fn()``'s arrays, computed ONCE per node when several data-
    parallel ranks share it (torch.distributed initialised, more than one rank on this
    host): the host's lowest global rank writes them as .npy files under /dev/shm, every
    rank of the host maps them read-only (``numpy.load(mmap_mode="r")``: one physical copy
    in the page cache, no per-rank host copy).  ``done()`` synchronises the ranks and
    removes the files.  Without peers it is ``fn()`` and a no-op.  The host's ranks are
    found by host name (not LOCAL_RANK, which launchers that share one GPU between ranks
    may set alike); a failing export is reported to every rank instead of leaving them in
    a barrier."""
    import os
    import shutil
    import socket

    import torch.distributed as dist

    on = dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1
    if not on or os.environ.get("EULER_AMD_SHARED_EXPORT", "1") == "0":
        return fn(), (lambda: None)
    me = dist.get_rank()
    hosts = [None] * dist.get_world_size()
    dist.all_gather_object(hosts, socket.gethostname())
    peers = [r for r, h in enumerate(hosts) if h == hosts[me]]
    if len(peers) <= 1:
        return fn(), (lambda: None)
    leader = min(peers)
    # one directory per host leader (every rank learns every leader's choice)
    name = "/dev/shm/euler_amd_export_%d_%d" % (os.getpid(), int(time.time() * 1e3)) if me == leader else None
    names = [None] * dist.get_world_size()
    dist.all_gather_object(names, name)
    d = names[leader]
    err = None
    if me == leader:
        try:
            arrays = fn()
            os.makedirs(d, exist_ok=True)
            for k, v in arrays.items():
                np.save(os.path.join(d, k + ".tmp.npy"), np.asarray(v))
                os.replace(os.path.join(d, k + ".tmp.npy"), os.path.join(d, k + ".npy"))
            keys = sorted(arrays)
            del arrays
            with open(os.path.join(d, "KEYS"), "w") as f:
                f.write("\n".join(keys))
        except Exception as e:  # reported to the host's ranks below
            err = "%s: %s" % (type(e).__name__, e)
    errs = [None] * dist.get_world_size()
    dist.all_gather_object(errs, err)
    if errs[leader] is not None:
        if me == leader:
            shutil.rmtree(d, ignore_errors=True)
        raise RuntimeError("shared graph export on rank %d failed: %s" % (leader, errs[leader]))
    with open(os.path.join(d, "KEYS")) as f:
        keys = [k for k in f.read().split("\n") if k]
    mapped = {k: np.load(os.path.join(d, k + ".npy"), mmap_mode="r", allow_pickle=False) for k in keys}

    def done():
        dist.barrier()
        if me == leader:
            shutil.rmtree(d, ignore_errors=True)

    return mapped, done


_UPLOAD_CHUNK = 1 << 26  # elements per host -> device chunk


def _upload(a, dtype, device) -> torch.Tensor:
    """``a`` (numpy, possibly a read-only memory map, or a tensor) as a ``dtype`` tensor on
    ``device``, converted and copied ``_UPLOAD_CHUNK`` elements at a time"""
    if isinstance(a, torch.Tensor):
        return a.to(device=device, dtype=dtype).contiguous()
    a = np.asarray(a).reshape(-1)
    out = torch.empty(a.shape[0], dtype=dtype, device=device)
    npd = {torch.int64: np.int64, torch.int32: np.int32, torch.float32: np.float32, torch.float64: np.float64}[dtype]
    for s in range(0, a.shape[0], _UPLOAD_CHUNK):
        chunk = np.array(a[s: s + _UPLOAD_CHUNK], dtype=npd)  # one bounded host copy (also un-maps)
        out[s: s + chunk.shape[0]].copy_(torch.from_numpy(chunk))
    return out


def build_alias_table(weights: np.ndarray):
    """Vose alias table (reference ``euler/common/alias_method.cc:23-70``), vectorised."""
    w = np.asarray(weights, dtype=np.float64)
    n = w.shape[0]
    if n == 0:
        return np.zeros(0, np.float32), np.zeros(0, np.int32)
    total = w.sum()
    if total <= 0:
        w = np.ones(n)
        total = float(n)
    p = w * (n / total)
    prob = np.ones(n, dtype=np.float64)
    alias = np.arange(n, dtype=np.int64)
    if np.allclose(p, 1.0):
        return prob.astype(np.float32), alias.astype(np.int32)
    small = list(np.nonzero(p < 1.0)[0])
    large = list(np.nonzero(p >= 1.0)[0])
    p = p.copy()
    while small and large:
        s = small.pop()
        l = large[-1]
        prob[s] = p[s]
        alias[s] = l
        p[l] = p[l] - (1.0 - p[s])
        if p[l] < 1.0:
            large.pop()
            small.append(l)
    for i in small + large:
        prob[i] = 1.0
    return prob.astype(np.float32), alias.astype(np.int32)


class DeviceGraph:
    def __init__(self, indptr, nbr, cumw, num_types=1, node_prob=None, node_alias=None, ids=None,
                 seed: int = 0, device=None):
        device = torch.device(device) if device is not None else indptr.device
        self.device = device
        self.indptr = indptr.to(device=device, dtype=torch.int64).contiguous()
        self.nbr = nbr.to(device=device, dtype=torch.int32).contiguous()
        self.cumw = cumw.to(device=device, dtype=torch.float32).contiguous()
        self.num_types = int(num_types)
        self.num_rows = (self.indptr.numel() - 1) // self.num_types
        assert self.indptr.numel() == self.num_rows * self.num_types + 1, "indptr must be [N*T+1]"
        if node_prob is None:
            node_prob = torch.ones(self.num_rows, dtype=torch.float32)
            node_alias = torch.arange(self.num_rows, dtype=torch.int32)
        self.node_prob = torch.as_tensor(node_prob, dtype=torch.float32).to(device).contiguous()
        self.node_alias = torch.as_tensor(node_alias, dtype=torch.int32).to(device).contiguous()
        self.ids = ids
        self.root_rows = None  # optional candidate -> row map of the root sampler (node-type subset)
        self.features = None   # optional dense node feature table [N, D] (from_engine)
        self.labels = None     # optional label table (from_engine)
        self.rng = torch.tensor([int(seed), 0], dtype=torch.int64, device=device)
        self._cpu_gen = torch.Generator(device="cpu")
        self._cpu_gen.manual_seed(int(seed))

    # ------------------------------------------------------------------ construction
    @classmethod
    def synthetic(cls, num_nodes: int, avg_degree: float = 10.0, max_degree: int = 2048, seed: int = 0,
                  device="cuda"):
        """Power-law random graph generated directly in HBM (GPU) or with torch (CPU)."""
        device = torch.device(device)
        if device.type == "cuda":
            indptr, nbr, cumw = hip().synth_csr(int(num_nodes), float(avg_degree), int(max_degree), int(seed),
                                               device.index if device.index is not None else
                                               torch.cuda.current_device())
        else:
            indptr, nbr, cumw = _synth_cpu(int(num_nodes), float(avg_degree), int(max_degree), int(seed))
        return cls(indptr, nbr, cumw, 1, seed=seed, device=device)

    @classmethod
    def from_csr(cls, indptr, nbr, weights, num_types=1, node_weights=None, ids=None, seed=0, device="cuda"):
        """From host CSR arrays with *raw* edge weights (prefix sums computed per segment on
        the target device).  The arrays are uploaded in bounded chunks (``_upload``): host
        memory stays the caller's arrays — which may be memory-mapped shared exports."""
        device = torch.device(device)
        indptr_t = _upload(indptr, torch.int64, device)
        w = _upload(weights, torch.float32, device)
        cs = torch.cumsum(w.double(), 0)
        del w
        seg_start = torch.repeat_interleave(indptr_t[:-1], torch.diff(indptr_t))
        base = torch.cat([torch.zeros(1, dtype=torch.float64, device=device), cs])[seg_start]
        del seg_start
        cumw = (cs - base).float()
        del cs, base
        prob = alias = None
        if node_weights is not None:
            prob, alias = build_alias_table(np.asarray(node_weights))
            prob, alias = torch.from_numpy(prob), torch.from_numpy(alias)
        return cls(indptr_t, _upload(nbr, torch.int32, device), cumw, num_types, prob, alias, ids, seed, device)

    @classmethod
    def from_engine(cls, engine=None, node_type=-1, features=(), feature_dims=(), label=None, label_dim=None,
                    feature_dtype=torch.bfloat16, seed=0, device="cuda", share=False):
        """Upload the engine's local graph shard to HBM.

        The C++ engine's columnar store (``csrc/graph``) is already a per-(row, edge type)
        CSR with raw uint64 ids; this copies it once as ``indptr`` / int32 neighbour rows /
        per-segment prefix-sum weights, builds the root sampler of ``node_type`` (reference
        ``sample_node(count, node_type)``: node-weighted, -1 = every type, as
        ``graph.cc:333-403``) and, optionally, the dense ``features`` columns (concatenated,
        ``feature_dtype``) and the dense ``label`` column as device tables.  Rows are the
        engine's rows (sorted by node id); :meth:`rows_of` maps raw ids to rows.  A sharded
        engine (remote shard servers, local_sharded) is assembled from every shard's export
        (:meth:`_from_shards`): one GPU's 288 GB of HBM holds the whole graph.

        ``share=True`` (every data-parallel rank calls this together, as the estimator's
        device path does): local rank 0 exports once into /dev/shm and every local rank
        uploads from the shared read-only mapping (:func:`shared_export`)."""
        from euler_amd.ops import base

        eng = engine if engine is not None else base.get_engine()
        names = [] if not features else ([features] if isinstance(features, (str, int)) else list(features))
        dims = [] if not features else ([feature_dims] if isinstance(feature_dims, int) else list(feature_dims))
        if getattr(eng, "mode", "local") != "local":
            return cls._from_shards(eng, node_type, names, dims, label, label_dim, feature_dtype, seed, device)
        # data-parallel ranks on one node: local rank 0 exports once into /dev/shm, every rank
        # maps it (host memory does not grow with the number of ranks)
        export = (lambda: _export_local(eng, names, dims, label, label_dim))
        arrays, done = shared_export(export) if share else (export(), lambda: None)
        try:
            ids = np.array(arrays["ids"])
            g = cls.from_csr(arrays["indptr"], arrays["nbr"], arrays["w"], int(np.asarray(arrays["T"])[0]), ids=ids,
                             seed=seed, device=device)
            g.node_types = np.array(arrays["types"])
            g.set_root_type(node_type, node_weights=np.asarray(arrays["nw"]))
            if names:
                g.features = _upload(arrays["features"], torch.float32, device).view(len(ids), -1).to(feature_dtype)
            if label is not None:
                g.labels = _upload(arrays["labels"], torch.float32, device).view(len(ids), -1)
        finally:
            del arrays
            done()
        return g

    @classmethod
    def _from_shards(cls, eng, node_type, names, dims, label, label_dim, feature_dtype, seed, device):
        """The whole graph of a sharded engine (``remote``: shard servers over RPC, or
        ``local_sharded``) assembled in HBM: every shard exports its nodes, out-adjacency
        (neighbour ids) and dense features in one ``API_EXPORT_SHARD`` call
        (csrc/ops/graph_ops.cc); rows are the union sorted by node id — the row order a
        local engine over the same data has — so the device graph, its samplers and every
        batch drawn from it are identical to the in-process job's."""
        cols = ["dense_" + str(n) for n in names] + ([] if label is None else ["dense_" + str(label)])
        widths = [int(d) for d in dims] + ([] if label is None else [int(label_dim)])
        parts = [eng.export_shard(k, cols, widths) for k in range(int(eng.shard_num))]
        ids = np.concatenate([np.asarray(p[0], np.uint64) for p in parts])
        types = np.concatenate([np.asarray(p[1], np.int32) for p in parts])
        nw = np.concatenate([np.asarray(p[2], np.float32) for p in parts])
        # the edge-type count from the first shard that holds nodes (an empty shard says nothing)
        first = next((p for p in parts if len(p[0])), None)
        T = max(1, (len(first[3]) - 1) // len(first[0])) if first is not None else 1
        for p in parts:
            if len(p[0]) and (len(p[3]) - 1) != len(p[0]) * T:
                raise ValueError("shards disagree on the number of edge types")
        # per node: its T segment lengths and its edge range in the concatenated edge arrays
        seg = np.concatenate([np.diff(np.asarray(p[3], np.int64)).reshape(-1, T) for p in parts], 0)
        nbr_ids = np.concatenate([np.asarray(p[4], np.uint64) for p in parts])
        ew = np.concatenate([np.asarray(p[5], np.float32) for p in parts])
        order = np.argsort(ids, kind="stable")
        if len(ids) > 1 and (np.diff(ids[order].astype(np.int64)) == 0).any():
            raise ValueError("a node id is stored on more than one shard")
        nlen = seg.sum(1)
        nstart = np.concatenate([[0], np.cumsum(nlen)[:-1]])
        seg = seg[order]
        indptr = np.concatenate([[0], np.cumsum(seg.reshape(-1))]).astype(np.int64)
        lens = nlen[order]
        take = np.repeat(nstart[order] - np.concatenate([[0], np.cumsum(lens)[:-1]]), lens) + np.arange(lens.sum())
        sids = ids[order]
        pos = np.searchsorted(sids, nbr_ids[take])
        posc = np.minimum(pos, max(len(sids) - 1, 0))
        rows = np.where((pos < len(sids)) & (sids[posc] == nbr_ids[take]), posc, -1).astype(np.int64)
        g = cls.from_csr(indptr, rows, ew[take], int(T), ids=sids, seed=seed, device=device)
        g.node_types = types[order]
        g.set_root_type(node_type, node_weights=nw[order])
        tabs = [np.concatenate([np.asarray(p[6 + k], np.float32).reshape(-1, widths[k]) for p in parts])[order]
                for k in range(len(widths))]
        if names:
            g.features = torch.from_numpy(np.concatenate(tabs[: len(names)], 1)).to(device=device, dtype=feature_dtype)
        if label is not None:
            g.labels = torch.from_numpy(tabs[-1]).to(device)
        return g

    def set_root_type(self, node_type=-1, node_weights=None):
        """Root sampler over the rows of ``node_type`` (-1: all rows), weighted by
        ``node_weights`` (default 1)."""
        n = self.num_rows
        w = np.ones(n, np.float64) if node_weights is None else np.asarray(node_weights, np.float64)
        if node_type is None or int(node_type) < 0:
            rows = None
            ww = w
        else:
            types = getattr(self, "node_types", None)
            if types is None:
                raise ValueError("node types unknown: build the graph with from_engine")
            rows = np.flatnonzero(np.asarray(types) == int(node_type)).astype(np.int32)
            if rows.size == 0:
                raise ValueError(f"no node of type {node_type}")
            ww = w[rows]
        prob, alias = build_alias_table(ww)
        self.node_prob = torch.from_numpy(prob).to(self.device)
        self.node_alias = torch.from_numpy(alias).to(self.device)
        self.root_rows = None if rows is None else torch.from_numpy(rows).to(self.device)

    def rows_of(self, ids) -> torch.Tensor:
        """Rows of raw node ids (-1 when absent)."""
        q = np.asarray(ids, dtype=np.uint64).reshape(-1)
        if self.ids is None:
            r = q.astype(np.int64)
            r[(r < 0) | (r >= self.num_rows)] = -1
            return torch.from_numpy(r)
        srt = np.asarray(self.ids, dtype=np.uint64)
        pos = np.searchsorted(srt, q)
        pos_c = np.minimum(pos, max(len(srt) - 1, 0))
        hit = (pos < len(srt)) & (srt[pos_c] == q) if len(srt) else np.zeros(q.shape, bool)
        return torch.from_numpy(np.where(hit, pos_c, -1).astype(np.int64))

    # ------------------------------------------------------------------ randomness
    def advance(self, inc: int = 1):
        """Bump the device-side Philox counter (once per training step)."""
        if use_hip(self.rng):
            hip().rng_advance(self.rng, int(inc))
        else:
            self.rng[1] += inc

    def manual_seed(self, seed: int):
        self.rng.fill_(0)
        self.rng[0] = int(seed)
        self._cpu_gen.manual_seed(int(seed))

    def reseed_cpu(self):
        """CPU twin: re-key the host generator from the (seed, counter) pair, so a CPU batch
        is a function of the device RNG state alone (as the Philox draws are on the GPU) and
        a checkpointed (seed, counter) reproduces it after a restart."""
        self._cpu_gen.manual_seed((int(self.rng[0]) * 1000003 + int(self.rng[1])) % (1 << 63))

    def _mask(self, edge_types) -> int:
        if edge_types is None:
            return (1 << self.num_types) - 1
        m = 0
        for t in ([edge_types] if isinstance(edge_types, int) else edge_types):
            m |= 1 << int(t)
        return m

    # ------------------------------------------------------------------ sampling
    def sample_node(self, count: int, stream_id: int = 1) -> torch.Tensor:
        if use_hip(self.node_prob):
            return hip().alias_sample(self.node_prob, self.node_alias, self.root_rows, int(count), self.rng,
                                      int(stream_id))
        n = self.node_prob.numel()
        k = torch.randint(0, n, (count,), generator=self._cpu_gen)
        u = torch.rand(count, generator=self._cpu_gen)
        pick = torch.where(u < self.node_prob[k], k, self.node_alias[k].long())
        if self.root_rows is not None:
            pick = self.root_rows.long()[pick]
        return pick.int()

    def sample_neighbor(self, rows: torch.Tensor, count: int, edge_types=None, default: int = -1,
                        stream_id: int = 2, with_weights: bool = False):
        rows = rows.reshape(-1)
        if use_hip(self.indptr, rows):
            res = hip().sample_neighbor(self.indptr, self.nbr, self.cumw, self.num_rows, self.num_types,
                                        self._mask(edge_types), rows.contiguous(), int(count), int(default),
                                        self.rng, int(stream_id), bool(with_weights))
            return tuple(res) if with_weights else res[0]
        return self._sample_neighbor_cpu(rows, count, self._mask(edge_types), default, with_weights)

    def _sample_neighbor_cpu(self, rows, count, mask, default, with_weights):
        n = rows.numel()
        T = self.num_types
        r = rows.long()
        valid = (r >= 0) & (r < self.num_rows)
        rc = torch.where(valid, r, torch.zeros_like(r))
        base = rc * T
        starts = torch.stack([self.indptr[base + t] for t in range(T)], 1)
        ends = torch.stack([self.indptr[base + t + 1] for t in range(T)], 1)
        tot = torch.where(ends > starts, self.cumw[(ends - 1).clamp(min=0)], torch.zeros(()))
        sel = torch.tensor([(mask >> t) & 1 for t in range(T)], dtype=torch.bool)
        tot = tot * sel.unsqueeze(0)
        out = torch.full((n, count), default, dtype=torch.int32)
        wout = torch.zeros((n, count), dtype=torch.float32)
        tout = torch.full((n, count), -1, dtype=torch.int32)
        cum_t = torch.cumsum(tot, 1)
        ttot = cum_t[:, -1]
        ok = valid & (ttot > 0)
        if count > 0 and bool(ok.any()):
            u1 = torch.rand((n, count), generator=self._cpu_gen) * ttot.unsqueeze(1)
            t = torch.searchsorted(cum_t.contiguous(), u1.contiguous(), right=True).clamp(max=T - 1)
            s = torch.gather(starts, 1, t)
            e = torch.gather(ends, 1, t)
            g = torch.gather(tot, 1, t)
            u2 = torch.rand((n, count), generator=self._cpu_gen) * g
            # binary search per draw inside [s, e)
            lo, hi = s.clone(), (e - 1).clamp(min=0)
            for _ in range(64):
                act = lo < hi
                if not bool(act.any()):
                    break
                mid = (lo + hi) // 2
                go_left = self.cumw[mid] > u2
                hi = torch.where(act & go_left, mid, hi)
                lo = torch.where(act & ~go_left, mid + 1, lo)
            pos = lo
            okm = ok.unsqueeze(1).expand(n, count)
            out = torch.where(okm, self.nbr[pos], out)
            prev = torch.where(pos > s, self.cumw[(pos - 1).clamp(min=0)], torch.zeros(()))
            wout = torch.where(okm, self.cumw[pos] - prev, wout)
            tout = torch.where(okm, t.int(), tout)
        if with_weights:
            return out, wout, tout
        return out

    def random_walk(self, starts: torch.Tensor, walk_len: int, edge_types=None, default: int = -1,
                    stream_id: int = 3, p: float = 1.0, q: float = 1.0) -> torch.Tensor:
        """Walks [n, walk_len + 1] of rows; node2vec-biased when p or q != 1 (see
        ``random_walk_kernel`` in csrc/hip/sampling.hip; neighbour segments must be sorted
        by row, as from_engine / synthetic build them)."""
        if float(p) <= 0.0 or float(q) <= 0.0:
            raise ValueError("random_walk: p and q must be positive")
        starts = starts.reshape(-1).int()
        if use_hip(self.indptr, starts):
            # per-step type masks: built once per (mask, length) and kept on the device, so a
            # walk inside a hipGraph capture issues no host->device copy
            key = (self._mask(edge_types), int(walk_len))
            cache = self.__dict__.setdefault("_walk_masks", {})
            if key not in cache:
                m = torch.tensor([key[0]] * key[1], dtype=torch.int64)
                cache[key] = ((m + 2 ** 31) % 2 ** 32 - 2 ** 31).int().to(self.device)
            return hip().random_walk(self.indptr, self.nbr, self.cumw, self.num_rows, self.num_types,
                                     cache[key], starts.contiguous(), int(default), self.rng,
                                     int(stream_id), float(p), float(q))
        if float(p) == 1.0 and float(q) == 1.0:
            cols = [starts]
            cur = starts
            for _ in range(int(walk_len)):
                cur = self._sample_neighbor_cpu(cur, 1, self._mask(edge_types), default, False).reshape(-1)
                cols.append(cur)
            return torch.stack(cols, 1)
        return self._node2vec_cpu(starts, int(walk_len), self._mask(edge_types), int(default), float(p), float(q))

    def _candidates_cpu(self, rows: torch.Tensor, mask: int):
        """(walk index, edge index) of every out edge of rows[i] under the type mask"""
        T = self.num_types
        ok = (rows >= 0) & (rows < self.num_rows)  # a default row past the table ends a walk
        walk, seg = [], []
        for t in range(T):
            if not (mask >> t) & 1:
                continue
            w = torch.nonzero(ok).reshape(-1)
            walk.append(w)
            seg.append(rows[w].long() * T + t)
        if not walk:
            return torch.zeros(0, dtype=torch.long), torch.zeros(0, dtype=torch.long)
        walk, seg = torch.cat(walk), torch.cat(seg)
        order = torch.argsort(walk, stable=True)  # walk-major (candidates of a walk contiguous)
        walk, seg = walk[order], seg[order]
        a, b = self.indptr[seg].cpu(), self.indptr[seg + 1].cpu()
        ln = (b - a).clamp(min=0)
        wi = torch.repeat_interleave(walk, ln)
        off = torch.arange(int(ln.sum())) - torch.repeat_interleave(torch.cumsum(ln, 0) - ln, ln)
        return wi, torch.repeat_interleave(a, ln) + off

    def _node2vec_cpu(self, starts, walk_len, mask, default, p, q):
        gen = torch.Generator().manual_seed(int(self.rng[0]) * 1000003 + int(self.rng[1]))
        n, N = starts.numel(), self.num_rows
        nbr, cumw, indptr = self.nbr.cpu().long(), self.cumw.cpu().double(), self.indptr.cpu()
        seg_first = torch.zeros_like(cumw, dtype=torch.bool)
        seg_first[indptr[:-1][indptr[:-1] < indptr[1:]]] = True
        ew = torch.where(seg_first, cumw, cumw - torch.roll(cumw, 1))  # per-edge weights
        cur = starts.long().cpu()
        prev, prev_keys = cur.clone(), None
        cols = [cur.clone()]
        for _ in range(walk_len):
            wi, e = self._candidates_cpu(cur, mask)
            c = nbr[e]
            w = ew[e] * torch.where(c == prev[wi], 1.0 / p, 1.0 / q)
            keys = wi * N + c
            if prev_keys is not None:
                common = torch.isin(keys, prev_keys) & (c != prev[wi])
                w = torch.where(common, ew[e], w)
            nxt = torch.full((n,), default, dtype=torch.long)
            if wi.numel():
                cum = torch.cumsum(w, 0)
                ar = torch.arange(n)
                st = torch.searchsorted(wi, ar, right=False)
                en = torch.searchsorted(wi, ar, right=True)
                has = en > st
                base = torch.where(st > 0, cum[(st - 1).clamp(min=0)], torch.zeros(n, dtype=cum.dtype))
                tot = torch.where(has, cum[(en - 1).clamp(min=0)] - base, torch.zeros(n, dtype=cum.dtype))
                u = base + torch.rand(n, generator=gen, dtype=torch.float64) * tot
                pick = torch.minimum(torch.searchsorted(cum, u, right=True), (en - 1).clamp(min=0))
                okw = has & (tot > 0)
                nxt[okw] = c[pick[okw]]
            prev_keys = keys
            prev, cur = cur, nxt
            cols.append(cur.clone())
        return torch.stack(cols, 1).int()

    def degree(self, rows: torch.Tensor) -> torch.Tensor:
        r = rows.long()
        return self.indptr[(r + 1) * self.num_types] - self.indptr[r * self.num_types]

    @property
    def num_edges(self) -> int:
        return int(self.nbr.numel())

    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in (self.indptr, self.nbr, self.cumw, self.node_prob,
                                                           self.node_alias))


def _synth_cpu(n: int, avg_deg: float, max_deg: int, seed: int):
    """CPU twin of the device generator (same distribution family, not bitwise)."""
    g = torch.Generator().manual_seed(seed)
    u = torch.rand(n, generator=g).clamp(min=1e-7)
    deg = (avg_deg * 0.5 / torch.sqrt(u)).long().clamp(1, max_deg)
    indptr = torch.zeros(n + 1, dtype=torch.int64)
    torch.cumsum(deg, 0, out=indptr[1:])
    e = int(indptr[-1])
    src = torch.repeat_interleave(torch.arange(n), deg)
    nbr = torch.randint(0, n, (e,), generator=g)
    nbr = torch.where(nbr == src, (nbr + 1) % n, nbr)
    # sort neighbors inside each row
    key = src * n + nbr
    order = torch.argsort(key)
    nbr = nbr[order]
    w = 0.5 + torch.rand(e, generator=g)
    cs = torch.cumsum(w.double(), 0)
    base = torch.cat([torch.zeros(1, dtype=torch.float64), cs])[indptr[:-1]]
    cumw = (cs - torch.repeat_interleave(base, deg)).float()
    return indptr, nbr.int(), cumw
