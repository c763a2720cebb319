"""Row-sharded embedding tables with row-sparse training — the MI355X replacement for
the reference's parameter-server ``mod``-partitioned embedding variables and their
sparse ``scatter_update`` / optimizer slots (``tf_euler/python/utils/embedding.py:24-68``,
``layers.py:135-149``; SURVEY §2.7 C2/K12, §2.8 "Embedding / model parallelism").

Row ``r`` lives on rank ``r % world`` at local row ``r // world``.  One training step of
a table is explicit (no autograd, no dense gradient of the table):

  lookup(ids)                 ids de-duplicated on the GPU (hash kernel, unique.hip),
                              routed to their owners with one RCCL all-to-all of ids and
                              one of rows (fwd) — only the touched rows move over xGMI
  apply(handle, grad_rows)    per-unique-row gradients go back to the owners with one
                              all-to-all; the owner merges rows requested by several
                              ranks and applies a row-sparse Adam / Adagrad / SGD update
                              (optim.hip sparse_optim) to its shard in place

With world == 1 the same code runs without collectives.  With 288 GB of HBM a rank
holds ~100M x 128 fp32 rows plus Adam slots, so DeepWalk/LINE tables of billions of
rows fit across one node.

Fixed-capacity form (``lookup_static`` / ``apply_static``): for hipGraph-captured steps
nothing may depend on a host-read size.  Ids arrive padded (-1 = no id, from
``unique_first_padded``), each owner gets a fixed ``C`` slots per peer, and every
exchange is an equal-split ``all_to_all_single`` of ``W * C`` entries — no count
exchange, no ``.cpu()``.  ``C`` = mean + 6 sigma + 64 of the per-owner load of ``n``
hashed ids (``capacity``); an id that would not fit raises the device-side ``overflow``
flag (``check_overflow`` reads it, e.g. once per log interval) instead of being silently
dropped unnoticed.  Expected traffic per step and rank with n ids of D fp32: ids
8 W C bytes, rows and gradients 2 x 4 D W C bytes, ~3 x n / W of it leaving the rank.

``wire_dtype="bf16"`` moves the row and gradient exchanges (both forms) as bf16: half the
bytes on xGMI for the two large all-to-alls; the table, its optimizer slots and the
update stay fp32 (rows are widened on arrival, gradients rounded once before sending).
The fixed-capacity form can keep the wire dtype end to end (``keep_wire``): the owner
gathers its fp32 rows straight into the bf16 send buffer (one converting gather kernel),
the caller's kernels read the received bf16 rows and write bf16 gradients, and the
row-sparse optimizer reads those gradients from the receive buffer — no fp32 copies of
the W*C exchanged rows on either side (DeepWalk, models/deepwalk_step.py).
"""
from __future__ import annotations

import math

import torch
import torch.distributed as dist

from euler_amd.ops import mp_ops
from euler_amd.ops._native import hip, use_hip
from euler_amd.ops.gnn_ops import route_by_owner, unique_first
from euler_amd.parallel import comm

__all__ = ["ShardedTable", "LookupHandle", "StaticHandle"]

_KINDS = {"adam": 0, "adagrad": 1, "sgd": 2}


class LookupHandle:
    __slots__ = ("order", "send", "recv", "local_rows", "n", "rank")

    def __init__(self, order, send, recv, local_rows, n, rank=None):
        self.order, self.send, self.recv, self.local_rows, self.n = order, send, recv, local_rows, n
        # sorted_out lookups: position of ids[k] in the returned (owner-sorted) rows
        self.rank = rank


class StaticHandle:
    """``pos[k]``: slot (in the W*C exchange space) of padded id k (W*C = none);
    ``local``: the owner-local rows this rank serves per slot (-1 = empty slot)."""
    __slots__ = ("pos", "local")

    def __init__(self, pos, local):
        self.pos, self.local = pos, local


class ShardedTable:
    def __init__(self, num_rows, dim, device, group=None, optimizer="adam", lr=0.01, init_std=0.1, seed=0,
                 beta1=0.9, beta2=0.999, eps=1e-8, force_comm=False, wire_dtype="fp32", init="normal", slots=True):
        self.num_rows, self.dim = int(num_rows), int(dim)
        if wire_dtype not in ("fp32", "bf16"):
            raise ValueError("wire_dtype must be fp32 or bf16")
        self.wire = torch.bfloat16 if wire_dtype == "bf16" else torch.float32
        self.group = group
        pg = dist.is_available() and dist.is_initialized()
        dist_on = pg and dist.get_world_size(group) > 1
        self.world = dist.get_world_size(group) if dist_on else 1
        self.rank = dist.get_rank(group) if dist_on else 0
        # collectives on (force_comm: also with one rank, to exercise the all-to-all path)
        self.comm = dist_on or (pg and force_comm)
        self.device = torch.device(device)
        local = max(0, math.ceil((self.num_rows - self.rank) / self.world))
        g = torch.Generator(device=self.device).manual_seed(int(seed) * 131 + self.rank)
        self.weight = torch.empty(local, self.dim, device=self.device)
        if init == "normal":
            self.weight.normal_(0.0, init_std, generator=g)
        elif init is not None:  # None: the caller fills every row (e.g. from a model's table)
            raise ValueError("init must be 'normal' or None")
        self.kind = _KINDS[optimizer]
        self.m = self.v = None
        if slots:
            self.alloc_slots()
        self.step = torch.zeros(1, dtype=torch.int64, device=self.device)
        self.lr, self.b1, self.b2, self.eps = float(lr), float(beta1), float(beta2), float(eps)
        self.overflow = torch.zeros(1, dtype=torch.int32, device=self.device)
        self.cap_override = None  # fixed per-peer slot count (tests / tuning)

    def alloc_slots(self):
        """the optimizer slots: Adam keeps m and v, Adagrad only the accumulator v, SGD none
        (the kernel never touches an unused slot, so it aliases a used one or the weight).
        ``slots=False`` at construction defers this, e.g. until a model's table has been
        moved into :attr:`weight` and freed (a 100M x 128 table pair is 102 GB)."""
        if self.m is not None:
            return
        self.v = torch.zeros_like(self.weight) if self.kind in (0, 1) else self.weight
        self.m = torch.zeros_like(self.weight) if self.kind == 0 else self.v

    # ------------------------------------------------------------------ fixed capacity
    def capacity(self, n: int) -> int:
        """slots per peer for ``n`` (padded) ids per rank"""
        if self.cap_override is not None:
            return int(self.cap_override)
        if self.world == 1:
            return int(n)
        mean = n / self.world
        return min(int(n), int(math.ceil((mean + 6.0 * math.sqrt(mean) + 64) / 64.0)) * 64)

    def lookup_static(self, ids: torch.Tensor, trash_row: bool = False, keep_wire: bool = False):
        """rows [W*C, D] in slot order for padded DISTINCT ids [n] (-1 = none) and the
        :class:`StaticHandle`; row ``handle.pos[k]`` is the row of ``ids[k]``.  Shapes
        depend on n only: safe inside a hipGraph capture.

        An id dropped by a capacity overflow gets ``pos = W*C``.  With ``trash_row`` the
        returned rows have one extra zero row at index W*C, so a dropped id reads zeros
        and a caller's gradient for it lands in that row (never in a live slot); pass only
        the first W*C gradient rows to :meth:`apply_static`.  ``keep_wire``: rows in the
        wire dtype (bf16 wire: no fp32 copy) when they went through a collective."""
        ids = ids.reshape(-1).long()
        n = ids.numel()
        extra = 1 if trash_row else 0
        if not self.comm:
            pos = torch.arange(n, device=ids.device)
            rows = self._gather(ids)
            if extra:
                rows = torch.cat([rows, rows.new_zeros(1, self.dim)])
            return rows, StaticHandle(pos, ids)
        return self.exchange_static(self.route_static(ids), trash_row, keep_wire=keep_wire)

    def route_static(self, ids: torch.Tensor):
        """first half of :meth:`lookup_static` (no collective): the exchange slots of the
        padded distinct ids -> ``(pos, send)``, for a caller that overlaps the exchange"""
        ids = ids.reshape(-1).long()
        return route_by_owner(ids, self.world, self.capacity(ids.numel()), self.overflow, self.rank)

    def _peer_splits(self, C):
        """equal C-slot splits to / from every peer, none to / from this rank (its own
        slots are the last block of the layout and never enter the collective)"""
        return [0 if r == self.rank else int(C) for r in range(self.world)]

    def exchange_static(self, routed, trash_row: bool = False, bufs=None, keep_wire: bool = False):
        """second half of :meth:`lookup_static`: the id and row all-to-alls of routed ids
        (``bufs``: persistent buffers for the collectives, see :meth:`_buf`; ``keep_wire``:
        return the received rows in the wire dtype).

        Slot layout (``route_by_owner(..., self_rank)``): the peers' C-slot blocks in rank
        order, then this rank's own block.  Only the peers' prefix (W-1)*C goes through the
        uneven-split all-to-alls; the own block's ids are served here — its rows are gathered
        straight into the output — so no rank copies its own rows through RCCL (with one
        rank there is no collective at all)."""
        pos, send = routed
        W = self.world
        trash = send.numel() - 1
        C = trash // W
        P = trash - C  # the peers' slots
        dev = send.device
        recv = self._buf(bufs, "recv", (trash,), torch.long, dev)
        if P:
            sd = self._buf(bufs, "send", (P,), torch.long, dev)
            sd.copy_(send[:P])
            sp = self._peer_splits(C)
            comm.all_to_all_single(recv[:P], sd, sp, sp, group=self.group)
        recv[P:].copy_(send[P:trash])  # own requests
        local = torch.where(recv >= 0, torch.div(recv, W, rounding_mode="floor"), torch.full_like(recv, -1))
        extra = 1 if trash_row else 0
        out = self._buf(bufs, "rows_out", (trash + extra, self.dim), self.wire, dev)
        if extra:
            out[trash:].zero_()
        if P:
            xw = self._buf(bufs, "rows_in", (P, self.dim), self.wire, dev)
            self._gather_into(local[:P], xw)
            comm.all_to_all_single(out[:P], xw, sp, sp, group=self.group)
        self._gather_into(local[P:], out[P:trash])
        return (out if keep_wire else out.float()), StaticHandle(pos, local)

    def apply_static(self, handle: StaticHandle, grad_rows: torch.Tensor, bufs=None):
        """row-sparse update from gradients [W*C, D] in slot order (rows of empty slots
        are ignored).  fp32 or wire-dtype gradients; a bf16 wire sends them as they are
        and the optimizer reads them from the receive buffer.  The peers' slots go back to
        their owners over the all-to-all; the own block's gradients are applied here."""
        g = grad_rows.contiguous()
        if g.dtype not in (torch.float32, self.wire):
            g = g.float()
        rows = handle.local
        if self.comm and self.world > 1:
            W = self.world
            trash = g.shape[0]
            C = trash // W
            P = trash - C
            if g.dtype != self.wire:
                gw = self._buf(bufs, "grad_in", (P, self.dim), self.wire, g.device)
                gw.copy_(g[:P])
            else:
                gw = g[:P]
            gr = self._buf(bufs, "grad_out", (trash, self.dim), self.wire, g.device)
            sp = self._peer_splits(C)
            comm.all_to_all_single(gr[:P], gw, sp, sp, group=self.group)
            gr[P:].copy_(g[P:])  # own block
            g = gr
            # several ranks may have asked for the same row: merge (empty slots, local
            # row -1, have inverse -1: the merge skips them and the -1 fill of rows_u
            # past the distinct rows is skipped by the update)
            from euler_amd.ops.gnn_ops import unique_first_padded

            rows_u, inv, _ = unique_first_padded(rows)
            acc = torch.zeros(g.shape, dtype=torch.float32, device=g.device)
            if use_hip(acc, inv):
                hip().index_add_rows_(acc, inv.contiguous(), g)
            else:
                keep = inv >= 0
                acc.index_add_(0, inv[keep], g[keep].float())
            rows, g = rows_u, acc
        self._update(rows.contiguous(), g)

    def check_overflow(self):
        """host read of the overflow flag of the fixed-capacity exchanges (a sync)"""
        if int(self.overflow.item()):
            raise RuntimeError("ShardedTable: a fixed-capacity exchange overflowed its per-peer slots; "
                               "ids were dropped (raise the capacity or use lookup/apply)")

    # ------------------------------------------------------------------ forward
    def lookup(self, ids: torch.Tensor, sorted_out: bool = False):
        """rows [n, D] (fp32) of the DISTINCT global ids ``ids`` (callers de-duplicate
        with :func:`unique_first`), plus the handle needed by :meth:`apply`.

        ``sorted_out``: with collectives the rows are returned in the owner-sorted order
        they arrive in and ``handle.rank[k]`` is the row of ``ids[k]`` — callers remap
        their (small) index arrays instead of permuting [n, D] rows twice per step."""
        ids = ids.reshape(-1).long()
        if not self.comm:
            rank = torch.arange(ids.numel(), device=ids.device) if sorted_out else None
            return self._gather(ids), LookupHandle(None, None, None, ids, ids.numel(), rank)
        W = self.world
        owner = torch.remainder(ids, W)
        # stable bucket order by owner: radix sort on a small key
        key = owner.to(torch.uint8) if W <= 256 else owner
        order = torch.sort(key, stable=True)[1]
        send_counts = torch.bincount(owner, minlength=W)
        recv_counts = torch.empty_like(send_counts)
        comm.all_to_all_single(recv_counts, send_counts, group=self.group)
        counts = torch.stack([send_counts, recv_counts]).cpu()  # one host sync for both
        send, recv = counts[0].tolist(), counts[1].tolist()
        recv_ids = torch.empty(sum(recv), dtype=ids.dtype, device=ids.device)
        comm.all_to_all_single(recv_ids, ids[order].contiguous(), recv, send, group=self.group)
        local = torch.div(recv_ids, W, rounding_mode="floor")
        out_sorted = self._a2a_rows(self._gather(local), send, recv)
        if sorted_out:
            rank = torch.empty_like(order)
            rank[order] = torch.arange(order.numel(), device=order.device)
            return out_sorted, LookupHandle(order, send, recv, local, ids.numel(), rank)
        out = torch.empty_like(out_sorted)
        out[order] = out_sorted
        return out, LookupHandle(order, send, recv, local, ids.numel())

    @staticmethod
    def _buf(bufs, name, shape, dtype, device):
        """persistent exchange buffer ``name`` of ``bufs`` (None: a fresh tensor).  Buffers
        that collectives read or write on a side stream of a captured graph must outlive
        the capture (allocated by the first eager step, reused by the capture)."""
        if bufs is None:
            return torch.empty(shape, dtype=dtype, device=device)
        t = bufs.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype:
            t = bufs[name] = torch.empty(shape, dtype=dtype, device=device)
        return t

    def _a2a_rows(self, x, out_splits=None, in_splits=None, extra=0, bufs=None, tag="", keep_wire=False):
        """all-to-all of [*, D] rows in the wire dtype; returns fp32 rows (``keep_wire``:
        the wire-dtype receive buffer) plus ``extra`` zero rows at the end.  Rows already
        in the wire dtype are sent as they are."""
        if x.dtype == self.wire and x.is_contiguous():
            xw = x
        else:
            xw = self._buf(bufs, tag + "in", (x.shape[0], self.dim), self.wire, x.device)
            xw.copy_(x)
        n = xw.shape[0] if out_splits is None else sum(out_splits)
        out = self._buf(bufs, tag + "out", (n + extra, self.dim), self.wire, xw.device)
        if extra:
            out[n:].zero_()
        comm.all_to_all_single(out[:n], xw, out_splits, in_splits, group=self.group)
        return out if keep_wire else out.float()

    def _gather_into(self, local, out):
        """``out[k] = weight[local[k]]`` in out's dtype (local < 0: a zero row)"""
        if out.dtype == torch.bfloat16 and use_hip(self.weight, local) and self.dim % 4 == 0:
            hip().gather_f32_bf16(self.weight, local.contiguous(), out)
            return
        out.copy_(self._gather(local))

    def _gather(self, local):
        if use_hip(self.weight, local):
            return mp_ops.gather(self.weight, local)
        return self.weight[local]

    # ------------------------------------------------------------------ backward + update
    def apply(self, handle: LookupHandle, grad_rows: torch.Tensor, sorted_in: bool = False):
        """Row-sparse optimizer step with ``grad_rows`` [n, D] = gradient of the rows
        returned by :meth:`lookup` (same order; ``sorted_in``: in the owner-sorted order
        of a ``sorted_out`` lookup)."""
        g = grad_rows.float().contiguous()
        if self.comm:
            g_sorted = g if sorted_in else g[handle.order].contiguous()
            rows, g = handle.local_rows, self._a2a_rows(g_sorted, handle.recv, handle.send)
            # several ranks may have asked for the same row: merge before the update
            # (one rank's ids are distinct already)
            rows_u, inv = unique_first(rows) if self.world > 1 else (rows, None)
            if rows_u.numel() != rows.numel():
                acc = torch.zeros(rows_u.numel(), self.dim, dtype=g.dtype, device=g.device)
                if use_hip(acc, inv):
                    hip().index_add_rows_(acc, inv.contiguous(), g)
                else:
                    acc.index_add_(0, inv, g)
                rows, g = rows_u, acc
        else:
            rows = handle.local_rows
        self._update(rows.contiguous(), g)

    def _update(self, rows, g):
        if g.dtype != torch.float32 and not (g.dtype == torch.bfloat16 and use_hip(self.weight, rows, g)
                                             and self.dim % 4 == 0):
            g = g.float()
        if use_hip(self.weight, rows, g):
            hip().sparse_optim_(self.weight, self.m, self.v, rows, g, self.step, self.lr, self.b1, self.b2,
                                self.eps, self.kind)
            return
        keep = (rows >= 0) & (rows < self.weight.shape[0])  # -1: empty slot (fixed-capacity path)
        if not bool(keep.all()):
            rows, g = rows[keep], g[keep]
        self.step += 1
        if self.kind == 0:
            t = float(self.step.item())
            m = self.b1 * self.m[rows] + (1 - self.b1) * g
            v = self.b2 * self.v[rows] + (1 - self.b2) * g * g
            self.m[rows], self.v[rows] = m, v
            upd = (m / (1 - self.b1 ** t)) / ((v / (1 - self.b2 ** t)).sqrt() + self.eps)
            self.weight[rows] -= self.lr * upd
        elif self.kind == 1:
            acc = self.v[rows] + g * g
            self.v[rows] = acc
            self.weight[rows] -= self.lr * g / (acc.sqrt() + self.eps)
        else:
            self.weight[rows] -= self.lr * g

    def fused_sgns_ok(self, *tensors):
        """True when a skip-gram update can be applied in place by the fused kernel
        (one rank owns every row, GPU tensors, D % 4 == 0)."""
        return not self.comm and use_hip(self.weight, *tensors) and self.dim % 4 == 0 and self.dim <= 256

    def apply_sgns(self, side, ptr, lst, coef, K, src, smap, sinv, ids, inc_step=True):
        """fused row-sparse update from occurrence lists (embed.hip sgns_update, see
        gnn_ops.sgns_grad): gradients of the unique ids ``ids`` are rebuilt and applied
        in one pass, no gradient rows are materialised.  ``inc_step`` advances the
        optimizer step (once per training step when several updates hit one table).
        Requires :meth:`fused_sgns_ok`."""
        hip().sgns_apply_(int(side), ptr, lst, coef, int(K), src, smap, sinv, self.weight, self.m, self.v,
                          ids.contiguous(), self.step, bool(inc_step), self.lr, self.b1, self.b2, self.eps,
                          self.kind)

    def global_ids(self):
        return torch.arange(self.weight.shape[0], device=self.device) * self.world + self.rank

    def full(self) -> torch.Tensor:
        """the whole [num_rows, D] table on every rank (a collective when world > 1):
        checkpoints keep a sharded table under the model's own parameter name"""
        if self.world == 1:
            return self.weight.detach().clone()
        rows = -(-self.num_rows // self.world)
        pad = torch.zeros(rows, self.dim, device=self.weight.device)
        pad[: self.weight.shape[0]] = self.weight.detach()
        parts = [torch.zeros_like(pad) for _ in range(self.world)]
        dist.all_gather(parts, pad, group=self.group)
        return torch.stack(parts, 1).reshape(-1, self.dim)[: self.num_rows].clone()  # row r = parts[r % W][r // W]

    def load(self, w: torch.Tensor):
        """this rank's rows from a whole table ([num_rows, D]) or from its own shard"""
        w = torch.as_tensor(w).to(self.weight)
        with torch.no_grad():
            self.weight.copy_(w[self.global_ids()] if w.shape[0] == self.num_rows and self.world > 1 else
                              w[: self.weight.shape[0]])

    def slot_state(self):
        return {"m": self.m.cpu().clone(), "v": self.v.cpu().clone(), "step": int(self.step.item())}

    def load_slot_state(self, s):
        """optimizer slots saved by :meth:`slot_state` (skipped for another shard shape)"""
        if s is None or torch.as_tensor(s["m"]).shape != self.m.shape:
            return
        self.m.copy_(torch.as_tensor(s["m"]).to(self.m))
        self.v.copy_(torch.as_tensor(s["v"]).to(self.v))
        self.step.fill_(int(s["step"]))

    # ------------------------------------------------------------------ per-rank checkpoints
    def slot_kinds(self):
        """the optimizer slots this table keeps (Adam: m, v; Adagrad: v; SGD: none)"""
        return {0: ("m", "v"), 1: ("v",), 2: ()}[self.kind]

    def shard_tensors(self, lo=0, hi=None):
        """kind -> local rows [lo, hi) of the weight and of every optimizer slot"""
        out = {"weight": self.weight[lo:hi]}
        for k in self.slot_kinds():
            out[k] = getattr(self, k)[lo:hi]
        return out

    def save_shard(self, ckpt_path, name, num=None, lo=0, rows_of=None):
        """write this rank's rows (and their slots) next to ``ckpt_path``
        (parallel/shard_io.py); ``lo``: first local row of a table slice that is itself
        ``mod``-sharded (a half of a two-table layout whose offset is a multiple of world),
        ``num``: global rows of that slice"""
        from euler_amd.parallel.shard_io import save_rows

        num = self.num_rows if num is None else int(num)
        n_local = -(-num // self.world)
        return save_rows(ckpt_path, name, self.shard_tensors(lo, lo + n_local), num, self.world, self.rank)

    def load_shard(self, dirname, metas, lo=0, n_local=None, name="table"):
        """fill local rows [lo, lo + n_local) (global slice rows ``j * world + rank``) and
        their slots from a checkpoint written by any number of ranks; slots the checkpoint
        does not hold (another optimizer) restart at zero"""
        import logging

        from euler_amd.parallel.shard_io import read_rows

        n_local = self.weight.shape[0] - lo if n_local is None else int(n_local)
        rows = torch.arange(n_local, dtype=torch.int64) * self.world + self.rank
        with torch.no_grad():
            read_rows(dirname, metas, "weight", rows, self.weight[lo:lo + n_local])
            for k in self.slot_kinds():
                dst = getattr(self, k)[lo:lo + n_local]
                if not read_rows(dirname, metas, k, rows, dst):
                    dst.zero_()
                    logging.getLogger("euler_amd.estimator").warning(
                        "%s: the checkpoint has no '%s' optimizer slot (another optimizer); it restarts at zero",
                        name, k)

    def state_tensors(self):
        """every tensor a training step changes (rollback snapshots, re-sync broadcasts)"""
        ts = [self.weight]
        for t in (self.m, self.v):
            if all(t is not u for u in ts):
                ts.append(t)
        return ts + [self.step]

    def nbytes(self):
        ts = {id(t): t for t in (self.weight, self.m, self.v)}.values()
        return sum(t.numel() * t.element_size() for t in ts)

    @staticmethod
    def bytes_per_row(dim, optimizer):
        return dim * 4 * {"adam": 3, "adagrad": 2, "sgd": 1}[optimizer]
