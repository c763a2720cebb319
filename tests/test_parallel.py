"""Data parallelism and sharded embeddings on 2 CPU ranks over gloo (the same code
path runs over RCCL on MI355X)."""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                       "WORLD_SIZE": str(world), "LOCAL_RANK": str(rank)})
    from euler_amd.parallel import dp

    dp.init_distributed(backend="gloo", device=torch.device("cpu"))


def _worker_gradsync(rank, world, port, q):
    try:
        _init(rank, world, port)
        from euler_amd.parallel.dp import GradSync, broadcast_module
        from euler_amd.parallel.flat import FlatParams

        torch.manual_seed(100 + rank)  # different init per rank -> broadcast must fix it
        net = torch.nn.Sequential(torch.nn.Linear(6, 5), torch.nn.ReLU(), torch.nn.Linear(5, 3))
        broadcast_module(net)
        ok_bcast = True
        for p in net.parameters():
            other = [torch.zeros_like(p) for _ in range(world)]
            dist.all_gather(other, p.detach())
            ok_bcast &= all(torch.equal(o, other[0]) for o in other)
        # rank-specific data; the synced grad must equal the mean of per-rank grads
        x = torch.randn(4, 6, generator=torch.Generator().manual_seed(rank))
        ref = []
        for r in range(world):
            xr = torch.randn(4, 6, generator=torch.Generator().manual_seed(r))
            net.zero_grad()
            net(xr).square().sum().backward()
            ref.append([p.grad.clone() for p in net.parameters()])
        mean = [sum(g[i] for g in ref) / world for i in range(len(ref[0]))]
        for use_flat in (False, True):
            net.zero_grad(set_to_none=True)
            flat = FlatParams(net.parameters()) if use_flat else None
            sync = GradSync(net.parameters(), bucket_bytes=64, flat=flat)  # tiny buckets -> several launches
            net(x).square().sum().backward()
            sync.finish()
            sync.remove()
            ok = all(torch.allclose(p.grad, m, atol=1e-5) for p, m in zip(net.parameters(), mean))
            q.put((rank, "flat" if use_flat else "plain", bool(ok)))
        q.put((rank, "bcast", bool(ok_bcast)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover - surfaced through the queue
        q.put((rank, "error", repr(e)))


def _worker_sharded(rank, world, port, q):
    try:
        _init(rank, world, port)
        from euler_amd.parallel.embedding import ShardedEmbedding

        torch.manual_seed(0)
        full = torch.randn(23, 4)
        emb = ShardedEmbedding(22, 4)  # 23 rows
        with torch.no_grad():
            emb.weight.copy_(full[emb.global_ids()])
        ids = torch.tensor([[0, 5, 22], [7, 7, 1]]) + rank
        out = emb(ids)
        ok_fwd = torch.allclose(out, full[ids.clamp(max=22)])
        out.sum().backward()
        # expected grad of the owned rows = total occurrences of each id over all ranks
        counts = torch.zeros(23)
        for r in range(world):
            i = (torch.tensor([[0, 5, 22], [7, 7, 1]]) + r).clamp(max=22).reshape(-1)
            counts.index_add_(0, i, torch.ones(i.numel()))
        exp = counts[emb.global_ids()].unsqueeze(1).expand(-1, 4)
        ok_bwd = torch.allclose(emb.weight.grad, exp)
        q.put((rank, "sharded", bool(ok_fwd and ok_bwd)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def _worker_estimator(rank, world, port, q, data_dir, model_dir):
    try:
        _init(rank, world, port)
        import euler_amd as ea
        from euler_amd import models as Z
        from euler_amd.dataset import get_dataset
        from euler_amd.estimator import NodeEstimator

        ds = get_dataset("cora", data_dir=data_dir, scale=0.05)
        ds.load_graph()
        ea.set_seed(17 + rank)
        torch.manual_seed(rank)
        m = Z.SupervisedGraphSage([8, 8, ds.label_dim], [3, 3], [["train"], ["train"]], "feature", 1433, "label",
                                  ds.label_dim, max_id=ds.max_node_id)
        est = NodeEstimator(m, {"model_dir": model_dir, "batch_size": 8, "total_step": 3, "learning_rate": 0.01,
                                "log_steps": 1, "train_node_type": "train", "device": "cpu"})
        est.train()
        flat = torch.cat([p.detach().reshape(-1) for p in m.parameters()])
        gathered = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(gathered, flat)
        q.put((rank, "dp_in_sync", bool(torch.allclose(gathered[0], gathered[1]))))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def _run(fn, *args, world=2):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=fn, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(300)
    out = []
    while not q.empty():
        out.append(q.get())
    for p in procs:
        if p.is_alive():
            p.kill()
    return out


def test_gradsync_and_broadcast():
    res = _run(_worker_gradsync)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 6 and all(r[2] for r in res), res


def test_sharded_embedding_all_to_all():
    res = _run(_worker_sharded)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def test_data_parallel_estimator(tmp_path):
    res = _run(_worker_estimator, str(tmp_path / "data"), str(tmp_path / "ckpt"))
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_sparse_table(rank, world, port, q):
    try:
        _init(rank, world, port)
        from euler_amd.ops.gnn_ops import unique_first
        from euler_amd.parallel.sparse_table import ShardedTable

        torch.manual_seed(0)
        full = torch.randn(31, 4)
        tab = ShardedTable(31, 4, "cpu", optimizer="sgd", lr=0.5)
        tab.weight.copy_(full[tab.global_ids()])
        # overlapping ids across ranks: the owner must merge the two ranks' grads
        ids = torch.tensor([3, 29, 7, 12, 3, 0]) + rank
        u, inv = unique_first(ids)
        rows, h = tab.lookup(u)
        ok_fwd = torch.allclose(rows, full[u])
        g = torch.arange(u.numel() * 4, dtype=torch.float32).view(-1, 4) + 100 * rank
        tab.apply(h, g)
        # expected: full - lr * (sum of every rank's grad rows for that id)
        exp = full.clone()
        for r in range(world):
            ur, _ = unique_first(torch.tensor([3, 29, 7, 12, 3, 0]) + r)
            gr = torch.arange(ur.numel() * 4, dtype=torch.float32).view(-1, 4) + 100 * r
            exp.index_add_(0, ur, -0.5 * gr)
        ok_upd = torch.allclose(tab.weight, exp[tab.global_ids()])
        q.put((rank, "sparse_table", bool(ok_fwd and ok_upd)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def _worker_deepwalk(rank, world, port, q):
    try:
        _init(rank, world, port)
        from euler_amd.graph.device_graph import DeviceGraph
        from euler_amd.models.deepwalk_step import DeepWalkTrainer

        g = DeviceGraph.synthetic(400, 6.0, 40, seed=3, device="cpu")
        g.manual_seed(11 + rank)
        tr = DeepWalkTrainer(g, 400, dim=16, batch_size=64, lr=0.05, optimizer="adagrad", seed=5)
        losses = [float(tr.step()) for _ in range(30)]
        q.put((rank, "deepwalk", bool(sum(losses[-5:]) < sum(losses[:5]))))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def _worker_sparse_table_static(rank, world, port, q, wire="fp32"):
    try:
        _init(rank, world, port)
        from euler_amd.ops.gnn_ops import unique_first_padded
        from euler_amd.parallel.sparse_table import ShardedTable

        torch.manual_seed(0)
        nrows = 31 + world  # ids go up to 29 + rank
        full = torch.randn(nrows, 4)
        tab = ShardedTable(nrows, 4, "cpu", optimizer="sgd", lr=0.5, wire_dtype=wire)
        # bf16 on the wire: rows and gradients rounded once (8 mantissa bits)
        tol = dict(rtol=1e-2, atol=1e-2) if wire == "bf16" else {}
        tab.weight.copy_(full[tab.global_ids()])
        raw = torch.tensor([3, 29, 7, 12, 3, 0, 7]) + rank
        u, inv, cnt = unique_first_padded(raw)          # 5 distinct + two -1 pads
        ok_pad = int(cnt) == 5 and u[5:].tolist() == [-1, -1] and torch.equal(u[inv], raw)
        rows, h = tab.lookup_static(u)
        assert rows.shape[0] == world * tab.capacity(u.numel())
        ok_fwd = torch.allclose(rows[h.pos[:5]], full[u[:5]], **tol)
        g_slot = torch.zeros_like(rows)
        g_id = torch.arange(5 * 4, dtype=torch.float32).view(5, 4) + 100 * rank
        g_slot[h.pos[:5]] = g_id
        tab.apply_static(h, g_slot)
        exp = full.clone()
        for r in range(world):
            ur, _, _ = unique_first_padded(torch.tensor([3, 29, 7, 12, 3, 0, 7]) + r)
            gr = torch.arange(5 * 4, dtype=torch.float32).view(5, 4) + 100 * r
            exp.index_add_(0, ur[:5], -0.5 * gr)
        if wire == "bf16":  # gradients up to ~120: bf16 spacing 0.5 there
            tol = dict(rtol=1e-2, atol=0.5)
        ok_upd = torch.allclose(tab.weight, exp[tab.global_ids()], **tol)
        tab.check_overflow()
        # a too-small capacity raises the device flag instead of silently dropping ids
        tab.cap_override = 1
        tab.lookup_static(u)
        try:
            tab.check_overflow()
            ok_flag = False
        except RuntimeError:
            ok_flag = True
        # dropped ids go to the trash row (index W*C), never onto a live slot: every live
        # row is updated by exactly its own id's gradient
        tab.weight.copy_(full[tab.global_ids()])
        rows, h = tab.lookup_static(u, trash_row=True)
        WC = world * 1
        ok_trash = rows.shape[0] == WC + 1 and float(rows[WC].abs().sum()) == 0.0
        g_slot = torch.zeros_like(rows)
        g_slot[h.pos[:5]] = g_id                         # dropped ids write the trash row
        live = h.pos[:5] < WC
        ok_trash = ok_trash and bool((~live).any()) and torch.allclose(rows[h.pos[:5]][live], full[u[:5]][live], **tol)
        tab.apply_static(h, g_slot[:WC])
        got = torch.zeros(world, dtype=torch.int64)
        dist.all_gather_into_tensor(got, live.sum().view(1))
        changed = (tab.weight - full[tab.global_ids()]).abs().sum(1) > 0
        ok_trash = ok_trash and int(changed.sum()) <= int(got.sum())
        q.put((rank, "sparse_table_static", bool(ok_pad and ok_fwd and ok_upd and ok_flag and ok_trash)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def _worker_deepwalk_static(rank, world, port, q, mbs=1):
    try:
        _init(rank, world, port)
        from euler_amd.graph.device_graph import DeviceGraph
        from euler_amd.models.deepwalk_step import DeepWalkTrainer

        g = DeviceGraph.synthetic(400, 6.0, 40, seed=3, device="cpu")
        g.manual_seed(11 + rank)
        tr = DeepWalkTrainer(g, 400, dim=16, batch_size=64, lr=0.05, optimizer="adagrad", seed=5, static=True,
                             micro_batches=mbs)
        losses = [float(tr.step()) for _ in range(30)]
        tr.table.check_overflow()
        # the shards together still hold one consistent table: every rank's lookups agree
        ids = torch.arange(0, 2 * tr.off, 7)
        rows, _ = tr.table.lookup(ids)
        allr = [torch.zeros_like(rows) for _ in range(world)]
        dist.all_gather(allr, rows)
        same = all(torch.equal(a, allr[0]) for a in allr)
        q.put((rank, f"deepwalk_static_mb{mbs}", bool(sum(losses[-5:]) < sum(losses[:5]) and same)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


@pytest.mark.parametrize("wire", ["fp32", "bf16"])
def test_sharded_table_fixed_capacity_exchange(wire):
    res = _run(_worker_sparse_table_static, wire)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def test_sharded_table_fixed_capacity_exchange_four_ranks():
    """4 ranks: the own-block-last slot layout with the own block in the middle of the
    rank order (ranks 1, 2), at the front (0) and at the end (3) of the peers' prefix"""
    res = _run(_worker_sparse_table_static, "fp32", world=4)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 4 and all(r[2] for r in res), res


@pytest.mark.parametrize("mbs", [1, 2])
def test_deepwalk_static_two_ranks(mbs):
    res = _run(_worker_deepwalk_static, mbs)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def test_sharded_table_row_sparse_update():
    res = _run(_worker_sparse_table)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def test_deepwalk_sharded_two_ranks():
    res = _run(_worker_deepwalk)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_replicated_store(rank, world, port, q):
    try:
        _init(rank, world, port)
        from euler_amd.parallel.replicated import apply_replicated

        store = torch.zeros(10, 3)
        grads = torch.zeros(10, 3)
        # rank r writes rows {r, 5} (row 5 shared: the higher rank wins) and adds to rows {7, 8 + r}
        rows = torch.tensor([rank, 5])
        vals = torch.full((2, 3), float(rank + 1))
        apply_replicated(store, rows, vals, "copy")
        apply_replicated(grads, torch.tensor([7, 8 + rank]), torch.ones(2, 3), "add")
        exp = torch.zeros(10, 3)
        for r in range(world):
            exp[r] = r + 1
        exp[5] = world
        eg = torch.zeros(10, 3)
        eg[7] = world
        for r in range(world):
            eg[min(8 + r, 9)] += 1
        apply_replicated(grads, torch.tensor([9]), None, "zero") if rank == 0 else \
            apply_replicated(grads, torch.empty(0, dtype=torch.long), None, "zero")
        eg[9] = 0
        q.put((rank, "replicated", bool(torch.equal(store, exp) and torch.equal(grads, eg))))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def _worker_sharded_store(rank, world, port, q):
    try:
        _init(rank, world, port)
        import euler_amd as ea
        from euler_amd.parallel.sharded_store import ShardedRowStore
        from euler_amd.utils import encoders as E

        # 1) store semantics: copy (later source rank wins), add, zero, read
        st = ShardedRowStore(11, 3, "cpu", init=lambda ids: ids.float().view(-1, 1).expand(-1, 3))
        flags = []
        ok = torch.equal(st.read(torch.tensor([10, 3, 3])), torch.tensor([[10.0] * 3, [3.0] * 3, [3.0] * 3]))
        st.write(torch.tensor([5, rank]), torch.full((2, 3), float(rank + 100)), "copy")
        st.write(torch.tensor([7]), torch.ones(1, 3), "add")
        st.write(torch.tensor([9]) if rank == 0 else torch.empty(0, dtype=torch.long), None, "zero")
        full = st.read(torch.arange(11))
        exp = torch.arange(11).float().view(-1, 1).expand(-1, 3).clone()
        for r in range(world):
            exp[r] = r + 100
        exp[5] = world - 1 + 100
        exp[7] += world
        exp[9] = 0
        ok = ok and torch.equal(full, exp)
        flags.append(("store", bool(ok)))
        # 2) Scalable encoder: sharded stores reproduce the replicated stores step by step
        ea.synthetic_graph(200, avg_degree=5, max_degree=16, feature_dim=6, label_dim=2, seed=3)
        encs = []
        for sharded in (False, True):
            torch.manual_seed(0)
            e = E.ScalableSageEncoder("0", 2, 2, 4, feature_idx="feature", feature_dim=6, max_id=199)
            e.train()
            e.store_group = None
            if sharded:
                e.use_sharded_stores()
            encs.append(e)
        for step in range(3):
            ids = torch.arange(6) + 10 * rank + step
            outs = []
            for e in encs:
                ea.set_seed(100 + step * 7 + rank)
                torch.manual_seed(step)  # the lazy layers materialise identically
                out = e(ids)
                (out.sum() + e.store_loss).backward()
                e.after_backward()
                outs.append(out.detach())
            ok = ok and torch.allclose(outs[0], outs[1], atol=1e-6)
            flags.append(("out", step, float((outs[0] - outs[1]).abs().max())))
        rep, shd = encs
        allids = torch.arange(rep.stores(0).shape[0])
        ok = ok and torch.allclose(rep.stores(0), shd._sharded[0][0].read(allids), atol=1e-6)
        flags.append(("st", float((rep.stores(0) - shd._sharded[0][0].read(allids)).abs().max())))
        ok = ok and torch.allclose(rep.gradient_stores(0), shd._sharded[0][1].read(allids), atol=1e-6)
        q.put((rank, "sharded_store", bool(ok), flags))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback
        q.put((rank, "error", traceback.format_exc()))


def test_sharded_historical_store_matches_replicated():
    res = _run(_worker_sharded_store)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def test_replicated_store_writes_reach_every_rank():
    res = _run(_worker_replicated_store)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


class _EmbModel(torch.nn.Module):
    def __init__(self):
        super().__init__()
        from euler_amd.parallel.embedding import ShardedEmbedding

        self.emb = ShardedEmbedding(9, 3)   # 10 rows, sharded mod world
        self.lin = torch.nn.Linear(3, 1)


def _worker_ckpt_save(rank, world, port, q, model_dir):
    try:
        _init(rank, world, port)
        from euler_amd.estimator.base import BaseEstimator

        torch.manual_seed(0)
        m = _EmbModel()
        with torch.no_grad():  # row value = its global id
            m.emb.weight.copy_(m.emb.global_ids().float().unsqueeze(1).repeat(1, 3))
        est = BaseEstimator(m, {"model_dir": model_dir, "device": "cpu"})
        est.optimizer = torch.optim.Adagrad(m.parameters(), lr=0.1)
        for p in m.parameters():
            p.grad = torch.ones_like(p)
        est.optimizer.step()
        est.global_step = 7
        est.save()
        dist.barrier()
        q.put((rank, "saved", True))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, "error", repr(e)))


def test_checkpoint_reshards_on_world_size_change(tmp_path):
    """2 ranks save their ShardedEmbedding shards; a 1-process run restores the whole
    table (rows re-interleaved) and its Adagrad slots."""
    from euler_amd.estimator.base import BaseEstimator
    from euler_amd.parallel.embedding import reshard_rows

    res = _run(_worker_ckpt_save, str(tmp_path))
    assert not [r for r in res if r[1] == "error"], res
    m = _EmbModel()
    est = BaseEstimator(m, {"model_dir": str(tmp_path), "device": "cpu"})
    est.optimizer = torch.optim.Adagrad(m.parameters(), lr=0.1)
    assert est.restore()
    w = m.emb.weight.detach()
    assert w.shape == (10, 3) and est.global_step == 7
    # every row took the same Adagrad step, so rows differ by their global ids
    torch.testing.assert_close(w[:, 0] - w[0, 0], torch.arange(10).float())
    st = est.optimizer.state_dict()["state"]
    emb_idx = [n for n, _ in m.named_parameters()].index("emb.weight")
    assert st[emb_idx]["sum"].shape == (10, 3)
    # 3-way re-shard of a 2-way sharded table
    full = torch.arange(10).float().unsqueeze(1)
    assert torch.equal(reshard_rows([full[0::2], full[1::2]], 1, 3), full[1::3])


def _worker_sage_dp(rank, world, port, q, dtype, buckets):
    """SageTrainer.step(grad_sync) on 2 gloo ranks with different sample streams: the
    parameters stay bit-identical across ranks and equal a single-process update on the
    summed gradients of the two ranks' batches, for 10 steps (fp32 or bf16 hand-off)."""
    try:
        import sys

        _init(rank, world, port)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from test_sage_trainer import _trainer

        def make(r):
            tr = _trainer("cpu", [5, 3], [32, 32, 16], 5, seed=3)
            tr.n_buckets = buckets
            tr.graph.manual_seed(1000 + r)  # per-rank sample stream
            tr.set_grad_sync_dtype(dtype)
            return tr

        calls = []

        def sync(g):
            calls.append(g.numel())
            dist.all_reduce(g)
            return 1.0 / world

        tr = make(rank)
        for _ in range(10):
            tr.step(sync)
        mine = tr.logical_params()
        names = list(mine)
        flat = torch.cat([mine[k].reshape(-1) for k in names])
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        lockstep = all(torch.equal(a, allp[0]) for a in allp)
        # single-process oracle: both ranks' batches, summed gradients, one update rule
        ref = [make(r) for r in range(world)]
        for _ in range(10):
            for t in ref:
                t.step_count += 1
                t._cpu_forward_backward()
            for k in names:
                gs = [t._cpu_params[k].grad for t in ref]
                s = gs[0].bfloat16() + gs[1].bfloat16() if dtype == "bf16" else gs[0] + gs[1]
                for t in ref:
                    t._cpu_params[k].grad = s.float().clone()
            for t in ref:
                t._cpu_apply(1.0 / world)
        rp = ref[0].logical_params()
        oracle = all(torch.equal(mine[k], rp[k]) for k in names)
        moved = any(not torch.equal(mine[k], make(rank).logical_params()[k]) for k in names)
        ncalls = len(calls) == 10 * buckets and len(set(calls)) == buckets
        q.put((rank, f"sage_dp_{dtype}_{buckets}", bool(lockstep and oracle and moved and ncalls)))
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("dtype,buckets", [("fp32", 1), ("bf16", 1), ("fp32", 2), ("bf16", 2)])
def test_sage_trainer_data_parallel_lockstep(dtype, buckets):
    res = _run(_worker_sage_dp, dtype, buckets)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_sharded_features(rank, world, port, q, dedup):
    """SageTrainer over a row-sharded feature table (graph/sharded_features.py): each
    rank holds rows r % 2 and every step's sampled rows come over the all-to-all.  Both
    ranks sample the same batches, so the data-parallel run must reproduce a single
    process on the whole table step by step (losses and parameters)."""
    try:
        import sys

        _init(rank, world, port)
        sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
        from test_sage_trainer import _graph, _tables
        from euler_amd.graph.sharded_features import ShardedFeatures
        from euler_amd.models.sage_trainer import SageTrainer

        def make(shard):
            g = _graph("cpu", seed=3)
            g.manual_seed(20)
            x, lab = _tables("cpu", g.num_rows, 32, 5, "class", torch.float32)
            fs = ShardedFeatures.from_full(x, force_comm=True, dedup=dedup) if shard else None
            tr = SageTrainer(g, 64, [5, 3], [32, 32, 16], 5, features=None if shard else x, labels=lab,
                             feature_shard=fs, init_seed=3)
            return tr, fs

        tr, fs = make(True)
        ref, _ = make(False)
        assert fs.shard.shape[0] == (ref.features.shape[0] - rank + world - 1) // world

        def sync(g):
            dist.all_reduce(g)
            return 1.0 / world

        diffs = []
        for _ in range(5):
            diffs.append(abs(float(tr.step(sync)) - float(ref.step())))
        a, b = tr.logical_params(), ref.logical_params()
        pdiff = max(float((a[k] - b[k]).abs().max()) for k in a)
        fs.check_overflow()
        q.put((rank, f"sharded_features_{dedup}", bool(max(diffs) < 1e-6 and pdiff < 1e-6), max(diffs), pdiff))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("dedup,world", [(True, 2), (False, 2), (True, 3)])
def test_sage_trainer_sharded_features_matches_whole_table(dedup, world):
    res = _run(_worker_sharded_features, dedup, world=world)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == world and all(r[2] for r in res), res


def _worker_estimator_device_dp(rank, world, port, q, tmp):
    """NodeEstimator(device_graph=True) under 2 gloo ranks (runner flags as under torchrun):
    per-rank sample streams, gradients summed through make_grad_sync every step, so both
    ranks end with bit-identical trainer parameters."""
    try:
        _init(rank, world, port)
        from euler_amd.tools import runner

        a = runner.parse_args(["--dataset", "ppi", "--scale", "0.05", "--batch_size", "32", "--total_step", "6",
                               "--log_steps", "3", "--model_dir", os.path.join(tmp, f"ckpt_r{rank}"),
                               "--device_graph", "--device", "cpu", "--seed", "1", "--fanouts", "5", "3"],
                              model="graphsage")
        _, est = runner.build(a)
        est.train()
        p = est.device_trainer.logical_params()
        flat = torch.cat([p[k].reshape(-1).float() for k in sorted(p)])
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        same = all(torch.equal(x, allp[0]) for x in allp)
        q.put((rank, "estimator_device_dp", bool(same and est.global_step == 6)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_estimator_device_graph_data_parallel_lockstep(tmp_path):
    res = _run(_worker_estimator_device_dp, str(tmp_path))
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_estimator_unsup_device_dp(rank, world, port, q, tmp):
    """the unsupervised GraphSAGE device path (UnsupSageTrainer) under 2 gloo ranks: the
    estimator finds its FlatParams gradient for make_grad_sync and the ranks stay in step"""
    try:
        _init(rank, world, port)
        from euler_amd.tools import runner

        a = runner.parse_args(["--dataset", "ppi", "--scale", "0.05", "--batch_size", "32", "--total_step", "4",
                               "--log_steps", "2", "--model_dir", os.path.join(tmp, f"ckpt_u{rank}"),
                               "--device_graph", "--device", "cpu", "--seed", "1", "--fanouts", "5", "3",
                               "--dim", "32"], model="graphsage_unsup")
        _, est = runner.build(a)
        est.train()
        flat = est.device_trainer.flat.flat.detach().clone()
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        same = all(torch.equal(x, allp[0]) for x in allp)
        q.put((rank, "estimator_unsup_device_dp", bool(same and est.global_step == 4)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_estimator_unsup_device_graph_data_parallel_lockstep(tmp_path):
    res = _run(_worker_estimator_unsup_device_dp, str(tmp_path))
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_estimator_device_resume(rank, world, port, q, tmp):
    """Device-path data parallelism with a SHARED model_dir (as a real job): run A trains 6
    steps straight; run B trains 3, stops, and a fresh estimator resumes to 6.  Every rank
    writes its own checkpoint file, so after the resume each rank continues ITS sample
    stream: rank r's last batch and the final parameters equal run A's, and the ranks'
    batches differ from each other (per-rank RNG state in checkpoints)."""
    try:
        _init(rank, world, port)
        from euler_amd.tools import runner

        def train(model_dir, total):
            torch.manual_seed(0)  # the same initial weights in every run of this process
            a = runner.parse_args(["--dataset", "ppi", "--scale", "0.05", "--batch_size", "32", "--total_step",
                                   str(total), "--log_steps", "3", "--model_dir", model_dir, "--device_graph",
                                   "--device", "cpu", "--seed", "1", "--fanouts", "5", "3"], model="graphsage")
            _, est = runner.build(a)
            est.train()
            tr = est.device_trainer
            p = tr.logical_params()
            return est, [s.clone() for s in tr.samples()], torch.cat([p[k].reshape(-1).float() for k in sorted(p)])

        est_a, smp_a, par_a = train(os.path.join(tmp, "a"), 6)
        dist.barrier()
        train(os.path.join(tmp, "b"), 3)
        dist.barrier()
        files = sorted(os.listdir(os.path.join(tmp, "b")))
        est_b, smp_b, par_b = train(os.path.join(tmp, "b"), 6)
        same_as_uninterrupted = all(torch.equal(x, y) for x, y in zip(smp_a, smp_b)) and torch.equal(par_a, par_b)
        roots = smp_b[0]
        other = [torch.zeros_like(roots) for _ in range(world)]
        dist.all_gather(other, roots)
        ranks_differ = not torch.equal(other[0], other[1])
        per_rank_files = "model.ckpt-3.pt" in files and "model.ckpt-3-rank1.pt" in files
        q.put((rank, "device_resume", bool(same_as_uninterrupted and ranks_differ and per_rank_files
                                           and est_b.global_step == 6), files))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_estimator_device_graph_resume_keeps_per_rank_streams(tmp_path):
    res = _run(_worker_estimator_device_resume, str(tmp_path))
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_deepwalk_estimator(rank, world, port, q, data_dir, model_dir):
    """NodeEstimator(device_graph=True) DeepWalk on 2 ranks: row-sharded tables (rank r
    holds trainer rows r % 2), per-rank walks, fixed-size all-to-alls; after training (and
    after a resume) every rank assembles the same full tables, and they moved"""
    try:
        _init(rank, world, port)
        import euler_amd as ea
        from euler_amd import models as Z
        from euler_amd.dataset import get_dataset
        from euler_amd.estimator import NodeEstimator

        ds = get_dataset("cora", data_dir=data_dir, scale=0.08)
        ds.load_graph()
        ea.set_seed(3)
        tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
        res = {}
        for total in (20, 30):  # 30: resumes the 20-step checkpoint (per-rank shards + streams)
            torch.manual_seed(0)
            m = Z.DeepWalk("train", ["train"], ds.max_node_id, 8, walk_len=3, num_negs=3)
            before = m.state_dict()["_target_encoder.embedding.weight"].clone()
            est = NodeEstimator(m, {"model_dir": model_dir, "batch_size": 32, "total_step": total,
                                    "optimizer": "adam", "learning_rate": 0.02, "log_steps": 10,
                                    "train_node_type": tnt, "device": "cpu", "device_graph": True, "seed": 11})
            out = est.train()
            tr = est.device_trainer
            res[f"sharded_{total}"] = tr.inner.table.world == 2 and tr.inner.table.weight.shape[0] < tr.inner.table.num_rows
            res[f"finite_{total}"] = bool(np.isfinite(out["loss"])) and out["step"] == total
            w = m.state_dict()["_target_encoder.embedding.weight"]
            allw = [torch.zeros_like(w) for _ in range(world)]
            dist.all_gather(allw, w.contiguous())
            res[f"same_tables_{total}"] = all(torch.equal(x, allw[0]) for x in allw)
            res[f"moved_{total}"] = not torch.equal(before, w)
        q.put((rank, "deepwalk_est", all(res.values()), res))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_deepwalk_estimator_device_path_two_ranks(tmp_path):
    import numpy  # noqa: F401  (the worker uses np through the module import below)

    res = _run(_worker_deepwalk_estimator, str(tmp_path / "cora"), str(tmp_path / "ckpt"))
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_device_trainer_dp(rank, world, port, q, tmp, model, argv, want):
    """one device-path estimator under 2 gloo ranks (runner flags as under torchrun): the
    trainer the registry picks, per-rank sample streams, the flat gradient summed through
    make_grad_sync every step -> bit-identical parameters on every rank"""
    try:
        _init(rank, world, port)
        from euler_amd.tools import runner

        a = runner.parse_args(argv + ["--model_dir", os.path.join(tmp, f"ckpt_{model}_r{rank}"), "--device_graph",
                                      "--device", "cpu", "--seed", "1"], model=model)
        _, est = runner.build(a)
        est.train()
        tr = est.device_trainer
        p = tr.logical_params()
        flat = torch.cat([p[k].reshape(-1).float() for k in sorted(p)])
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        same = all(torch.equal(x, allp[0]) for x in allp)
        # each rank drew its own batches (different sampler streams)
        s = tr.samples()
        drew = None
        if s is not None:
            mine = torch.cat([t.reshape(-1).long() for t in s])
            got = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(got, mine)
            drew = not all(torch.equal(g, got[0]) for g in got)
        ok = same and type(tr).__name__ == want and drew is True and bool(torch.isfinite(flat).all())
        q.put((rank, f"{model}_dp", bool(ok), type(tr).__name__, drew))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("model,argv,want", [
    ("gcn", ["--dataset", "ppi", "--scale", "0.05", "--batch_size", "16", "--total_step", "4", "--log_steps", "2"],
     "FullFlowTrainer"),
    ("transe", ["--scale", "0.05", "--batch_size", "32", "--total_step", "4", "--log_steps", "2", "--dim", "16"],
     "KGTrainer"),
    ("transe", ["--scale", "0.05", "--batch_size", "32", "--total_step", "4", "--log_steps", "2", "--dim", "16",
                "--sharded"], "RowSparseKGTrainer"),
    ("line", ["--scale", "0.1", "--batch_size", "32", "--total_step", "4", "--log_steps", "2", "--dim", "16",
              "--order", "1", "--sharded"], "RowSparseIdPairTrainer"),
    ("gae", ["--scale", "0.05", "--batch_size", "16", "--total_step", "4", "--log_steps", "2", "--dim", "16",
             "--fanouts", "4", "3"], "GaeTrainer"),
    ("gin", ["--scale", "0.2", "--batch_size", "8", "--total_step", "4", "--log_steps", "2"], "GraphTrainer"),
])
def test_device_trainers_data_parallel_lockstep(tmp_path, model, argv, want):
    res = _run(_worker_device_trainer_dp, str(tmp_path), model, argv, want)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_row_sparse_vs_dense_kg(rank, world, port, q, tmp):
    """one 2-rank step of TransE with the entity table dense in the all-reduced flat buffer
    (KGTrainer) and row-sharded / row-sparse (RowSparseKGTrainer, fixed-capacity all-to-all
    to the owners): Adam's first update of an untouched row is zero and the owners apply
    the ranks' mean row gradient, so both hold the same tables after the step"""
    try:
        _init(rank, world, port)
        from euler_amd.tools import runner

        out = {}
        for sparse in (False, True):
            a = runner.parse_args(["--scale", "0.05", "--batch_size", "32", "--total_step", "1", "--log_steps", "1",
                                   "--dim", "16", "--model_dir", os.path.join(tmp, f"ck_{int(sparse)}_r{rank}"),
                                   "--device_graph", "--device", "cpu", "--seed", "1"], model="transe")
            torch.manual_seed(0)
            _, est = runner.build(a)
            est.params["row_sparse_tables"] = sparse
            est.train()
            out[sparse] = (type(est.device_trainer).__name__, est.device_trainer.logical_params())
        (k0, p0), (k1, p1) = out[False], out[True]
        ok = k0 == "KGTrainer" and k1 == "RowSparseKGTrainer" and set(p0) == set(p1)
        for k in p0:
            ok = ok and torch.allclose(p0[k], p1[k], atol=1e-6)
        q.put((rank, "row_sparse_vs_dense", bool(ok)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_row_sparse_kg_two_ranks_matches_dense_first_step(tmp_path):
    res = _run(_worker_row_sparse_vs_dense_kg, str(tmp_path))
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_dw_shard_ckpt(rank, world, port, q, data_dir, model_dir, out_dir, total):
    """DeepWalk sharded=True through NodeEstimator(device_graph=True) at this world size:
    trains to ``total`` (or, already trained, only restores the per-rank shard checkpoint)
    and dumps this rank's model rows with their weight and sparse-optimizer slots"""
    try:
        _init(rank, world, port)
        import euler_amd as ea
        from euler_amd import models as Z
        from euler_amd.dataset import get_dataset
        from euler_amd.estimator import NodeEstimator

        ds = get_dataset("cora", data_dir=data_dir, scale=0.08)
        ds.load_graph()
        ea.set_seed(3)
        tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
        torch.manual_seed(0)
        m = Z.DeepWalk("train", ["train"], ds.max_node_id, 8, walk_len=3, num_negs=3, sharded=True)
        est = NodeEstimator(m, {"model_dir": model_dir, "batch_size": 32, "total_step": total, "optimizer": "adam",
                                "learning_rate": 0.02, "log_steps": 5, "train_node_type": tnt, "device": "cpu",
                                "device_graph": True, "seed": 11})
        est.train()
        tr = est.device_trainer
        t = tr.inner.table
        rows = tr._half_rows()
        keep = rows < tr.num
        dump = {"step": int(t.step.item()), "global_step": est.global_step}
        for h, key in enumerate(tr._keys):
            sl = slice(h * tr._offw, (h + 1) * tr._offw)
            dump[key] = {"rows": rows[keep].clone(), "weight": t.weight[sl][keep].clone(),
                         "m": t.m[sl][keep].clone(), "v": t.v[sl][keep].clone(),
                         "model": m.state_dict()[key].clone()}
        torch.save(dump, os.path.join(out_dir, "w%d_r%d.pt" % (world, rank)))
        files = sorted(f for f in os.listdir(model_dir) if ".npy" in f)
        q.put((rank, "dw_shard", True, files))
        if dist.is_initialized():
            dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_deepwalk_shard_checkpoint_reshards_rows_and_slots(tmp_path):
    """per-rank shard checkpoints (parallel/shard_io.py): saved by 2 ranks, restored by 1
    and by 4 ranks with identical tables AND sparse-optimizer slots — every rank reads only
    its own rows, no all-gather; the model's tables are views of the trainer's shard"""
    out = tmp_path / "dump"
    out.mkdir()
    ck = str(tmp_path / "ckpt")
    args = (str(tmp_path / "cora"), ck, str(out))
    res = _run(_worker_dw_shard_ckpt, *args, 10, world=2)
    assert not [r for r in res if r[1] == "error"], res
    files = res[0][3]
    # each rank wrote its rows and its Adam slots of both tables (3 kinds x 2 tables x 2 ranks)
    assert len(files) == 12 and any("rank1" in f for f in files), files

    def full(world):
        parts = [torch.load(out / ("w%d_r%d.pt" % (world, r)), weights_only=True) for r in range(world)]
        tabs = {}
        for key in [k for k in parts[0] if isinstance(parts[0][k], dict)]:
            n = sum(int(p[key]["rows"].numel()) for p in parts)
            tab = {k: torch.full((n, 8), float("nan")) for k in ("weight", "m", "v")}
            for p in parts:
                assert torch.equal(p[key]["model"], p[key]["weight"][: p[key]["model"].shape[0]])
                for k in tab:
                    tab[k][p[key]["rows"]] = p[key][k]
            tabs[key] = tab
        return tabs, {p["step"] for p in parts}, {p["global_step"] for p in parts}

    ref, steps, gsteps = full(2)
    assert steps == {10} and gsteps == {10}
    for world in (1, 4):
        res = _run(_worker_dw_shard_ckpt, *args, 10, world=world)
        assert not [r for r in res if r[1] == "error"], res
        got, steps, gsteps = full(world)
        assert steps == {10} and gsteps == {10}
        for key, tab in ref.items():
            for k in ("weight", "m", "v"):
                assert not torch.isnan(tab[k]).any()
                assert torch.equal(got[key][k], tab[k]), (world, key, k)


def _worker_scalable_device(rank, world, port, q, data_dir, model_dir, store):
    """ScalableSageEncoder through NodeEstimator(device_graph=True) on 2 gloo ranks: every
    rank draws its own roots; the flat gradient is all-reduced and the stores are kept
    consistent (replicated: every rank applies every rank's writes; sharded: row r on rank
    r % 2 over all-to-all) -> identical parameters (and replicas) on both ranks"""
    try:
        _init(rank, world, port)
        import euler_amd as ea
        from euler_amd.dataset import get_dataset
        from euler_amd.estimator import NodeEstimator
        from euler_amd.mp_utils.models import SuperviseModel
        from euler_amd.utils import encoders as E

        ds = get_dataset("ppi", data_dir=data_dir, scale=0.05)
        ds.load_graph()
        ea.set_seed(3)

        class M(SuperviseModel):
            def __init__(self):
                super().__init__(ds.label_idx, ds.label_dim)
                self.enc = E.ScalableSageEncoder(["train"], 4, 2, 16, feature_idx=ds.feature_idx,
                                                 feature_dim=ds.feature_dim, max_id=ds.max_node_id)

            def embed(self, n_id):
                return self.enc(n_id)

        torch.manual_seed(0)
        m = M()
        tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
        est = NodeEstimator(m, {"model_dir": model_dir, "batch_size": 16, "total_step": 5, "log_steps": 5,
                                "device": "cpu", "device_graph": True, "train_node_type": tnt, "seed": 1,
                                "device_feature_dtype": "fp32", "historical_store": store})
        est.train()
        flat = torch.cat([v.reshape(-1).float() for k, v in sorted(m.state_dict().items())])
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        same = all(torch.equal(x, allp[0]) for x in allp)
        moved = True
        if store == "replicated":
            s = m.enc.stores(0).contiguous()
            alls = [torch.zeros_like(s) for _ in range(world)]
            dist.all_gather(alls, s)
            same = same and all(torch.equal(x, alls[0]) for x in alls)
        q.put((rank, "scalable_dp", bool(same and moved and est.device_trainer.device_trainer_kind == "scalable"
                                          and est.global_step == 5)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("store", ["replicated", "sharded"])
def test_scalable_device_path_two_ranks_lockstep(tmp_path, store):
    res = _run(_worker_scalable_device, str(tmp_path / "ppi"), str(tmp_path / "ck"), store)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_shared_export(rank, world, port, q, data_dir, same_local=False):
    """DeviceGraph.from_engine(share=True) on 2 ranks of one node: only the host's lowest
    rank runs the engine export (also when a launcher gives both ranks LOCAL_RANK 0, as
    the GPU-sharing tests do); both ranks build the same graph as an unshared upload; the
    shared files are gone afterwards"""
    try:
        _init(rank, world, port)
        if same_local:
            os.environ["LOCAL_RANK"] = "0"
        import glob

        import euler_amd as ea
        import euler_amd.graph.device_graph as DG
        from euler_amd.dataset import get_dataset

        ds = get_dataset("cora", data_dir=data_dir, scale=0.05)
        ds.load_graph()
        ea.set_seed(3)
        calls = []
        orig = DG._export_local

        def counting(*a):
            calls.append(1)
            return orig(*a)

        DG._export_local = counting
        kw = dict(features=["feature"], feature_dims=[1433], label="label", label_dim=ds.label_dim,
                  feature_dtype=torch.float32, seed=1, device="cpu")
        g = DG.DeviceGraph.from_engine(share=True, **kw)
        n_shared = len(calls)
        ref = DG.DeviceGraph.from_engine(**kw)
        same = all(torch.equal(a, b) for a, b in ((g.indptr, ref.indptr), (g.nbr, ref.nbr), (g.cumw, ref.cumw),
                                                  (g.features, ref.features), (g.labels, ref.labels)))
        same = same and np.array_equal(g.ids, ref.ids)
        dist.barrier()
        left = glob.glob("/dev/shm/euler_amd_export_*")
        q.put((rank, "shared_export", bool(same and n_shared == (1 if rank == 0 else 0)), left))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("same_local", [False, True])
def test_device_graph_shared_export_once_per_node(tmp_path, same_local):
    res = _run(_worker_shared_export, str(tmp_path / "cora"), same_local)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res
