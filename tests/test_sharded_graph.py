"""A graph row-sharded over the data-parallel ranks (graph/sharded_graph.py) with
cross-rank neighbour sampling, and the trainer on it (models/full_trainer.py
ShardedFlowTrainer; reference euler/core/graph/graph.cc:90-98 shard filter,
euler/core/kernels/id_split_op.cc:46-49, remote_op.cc:60-146).

CPU (gloo): the local CSRs partition the whole graph's rows exactly; with 2-3 ranks every
draw is a real out-neighbour of the requested row (with -1 for rows without one), the
per-neighbour frequencies follow the edge weights and the root frequencies the global node
weights; feature / label fetches equal the whole table's rows; one rank reproduces the
unsharded trainer step for step; NodeEstimator(device_graph_sharded=True) trains on 2 ranks
in lockstep holding half of the graph each."""
import math
import os
import sys

import numpy as np
import pytest
import torch
import torch.distributed as dist

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from test_parallel import _init, _run  # noqa: E402


def _graph(n=300, T=2, seed=0, device="cpu"):
    from euler_amd.graph.device_graph import DeviceGraph

    g = torch.Generator().manual_seed(seed)
    deg = torch.randint(0, 9, (n * T,), generator=g)
    deg[7 * T: 7 * T + T] = 0  # a row without out-edges
    indptr = torch.zeros(n * T + 1, dtype=torch.long)
    indptr[1:] = torch.cumsum(deg, 0)
    E = int(indptr[-1])
    nbr = torch.randint(0, n, (E,), generator=g)
    w = torch.rand(E, generator=g) + 0.1
    nw = torch.rand(n, generator=g).numpy() + 0.05
    dg = DeviceGraph.from_csr(indptr.numpy(), nbr.numpy(), w.numpy(), T, node_weights=nw, seed=5, device=device)
    dg.features = torch.randn(n, 12, generator=g).to(device)
    dg.labels = (torch.rand(n, 3, generator=g) > 0.5).float().to(device)
    return dg, indptr, nbr, w, nw


def test_shard_csr_partitions_rows_cpu():
    from euler_amd.graph.sharded_graph import shard_csr

    _, indptr, nbr, w, _ = _graph()
    T, N = 2, 300
    for W in (1, 2, 3):
        for r in range(W):
            lip, ln, lw = shard_csr(indptr.numpy(), nbr.numpy(), w.numpy(), T, W, r)
            for i, row in enumerate(range(r, N, W)):
                for t in range(T):
                    a, b = int(indptr[row * T + t]), int(indptr[row * T + t + 1])
                    la, lb = int(lip[i * T + t]), int(lip[i * T + t + 1])
                    assert np.array_equal(ln[la:lb], nbr[a:b].numpy()) and np.allclose(lw[la:lb], w[a:b].numpy())


def _worker_sampling(rank, world, port, q):
    try:
        _init(rank, world, port)
        from euler_amd.graph.sharded_graph import ShardedDeviceGraph

        g, indptr, nbr, w, nw = _graph()
        sg = ShardedDeviceGraph.from_full(g, node_weights=nw)
        assert sg.local.num_rows == len(range(rank, g.num_rows, world))
        T = 2
        ok = True
        # every draw is a real neighbour of its row over the requested types
        rows = torch.randint(0, g.num_rows, (400,), generator=torch.Generator().manual_seed(rank))
        rows[3] = 7
        rows[10] = -1
        sg.advance()
        sg.reseed_cpu()
        nb, ww, tt = sg.sample_neighbor(rows, 6, edge_types=[1], with_weights=True)
        for k, r in enumerate(rows.tolist()):
            if r < 0 or r == 7:
                ok &= bool((nb[k] == -1).all())
                continue
            a, b = int(indptr[r * T + 1]), int(indptr[r * T + 2])
            cand = set(nbr[a:b].tolist())
            if not cand:
                ok &= bool((nb[k] == -1).all())
            else:
                ok &= set(nb[k].tolist()) <= cand and bool((tt[k] == 1).all())
        # frequencies of one row's neighbours follow the edge weights
        hot = int(torch.argmax(indptr[2::2] - indptr[1::2]))  # the row with the most type-1 edges
        cnt = torch.zeros(g.num_rows)
        for s in range(100):
            sg.advance()
            sg.reseed_cpu()
            d = sg.sample_neighbor(torch.full((60,), hot), 10, edge_types=[1]).reshape(-1).long()
            cnt.index_add_(0, d[d >= 0], torch.ones(int((d >= 0).sum())))
        a, b = int(indptr[hot * T + 1]), int(indptr[hot * T + 2])
        exp = torch.zeros(g.num_rows).index_add_(0, nbr[a:b], w[a:b])
        exp = exp / exp.sum() * cnt.sum()
        tv = float((cnt - exp).abs().sum() / (2 * cnt.sum()))
        ok &= tv < 0.03
        # roots follow the global node weights
        rc = torch.zeros(g.num_rows)
        for s in range(40):
            sg.advance()
            sg.reseed_cpu()
            r = sg.sample_node(1000).long()
            ok &= bool((r >= 0).all())
            rc.index_add_(0, r, torch.ones(r.numel()))
        pe = torch.from_numpy(nw / nw.sum()).float()
        tv_root = float((rc / rc.sum() - pe).abs().sum() / 2)
        ok &= tv_root < 0.06
        # features / labels
        ids = torch.tensor([5, -1, 299, 0, 5, 150])
        f = sg.gather_features(ids)
        ref = torch.where((ids >= 0).unsqueeze(1), g.features[ids.clamp(min=0)], torch.zeros(()))
        ok &= torch.equal(f, ref) and torch.equal(sg.gather_labels(ids[ids >= 0]), g.labels[ids[ids >= 0]])
        sg.check_overflow()
        q.put((rank, "sampling", bool(ok), tv, tv_root))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_sampling_exact_support_and_frequencies(world):
    res = _run(_worker_sampling, world=world)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == world and all(r[2] for r in res), res


def _model(ds):
    from euler_amd import models as Z

    torch.manual_seed(0)
    return Z.SupervisedGNN("gcn", "sage", [16, 16, ds.label_dim], [5, 3], [["train"], ["train"]], "feature",
                           ds.feature_dim, "label", ds.label_dim, max_id=ds.max_node_id)


def test_one_rank_sharded_trainer_equals_unsharded_cpu(tmp_path):
    """one rank: the sharded trainer (exchanges degenerate to local gathers) = the
    unsharded FullFlowTrainer on the same local graph, loss and parameters, 6 steps"""
    import copy

    from euler_amd.dataflow.device_flow import DeviceSageFlow
    from euler_amd.dataset import get_dataset
    from euler_amd.graph.device_graph import DeviceGraph
    from euler_amd.graph.sharded_graph import ShardedDeviceGraph
    from euler_amd.models.full_trainer import FullFlowTrainer, ShardedFlowTrainer

    ds = get_dataset("ppi", data_dir=str(tmp_path / "ppi"), scale=0.05)
    ds.load_graph()
    g = DeviceGraph.from_engine(features=["feature"], feature_dims=[ds.feature_dim], label="label",
                                label_dim=ds.label_dim, feature_dtype=torch.float32, seed=4, device="cpu")
    sg = ShardedDeviceGraph.from_full(g)
    loc = sg.local
    m1 = _model(ds)
    with torch.no_grad():
        from euler_amd.ops import graph_api as G  # noqa: F401
    tr1 = ShardedFlowTrainer.from_model(m1, sg, 32)
    m2 = copy.deepcopy(m1)
    flow = DeviceSageFlow(loc, tr1.flow.edge_types, [5, 3], 32, tr1.flow.self_loops)
    tr2 = FullFlowTrainer(m2, loc, 32, None, features=loc.features, labels=loc.labels, flow=flow)
    # same weights after materialisation (lazy layers): copy tr1's into tr2
    tr2.model.load_state_dict(tr1.model.state_dict())
    tr2.flat.flat.copy_(tr1.flat.flat)
    rng0 = loc.rng.clone()
    l1, l2 = [], []
    for _ in range(6):
        l1.append(float(tr1.step()))
    p1 = tr1.flat.flat.clone()
    loc.rng.copy_(rng0)
    for _ in range(6):
        l2.append(float(tr2.step()))
    assert l1 == l2, (l1, l2)
    assert torch.equal(p1, tr2.flat.flat)


def _worker_estimator(rank, world, port, q, tmp):
    """runner graphsage --device_graph_sharded (the fused tree step on trees drawn across
    the ranks) trains, stays in lockstep, resumes; a non-SAGE convolution on the sampled
    flow (ShardedFlowTrainer) too"""
    try:
        _init(rank, world, port)
        from euler_amd.dataset import get_dataset
        from euler_amd.estimator import NodeEstimator
        from euler_amd.models.full_trainer import ShardedFlowTrainer
        from euler_amd.models.sharded_sage import ShardedSageTrainer
        from euler_amd.tools import runner

        def same_on_all(t):
            allp = [torch.zeros_like(t) for _ in range(world)]
            dist.all_gather(allp, t)
            return all(torch.equal(x, allp[0]) for x in allp)

        flags = ["--dataset", "ppi", "--scale", "0.05", "--batch_size", "32", "--log_steps", "4",
                 "--model_dir", os.path.join(tmp, "ckpt"), "--device_graph_sharded", "--device", "cpu", "--seed", "1",
                 "--fanouts", "5", "3", "--device_feature_dtype", "fp32"]
        a = runner.parse_args(flags + ["--total_step", "8"], model="graphsage")
        _, est = runner.build(a)
        res = est.train()
        tr = est.device_trainer
        n = tr.sgraph.num_rows
        half = tr.sgraph.local.num_rows == len(range(rank, n, world)) and tr.sgraph.features.shard.shape[0] < n
        p = tr.logical_params()
        flat = torch.cat([p[k].reshape(-1).float() for k in sorted(p)])
        ok = (isinstance(tr, ShardedSageTrainer) and half and same_on_all(flat) and est.global_step == 8
              and math.isfinite(res["loss"]))
        a2 = runner.parse_args(flags + ["--total_step", "12"], model="graphsage")
        _, est2 = runner.build(a2)
        est2.train()
        ok &= est2.global_step == 12
        # evaluate / infer on the device in lockstep (batches of 32: rank 0 gets 32 + 16, rank 1 32)
        import euler_amd.ops.graph_api as ge

        ids = torch.as_tensor(ge.sample_node(80, -1)).reshape(-1)
        dist.broadcast(ids, 0)
        idf = os.path.join(tmp, "ids.txt")
        if rank == 0:
            with open(idf, "w") as f:
                f.write("\n".join(str(int(i)) for i in ids.tolist()))
        dist.barrier()
        est2.params["id_file"] = idf
        ev = est2.evaluate()
        est2.params["infer_dir"] = os.path.join(tmp, "infer")
        out_ids, embs = est2.infer()
        ok &= math.isfinite(ev["loss"]) and embs.shape[0] == (48 if rank == 0 else 32) == len(out_ids)
        # another convolution on the sampled flow: the generic trainer over the sharded graph
        ds = get_dataset("ppi", data_dir=os.path.join(tmp, "ppi2"), scale=0.05)
        ds.load_graph()
        m = _model(ds)
        tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
        est3 = NodeEstimator(m, {"model_dir": os.path.join(tmp, "ckpt3"), "batch_size": 32, "total_step": 6,
                                 "log_steps": 3, "device": "cpu", "device_graph": True, "device_graph_sharded": True,
                                 "train_node_type": tnt, "seed": 2, "device_feature_dtype": "fp32"})
        est3.train()
        tr3 = est3.device_trainer
        ok &= isinstance(tr3, ShardedFlowTrainer) and same_on_all(tr3.flat.flat.detach().clone())
        q.put((rank, "sharded_estimator", bool(ok), half))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_estimator_sharded_graph_two_ranks_lockstep(tmp_path):
    res = _run(_worker_estimator, str(tmp_path))
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def test_one_rank_sharded_sage_trainer_equals_sage_trainer_cpu():
    """one rank: the fused-step trainer on trees drawn through the sharded graph = the
    whole-graph SageTrainer (its CPU twin draws the same tree), 5 steps"""
    from euler_amd.graph.sharded_graph import ShardedDeviceGraph
    from euler_amd.models.sage_trainer import SageTrainer
    from euler_amd.models.sharded_sage import ShardedSageTrainer

    g, _, _, _, nw = _graph()
    g.labels = (torch.rand(g.num_rows, 5, generator=torch.Generator().manual_seed(1)) > 0.6).float()
    sg = ShardedDeviceGraph.from_full(g, node_weights=nw)
    loc = sg.local
    kw = dict(metapath=[[0, 1], [1]], init_seed=3, learning_rate=0.01)
    a = ShardedSageTrainer(sg, 32, [4, 3], [16, 16, 8], 5, **kw)
    assert a.D == 12 and a.fshard is None  # one rank: the forward reads the table itself
    b = SageTrainer(loc, 32, [4, 3], [16, 16, 8], 5, features=loc.features, labels=loc.labels, **kw)
    r0 = loc.rng.clone()
    la = [float(a.step()) for _ in range(5)]
    loc.rng.copy_(r0)
    lb = [float(b.step()) for _ in range(5)]
    assert la == lb, (la, lb)
    pa, pb = a.logical_params(), b.logical_params()
    assert all(torch.equal(pa[k], pb[k]) for k in pa)
    # device inference (the estimator's evaluate / infer): same tree draws, same model
    ids = torch.arange(0, 300, 7)
    r1 = loc.rng.clone()
    loc.reseed_cpu()
    ea, xa, ya = a.infer_logits(ids)
    loc.rng.copy_(r1)
    loc.reseed_cpu()
    eb, xb, yb = b.infer_logits(ids)
    assert torch.allclose(xa, xb, atol=1e-5) and torch.equal(ya, yb) and torch.allclose(ea, eb, atol=1e-5)
    ep, xp, yp = a.infer_logits(ids, pad_to=64)  # padded rows touch nothing
    assert xp.shape == xa.shape and bool(torch.isfinite(xp).all()) and torch.equal(yp, ya)


@pytest.mark.gpu
def test_sharded_graph_exchanges_on_the_gpu_one_rank_rccl():
    """the HIP route kernel + RCCL all-to-all path (force_comm on a 1-rank nccl group): every
    draw is a real neighbour, roots are valid rows, feature rows equal the table's"""
    from test_parallel import _free_port

    from euler_amd.graph.sharded_graph import ShardedDeviceGraph

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        g, indptr, nbr, w, nw = _graph(device="cuda")
        sg = ShardedDeviceGraph.from_full(g, force_comm=True, node_weights=nw)
        assert sg.comm and sg.world == 1
        rows = torch.randint(0, g.num_rows, (4096,), device="cuda")
        rows[3] = 7
        sg.advance()
        nb = sg.sample_neighbor(rows, 6, edge_types=[1]).long().cpu()
        for k, r in enumerate(rows.cpu().tolist()):
            a, b = int(indptr[r * 2 + 1]), int(indptr[r * 2 + 2])
            cand = set(nbr[a:b].tolist())
            assert (set(nb[k].tolist()) <= cand) if cand else bool((nb[k] == -1).all()), (k, r)
        roots = sg.sample_node(2048).long()
        assert bool(((roots >= 0) & (roots < g.num_rows)).all())
        ids = torch.tensor([5, -1, 299, 0, 5, 150], device="cuda")
        f = sg.gather_features(ids).float()
        ref = torch.where((ids >= 0).unsqueeze(1), g.features[ids.clamp(min=0)], torch.zeros((), device="cuda"))
        assert torch.equal(f, ref.float())
        # the owners' full-neighbourhood expansion (HIP full_neighbors behind the exchange)
        # = the whole graph's HIP expansion; the flow's blocks too
        _full_flow_matches(g, sg, rows[:300])
        sg.check_overflow()
        torch.cuda.synchronize()
    finally:
        dist.destroy_process_group()


def _full_flow_matches(g, sg, rows):
    from euler_amd.dataflow.device_flow import DeviceFullFlow
    from euler_amd.ops._native import hip

    for mask in (1, 3):
        o1 = torch.zeros(1, dtype=torch.int32, device=rows.device)
        o2 = torch.zeros(1, dtype=torch.int32, device=rows.device)
        a = sg.full_neighbors(rows, mask, 4096, o1)
        b = hip().full_neighbors(g.indptr, g.nbr, g.num_rows, g.num_types, mask, rows.long(), 4096, o2)
        for x, y in zip(a, b):
            assert torch.equal(x.long(), y.long()), mask
        assert int(o1) == 0 == int(o2)
    f1 = DeviceFullFlow(sg, [3, 1], 32, True, "bounded")
    f2 = DeviceFullFlow(g, [3, 1], 32, True, "bounded")
    assert f1.caps == f2.caps
    d1, d2 = f1.produce(rows[:32]), f2.produce(rows[:32])
    for b1, b2 in zip(d1, d2):
        assert torch.equal(b1.n_id, b2.n_id) and torch.equal(b1.edge_index, b2.edge_index)
    assert not f1.overflowed()


@pytest.mark.gpu
def test_sharded_sage_trainer_gpu_matches_bf16_oracle():
    """the fused tree step on a tree drawn through the sharded graph (HIP route kernel +
    RCCL all-to-all on a 1-rank nccl group): loss and gradients match the bf16-aware fp32
    oracle on the same tree and batch labels; every draw is a real edge; it trains"""
    import math

    from test_parallel import _free_port

    from euler_amd.graph.sharded_graph import ShardedDeviceGraph
    from euler_amd.models.sharded_sage import ShardedSageTrainer

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    try:
        g, indptr, nbr, w, nw = _graph(device="cuda")
        g.labels = (torch.rand(g.num_rows, 5, generator=torch.Generator().manual_seed(1)) > 0.6).float().cuda()
        sg = ShardedDeviceGraph.from_full(g, force_comm=True, node_weights=nw)
        tr = ShardedSageTrainer(sg, 64, [4, 3], [64, 64, 32], 5, metapath=[[0, 1], [1]], init_seed=3)
        tr.forward_backward()
        torch.cuda.synchronize()
        loss_k = float(tr.loss_acc.item())
        grads_k = tr.gradients()
        loss_b, grads_b = tr.reference_loss_and_grads_bf16()
        assert abs(loss_k - loss_b) <= 1e-4 * abs(loss_b), (loss_k, loss_b)
        for k in grads_b:
            rel = float((grads_k[k].float().cpu() - grads_b[k].float().cpu()).norm() /
                        grads_b[k].float().cpu().norm().clamp(min=1e-12))
            assert rel < 1e-3, (k, rel)
        roots, nodes, leaf = (t.cpu() for t in tr.samples())
        for i in range(0, nodes.numel(), 7):
            r = int(nodes[i])
            if r < 0:
                continue
            a, b = int(indptr[r * 2 + 1]), int(indptr[r * 2 + 2])
            cand = set(nbr[a:b].tolist())
            got = set(leaf[i].tolist())
            assert (got <= cand) if cand else got == {-1}, (i, r)
        tr.optimizer_step()
        first = None
        for _ in range(60):
            tr.step()
            first = first if first is not None else float(tr.loss.item())
        torch.cuda.synchronize()
        last = float(tr.loss.item())
        assert math.isfinite(last) and last < first, (first, last)
        emb, logits, y = tr.infer_logits(torch.arange(0, 300, 7), pad_to=64)
        assert logits.shape == (43, 5) and bool(torch.isfinite(logits).all())
        assert torch.equal(y.cpu(), g.labels[torch.arange(0, 300, 7)].cpu())
        sg.check_overflow()
    finally:
        dist.destroy_process_group()


def _worker_synth(rank, world, port, q):
    try:
        _init(rank, world, port)
        from euler_amd.graph.sharded_graph import ShardedDeviceGraph

        N = 1001
        g = ShardedDeviceGraph.synthetic(N, 6.0, 64, feature_dim=16, num_classes=5, seed=2, device="cpu")
        loc = g.local
        ok = loc.num_rows == len(range(rank, N, world)) and int(loc.nbr.min()) >= 0 and int(loc.nbr.max()) < N
        ok &= tuple(loc.features.shape) == (loc.num_rows, 16) and loc.labels.shape[0] == loc.num_rows
        # neighbour values reach every owner
        owners = set((loc.nbr.long() % world).unique().tolist())
        ok &= owners == set(range(world))
        g.advance()
        g.reseed_cpu()
        nb = g.sample_neighbor(g.sample_node(64).long(), 4)
        ok &= bool((nb >= 0).all()) and int(nb.max()) < N
        q.put((rank, "synth", bool(ok)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_sharded_synthetic_graph_two_ranks():
    res = _run(_worker_synth)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_shared_gpu(rank, world, port, q):
    """one rank of a 2-process sharded-graph SAGE job sharing the box's GPU (gloo; the
    all-to-alls staged through host memory, parallel/comm.py): each rank holds half of a
    synthetic graph in HBM, draws trees across both, trains the fused step in lockstep"""
    try:
        os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                           "WORLD_SIZE": str(world), "LOCAL_RANK": "0"})
        from euler_amd.graph.sharded_graph import ShardedDeviceGraph
        from euler_amd.models.sharded_sage import ShardedSageTrainer
        from euler_amd.parallel import dp

        dp.init_distributed(backend="gloo", device=torch.device("cuda", 0))
        N = 200_000
        g = ShardedDeviceGraph.synthetic(N, 10.0, 256, feature_dim=64, num_classes=16, seed=5, device="cuda")
        tr = ShardedSageTrainer(g, 256, [10, 5], [64, 64, 32], 16, learning_rate=0.01, init_seed=0)

        def sync(buf):
            host = buf.detach().cpu()
            dist.all_reduce(host)
            buf.copy_(host)
            return 1.0 / world

        losses = []
        for _ in range(30):
            tr.step(sync)
            losses.append(float(tr.loss.item()))
        roots, nodes, leaf = tr.samples()
        ok = bool(((roots >= 0) & (roots < N)).all()) and int(leaf.max()) < N
        flat = tr.flat.detach().cpu().clone()
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        same = all(torch.equal(x, allp[0]) for x in allp)
        g.check_overflow()
        ok &= same and all(math.isfinite(v) for v in losses) and g.local.num_rows == N // world
        q.put((rank, "shared_gpu", bool(ok), losses[0], losses[-1]))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.gpu
def test_sharded_sage_two_ranks_share_the_gpu_in_lockstep():
    res = _run(_worker_shared_gpu)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


@pytest.mark.gpu
def test_sharded_sampled_flow_captures_over_rccl():
    """ShardedFlowTrainer on the sampled flow with its exchanges on a 1-rank RCCL group:
    the step (routes, owner draws, feature / label exchanges, model, Adam) captures into a
    hipGraph; the first captured replay's loss equals the eager step's from the same state
    (fp32 scatter sums: to rounding), and replays train"""
    import copy
    import math

    from test_parallel import _free_port

    from euler_amd import models as Z
    from euler_amd.dataflow.device_flow import DeviceSageFlow
    from euler_amd.graph.sharded_graph import ShardedDeviceGraph
    from euler_amd.models.full_trainer import ShardedFlowTrainer

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    tr = None
    try:
        g, indptr, nbr, w, nw = _graph(device="cuda")
        g.labels = (g.features[:, :3] > 0).float()  # learnable from the root's own features
        sg = ShardedDeviceGraph.from_full(g, force_comm=True, node_weights=nw)
        torch.manual_seed(0)
        m = Z.SupervisedGNN("gcn", "sage", [16, 16, 3], [4, 3], [[0], [0]], "f", 12, "l", 3, max_id=300).cuda()
        tr = ShardedFlowTrainer(m, sg, 32, DeviceSageFlow(sg, [None, None], [4, 3], 32, True), learning_rate=0.03)
        assert tr.capturable()
        tr.step()
        torch.cuda.synchronize()
        rng, flat = sg.rng.clone(), tr.flat.flat.clone()
        st = copy.deepcopy(tr.opt.state_dict())
        tr.step()
        eager_loss = float(tr.loss.item())
        tr.capture(None, warmup=0, steps=1)
        assert tr._graph_exec is not None
        # back to the state before the eager step, then the same step as a replay
        sg.rng.copy_(rng)
        tr.flat.flat.copy_(flat)
        tr.opt.load_state_dict(st)
        tr.replay(1)
        torch.cuda.synchronize()
        first = float(tr.loss.item())
        assert abs(first - eager_loss) <= 1e-5 * abs(eager_loss), (first, eager_loss)
        losses = []
        for _ in range(200):
            tr.replay(1)
            losses.append(tr.loss.clone())
        losses = torch.stack(losses).float().cpu()
        head, tail = float(losses[:20].mean()), float(losses[-20:].mean())
        assert math.isfinite(tail) and tail < 0.97 * head, (head, tail)
        # device inference through the RCCL exchanges (the estimator's collective evaluate)
        tr.release_graphs()
        emb, logits, y = tr.infer_logits(torch.arange(0, 300, 11), pad_to=64)
        assert logits.shape == (28, 3) and bool(torch.isfinite(logits).all())
        assert torch.equal(y.cpu(), g.labels[torch.arange(0, 300, 11)].cpu())
        sg.check_overflow()
    finally:
        if tr is not None:
            tr.release_graphs()  # a graph holding RCCL work blocks destroy_process_group
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_unsup_captures_over_rccl():
    """the sharded unsupervised GraphSAGE step with its exchanges on a 1-rank RCCL group
    captures into a hipGraph; the first replay's loss equals the eager step's from the same
    state; replays train (mean reciprocal rank rises); collective device embeddings"""
    import copy

    from test_parallel import _free_port

    from euler_amd.graph.sharded_graph import ShardedDeviceGraph
    from euler_amd.models.sharded_unsup import ShardedUnsupSageTrainer

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    tr = None
    try:
        g, indptr, nbr, w, nw = _graph(device="cuda")
        sg = ShardedDeviceGraph.from_full(g, force_comm=True, node_weights=nw)
        tr = ShardedUnsupSageTrainer(sg, 64, [4, 3], [32, 32, 16], num_negs=3, pos_edge_types=[0],
                                     metapath=[[0, 1], [1]], learning_rate=0.01, init_seed=3)
        assert tr.fshard is not None and tr.capturable()
        tr.step()
        torch.cuda.synchronize()
        rng, flat = sg.rng.clone(), tr.flat.flat.clone()
        st = copy.deepcopy(tr.opt.state_dict())
        tr.step()
        eager_loss = float(tr.loss.item())
        tr.capture(None, warmup=0, steps=1)
        sg.rng.copy_(rng)
        tr.flat.flat.copy_(flat)
        tr.opt.load_state_dict(st)
        tr.replay(1)
        torch.cuda.synchronize()
        first = float(tr.loss.item())
        assert abs(first - eager_loss) <= 1e-5 * abs(eager_loss), (first, eager_loss)
        tr.reset_metric()
        tr.replay(20)
        m0 = tr.metric()
        tr.replay(300)
        tr.reset_metric()
        tr.replay(20)
        m1 = tr.metric()
        assert m1 > m0, (m0, m1)
        tr.release_graphs()
        e = tr.infer_embed(torch.arange(0, 300, 7), pad_to=64)
        assert e.shape == (43, 16) and bool(torch.isfinite(e).all())
        sg.check_overflow()
    finally:
        if tr is not None:
            tr.release_graphs()
        dist.destroy_process_group()


@pytest.mark.gpu
def test_sharded_full_flow_captures_over_rccl():
    """GCN on full-neighbourhood blocks expanded by the owners through a 1-rank RCCL group:
    no host read in the step, so it captures; the first replay equals the eager step"""
    import copy

    from test_parallel import _free_port

    from euler_amd import models as Z
    from euler_amd.dataflow.device_flow import DeviceFullFlow
    from euler_amd.graph.sharded_graph import ShardedDeviceGraph
    from euler_amd.models.full_trainer import ShardedFlowTrainer

    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{_free_port()}", rank=0, world_size=1)
    tr = None
    try:
        g, indptr, nbr, w, nw = _graph(device="cuda")
        sg = ShardedDeviceGraph.from_full(g, force_comm=True, node_weights=nw)
        torch.manual_seed(0)
        m = Z.SupervisedGNN("gcn", "full", [16, 16, 3], [1, 1], [[0], [0]], "f", 12, "l", 3, max_id=300).cuda()
        tr = ShardedFlowTrainer(m, sg, 32, DeviceFullFlow(sg, [3, 1], 32, True, "bounded"), learning_rate=0.03)
        assert tr.capturable()
        tr.step()
        torch.cuda.synchronize()
        rng, flat = sg.rng.clone(), tr.flat.flat.clone()
        st = copy.deepcopy(tr.opt.state_dict())
        tr.step()
        eager_loss = float(tr.loss.item())
        tr.capture(None, warmup=0, steps=1)
        assert tr._graph_exec is not None
        sg.rng.copy_(rng)
        tr.flat.flat.copy_(flat)
        tr.opt.load_state_dict(st)
        tr.replay(1)
        torch.cuda.synchronize()
        first = float(tr.loss.item())
        assert abs(first - eager_loss) <= 1e-5 * abs(eager_loss), (first, eager_loss)
        tr.replay(50)
        torch.cuda.synchronize()
        assert math.isfinite(float(tr.loss.item()))
        assert not tr.flow.overflowed()
        sg.check_overflow()
    finally:
        if tr is not None:
            tr.release_graphs()
        dist.destroy_process_group()


def _worker_shared_gpu_full(rank, world, port, q):
    """2 ranks sharing the GPU (gloo, staged exchanges): the owners' HIP full-neighbourhood
    expansion of each rank's rows and the flow's blocks = the whole graph's on the device"""
    try:
        os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(rank),
                           "WORLD_SIZE": str(world), "LOCAL_RANK": "0"})
        from euler_amd.graph.sharded_graph import ShardedDeviceGraph
        from euler_amd.parallel import dp

        dp.init_distributed(backend="gloo", device=torch.device("cuda", 0))
        g, indptr, nbr, w, nw = _graph(device="cuda")
        sg = ShardedDeviceGraph.from_full(g, node_weights=nw)
        rows = torch.randint(0, g.num_rows, (300,), generator=torch.Generator().manual_seed(rank)).cuda()
        _full_flow_matches(g, sg, rows)
        sg.check_overflow()
        q.put((rank, "shared_gpu_full", sg.local.num_rows < g.num_rows))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.gpu
def test_sharded_full_flow_two_ranks_share_the_gpu():
    res = _run(_worker_shared_gpu_full)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_engine_shard(rank, world, port, q, data):
    """each rank's engine loads only its partitions (shard_idx = rank); the sharded device
    graph built from them holds the same nodes, neighbour multisets, weights, features and
    labels as the whole graph (compared per node id)"""
    try:
        _init(rank, world, port)
        from euler_amd.graph.sharded_graph import ShardedDeviceGraph
        from euler_amd.ops import base

        eng = base._engine_mod().Engine.from_config({"mode": "local", "data_path": data, "shard_idx": str(rank),
                                                     "shard_num": str(world)})
        full = base._engine_mod().Engine.from_config({"mode": "local", "data_path": data})
        kw = dict(features=["feature"], feature_dims=[8], label="label", label_dim=4, feature_dtype=torch.float32,
                  seed=1, device="cpu")
        g = ShardedDeviceGraph.from_engine_shard(eng, **kw)
        loc = g.local
        ok = g.num_rows % world == 0 and loc.num_rows == g.num_rows // world
        fp = full.export_shard(0, ["dense_feature", "dense_label"], [8, 4])
        fids = np.asarray(fp[0], np.uint64).astype(np.int64)
        find = {int(v): i for i, v in enumerate(fids)}
        T = (len(fp[3]) - 1) // len(fids)
        rid = g.row_ids
        n_local = int((eng.export_shard(0, [], [])[0]).shape[0])
        checked = 0
        for i in range(0, n_local, 7):
            gid = int(rid[i * world + rank])
            j = find[gid]
            for t in range(T):
                a, b = int(fp[3][j * T + t]), int(fp[3][j * T + t + 1])
                want = sorted(zip(np.asarray(fp[4][a:b]).astype(np.int64).tolist(),
                                  np.round(np.asarray(fp[5][a:b], np.float64), 5).tolist()))
                la, lb = int(loc.indptr[i * T + t]), int(loc.indptr[i * T + t + 1])
                nb = loc.nbr[la:lb].long()
                cw = loc.cumw[la:lb].double()
                w = torch.cat([cw[:1], cw[1:] - cw[:-1]]) if lb > la else cw
                got = sorted(zip(rid[nb].tolist(), np.round(w.numpy(), 5).tolist()))
                ok &= [x for x, _ in got] == [x for x, _ in want]
                ok &= np.allclose([y for _, y in got], [y for _, y in want], atol=1e-4)
            ok &= np.allclose(loc.features[i].numpy(), np.asarray(fp[6]).reshape(-1, 8)[j])
            ok &= np.allclose(loc.labels[i].numpy(), np.asarray(fp[7]).reshape(-1, 4)[j])
            checked += 1
        # rows_of maps ids back to rows; draws through the exchanges land on real rows
        ok &= int(g.rows_of([int(rid[rank])])[0]) == rank
        g.advance()
        g.reseed_cpu()
        nb = g.sample_neighbor(g.sample_node(64).long(), 3)
        ok &= bool((rid[nb[nb >= 0].long()] >= 0).all())
        q.put((rank, "engine_shard", bool(ok and checked > 10), checked))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_sharded_graph_from_per_rank_engine_shards(tmp_path):
    import euler_amd as ea

    data = str(tmp_path / "g")
    e = ea.synthetic_graph(3000, 6.0, 64, node_types=1, edge_types=2, feature_dim=8, label_dim=4, seed=3,
                           make_current=False)
    e.save(data, partitions=4, threads=4)
    res = _run(_worker_engine_shard, data)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_engine_shard_estimator(rank, world, port, q, data, tmp):
    """NodeEstimator(device_graph_sharded="engine_shards"): each rank's engine holds half of
    the partitions; a SupervisedGraphSage trains on the fused step in lockstep"""
    try:
        _init(rank, world, port)
        from euler_amd import models as Z
        from euler_amd.estimator import NodeEstimator
        from euler_amd.models.sharded_sage import ShardedSageTrainer
        from euler_amd.ops.base import initialize_graph

        initialize_graph({"mode": "local", "data_path": data, "shard_idx": rank, "shard_num": world})
        torch.manual_seed(0)
        m = Z.SupervisedGraphSage([16, 16, 8], [4, 3], [["0", "1"], ["0", "1"]], "feature", 8, "label", 4,
                                  max_id=2999)
        est = NodeEstimator(m, {"model_dir": os.path.join(tmp, "ck"), "batch_size": 32, "total_step": 6,
                                "log_steps": 3, "device": "cpu", "device_graph": True,
                                "device_graph_sharded": "engine_shards", "seed": 3, "train_node_type": -1,
                                "device_feature_dtype": "fp32"})
        res = est.train()
        tr = est.device_trainer
        p = tr.logical_params()
        flat = torch.cat([p[k].reshape(-1).float() for k in sorted(p)])
        allp = [torch.zeros_like(flat) for _ in range(world)]
        dist.all_gather(allp, flat)
        ok = isinstance(tr, ShardedSageTrainer) and all(torch.equal(x, allp[0]) for x in allp)
        ok &= est.global_step == 6 and math.isfinite(res["loss"]) and tr.sgraph.local.num_rows < 3000
        # evaluate / infer: this rank's engine holds half of the graph, the device path reaches
        # every id through the owners (ids of both halves in every batch)
        idf = os.path.join(tmp, "ids.txt")
        if rank == 0:
            with open(idf, "w") as f:
                f.write("\n".join(str(i) for i in range(0, 3000, 37)))
        dist.barrier()
        est.params["id_file"] = idf
        ev = est.evaluate()
        est.params["infer_dir"] = os.path.join(tmp, "infer")
        out_ids, embs = est.infer()
        rows = tr.sgraph.rows_of(torch.as_tensor(out_ids))
        ok &= math.isfinite(ev["loss"]) and embs.shape[0] == (50 if rank == 0 else 32) == len(out_ids)
        ok &= bool((rows >= 0).all()) and bool(np.isfinite(embs).all()) and bool((np.abs(embs).sum(1) > 0).all())
        q.put((rank, "engine_shard_est", bool(ok)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_estimator_on_per_rank_engine_shards(tmp_path):
    import euler_amd as ea

    data = str(tmp_path / "g")
    e = ea.synthetic_graph(3000, 6.0, 64, node_types=1, edge_types=2, feature_dim=8, label_dim=4, seed=3,
                           make_current=False)
    e.save(data, partitions=4, threads=4)
    res = _run(_worker_engine_shard_estimator, data, str(tmp_path))
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def _worker_full_flow(rank, world, port, q):
    """the owners' full-neighbourhood expansion = the whole graph's, entry for entry; the
    degree statistics and so the flow capacities = the whole graph's; a full-flow block
    stack over the sharded rows = the whole graph's; a short cap flags the overflow"""
    try:
        _init(rank, world, port)
        from euler_amd.dataflow.device_flow import DeviceFullFlow, bounded_caps, exact_caps, full_neighbors_cpu
        from euler_amd.graph.sharded_graph import ShardedDeviceGraph

        g, indptr, nbr, w, nw = _graph(seed=3)
        sg = ShardedDeviceGraph.from_full(g, node_weights=nw)
        ok = True
        gen = torch.Generator().manual_seed(11 + rank)  # every rank asks for different rows
        rows = torch.randint(0, g.num_rows, (90,), generator=gen)
        rows[4], rows[9], rows[20] = -1, 7, rows[3]
        for mask in (1, 2, 3):
            o1, o2 = torch.zeros(1, dtype=torch.int32), torch.zeros(1, dtype=torch.int32)
            a = sg.full_neighbors(rows, mask, 2048, o1)
            b = full_neighbors_cpu(g, mask, rows, 2048, o2)
            ok &= all(torch.equal(x.long(), y.long()) for x, y in zip(a, b)) and int(o1) == 0 == int(o2)
            st = sg.degree_stats(mask, 17)
            T = 2
            seg = (indptr[1:] - indptr[:-1]).view(-1, T)
            deg = sum(seg[:, t] for t in range(T) if (mask >> t) & 1)
            ok &= st == (int(deg.max()), int(deg.sum()), int(torch.topk(deg, 17).values.min()))
        # a cap below the expansion: flagged (the flow regrows and redoes the batch; the
        # per-peer slots may have dropped entries before the cut, so no prefix property)
        o1, o2 = torch.zeros(1, dtype=torch.int32), torch.zeros(1, dtype=torch.int32)
        a = sg.full_neighbors(rows, 3, 64, o1)
        b = full_neighbors_cpu(g, 3, rows, 64, o2)
        ok &= int(o1) == 1 == int(o2) and a[0].shape == b[0].shape
        masks = [3, 1]
        ok &= exact_caps(sg, masks, 24) == exact_caps(g, masks, 24)
        ok &= bounded_caps(sg, masks, 24) == bounded_caps(g, masks, 24)
        f1 = DeviceFullFlow(sg, masks, 24, True, "bounded")
        f2 = DeviceFullFlow(g, masks, 24, True, "bounded")
        roots = torch.randint(0, g.num_rows, (24,), generator=gen)
        d1, d2 = f1.produce(roots), f2.produce(roots)
        for b1, b2 in zip(d1, d2):
            ok &= torch.equal(b1.n_id, b2.n_id) and torch.equal(b1.res_n_id, b2.res_n_id)
            ok &= torch.equal(b1.edge_index, b2.edge_index) and b1.size == b2.size
        ok &= not f1.overflowed()
        sg.check_overflow()
        q.put((rank, "full_flow", bool(ok)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


@pytest.mark.parametrize("world", [2, 3, 4])
def test_sharded_full_neighbourhood_flow_equals_whole_graph(world):
    res = _run(_worker_full_flow, world=world)
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == world and all(r[2] for r in res), res


def _worker_full_flow_estimator(rank, world, port, q, tmp):
    """NodeEstimator(device_graph_sharded=True) on a GCN (full-neighbourhood GCNDataFlow):
    the sharded full-flow trainer trains on 2 ranks in lockstep holding half the rows"""
    try:
        _init(rank, world, port)
        from euler_amd import models as Z
        from euler_amd.dataset import get_dataset
        from euler_amd.estimator import NodeEstimator
        from euler_amd.models.full_trainer import ShardedFlowTrainer

        ds = get_dataset("ppi", data_dir=os.path.join(tmp, "ppi"), scale=0.05)
        ds.load_graph()
        torch.manual_seed(0)
        m = Z.SupervisedGNN("gcn", "full", [16, 16, ds.label_dim], [5, 3], [["train"], ["train"]], "feature",
                            ds.feature_dim, "label", ds.label_dim, max_id=ds.max_node_id)
        tnt = ds.train_node_type[0] if isinstance(ds.train_node_type, list) else ds.train_node_type
        est = NodeEstimator(m, {"model_dir": os.path.join(tmp, "ckpt"), "batch_size": 16, "total_step": 6,
                                "log_steps": 3, "device": "cpu", "device_graph": True, "device_graph_sharded": True,
                                "train_node_type": tnt, "seed": 2, "device_feature_dtype": "fp32"})
        res = est.train()
        tr = est.device_trainer
        allp = [torch.zeros_like(tr.flat.flat) for _ in range(world)]
        dist.all_gather(allp, tr.flat.flat.detach().clone())
        n = tr.graph.num_rows
        ok = (isinstance(tr, ShardedFlowTrainer) and tr.device_trainer_kind == "sharded_full_flow"
              and tr.graph.local.num_rows == len(range(rank, n, world)) and math.isfinite(res["loss"])
              and all(torch.equal(x, allp[0]) for x in allp) and est.global_step == 6)
        # device inference through the owners = the whole graph's full-neighbourhood blocks
        # on the same parameters (each rank its own ids, padded to one size, in lockstep)
        from euler_amd.dataflow.device_flow import DeviceFullFlow
        from euler_amd.graph.device_graph import DeviceGraph
        from euler_amd.models.full_trainer import full_flow_embed

        import euler_amd.ops.graph_api as ge

        all_ids = ge.sample_node(40, tnt)  # the engine holds the whole graph in this test
        all_ids = torch.as_tensor(all_ids).reshape(-1)
        dist.broadcast(all_ids, 0)
        mine = all_ids[:13] if rank == 0 else all_ids[13:40]
        emb, logits, y = tr.infer_logits(mine, pad_to=32)
        whole = DeviceGraph.from_engine(features=["feature"], feature_dims=[ds.feature_dim], label="label",
                                        label_dim=ds.label_dim, feature_dtype=torch.float32, device="cpu")
        rows = whole.rows_of(mine)
        tr.model.eval()
        with torch.no_grad():
            ref_emb, _ = full_flow_embed(tr.gnn, DeviceFullFlow(whole, tr.flow.masks, rows.numel(), tr.flow.self_loops,
                                                                "exact"), whole.features, rows)
            ref_logits = tr.model.out_fc(ref_emb).float()
        tr.model.train()
        chk = {"train": bool(ok), "shape": logits.shape == (mine.numel(), ds.label_dim),
               "logits": float((logits - ref_logits).abs().max()) if logits.shape == ref_logits.shape else -1.0,
               "labels": torch.equal(y, whole.labels[rows].float())}
        ok &= chk["shape"] and chk["logits"] <= 1e-4 * max(1.0, float(ref_logits.abs().max())) and chk["labels"]
        # estimator evaluate / infer over an id file whose batches differ in count per rank
        idf = os.path.join(tmp, "ids.txt")
        if rank == 0:
            with open(idf, "w") as f:
                f.write("\n".join(str(int(i)) for i in all_ids.tolist()))
        dist.barrier()
        est.params["id_file"] = idf
        ev = est.evaluate()
        chk["eval"] = ev
        ok &= math.isfinite(ev["loss"])
        est.params["infer_dir"] = os.path.join(tmp, "infer")
        ids_out, embs = est.infer()
        chk["infer"] = (tuple(embs.shape), len(ids_out))
        ok &= embs.shape[0] == (24 if rank == 0 else 16) and embs.shape[0] == len(ids_out)  # batches 16+8 / 16
        q.put((rank, "full_flow_estimator", bool(ok), chk))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_estimator_sharded_full_flow_two_ranks(tmp_path):
    res = _run(_worker_full_flow_estimator, str(tmp_path))
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res


def test_one_rank_sharded_unsup_equals_unsup_trainer_cpu():
    """one rank: unsupervised GraphSAGE with every draw through the sharded graph = the
    whole-graph trainer's torch twin (same draws in the same order), 5 steps"""
    from euler_amd.graph.sharded_graph import ShardedDeviceGraph
    from euler_amd.models.sage_tower import UnsupSageTrainer
    from euler_amd.models.sharded_unsup import ShardedUnsupSageTrainer

    g, _, _, _, nw = _graph()
    sg = ShardedDeviceGraph.from_full(g, node_weights=nw)
    loc = sg.local
    kw = dict(num_negs=3, pos_edge_types=[0], metapath=[[0, 1], [1]], learning_rate=0.01, init_seed=3)
    a = ShardedUnsupSageTrainer(sg, 32, [4, 3], [16, 16, 8], **kw)
    assert a.fshard is None and not a.towers
    b = UnsupSageTrainer(loc, 32, [4, 3], [16, 16, 8], features=loc.features, **kw)
    r0 = loc.rng.clone()
    la = [float(a.step()) for _ in range(5)]
    loc.rng.copy_(r0)
    lb = [float(b.step()) for _ in range(5)]
    assert la == lb, (la, lb)
    pa, pb = a.logical_params(), b.logical_params()
    assert all(torch.equal(pa[k], pb[k]) for k in pa)
    assert a.metric() == b.metric()
    e = a.infer_embed(torch.arange(0, 300, 7), pad_to=64)
    assert e.shape == (43, 8) and bool(torch.isfinite(e).all())


def _worker_unsup_estimator(rank, world, port, q, tmp):
    """runner graphsage_unsup --device_graph_sharded: the sharded unsupervised trainer on 2
    ranks holding half the rows each, in lockstep; collective device infer"""
    try:
        _init(rank, world, port)
        from euler_amd.models.sharded_unsup import ShardedUnsupSageTrainer
        from euler_amd.tools import runner

        flags = ["--dataset", "cora", "--batch_size", "32", "--log_steps", "4", "--model_dir",
                 os.path.join(tmp, "ckpt"), "--device_graph_sharded", "--device", "cpu", "--seed", "1",
                 "--fanouts", "5", "3", "--device_feature_dtype", "fp32", "--total_step", "8"]
        a = runner.parse_args(flags, model="graphsage_unsup")
        _, est = runner.build(a)
        res = est.train()
        tr = est.device_trainer
        allp = [torch.zeros_like(tr.flat.flat) for _ in range(world)]
        dist.all_gather(allp, tr.flat.flat.detach().clone())
        n = tr.sgraph.num_rows
        ok = (isinstance(tr, ShardedUnsupSageTrainer) and tr.sgraph.local.num_rows == len(range(rank, n, world))
              and all(torch.equal(x, allp[0]) for x in allp) and est.global_step == 8 and math.isfinite(res["loss"]))
        idf = os.path.join(tmp, "ids.txt")
        if rank == 0:
            with open(idf, "w") as f:
                f.write("\n".join(str(i) for i in range(0, 80)))
        dist.barrier()
        est.params["id_file"] = idf
        est.params["infer_dir"] = os.path.join(tmp, "infer")
        calls = []
        orig = tr.infer_embed
        tr.infer_embed = lambda ids, **kw: calls.append(kw) or orig(ids, **kw)  # the device path answers
        out_ids, embs = est.infer()
        ok &= embs.shape[0] == (48 if rank == 0 else 32) == len(out_ids) and bool(np.isfinite(embs).all())
        ok &= len(calls) == 2 and all(c == {"pad_to": 32} for c in calls)  # rank 1 runs a padding batch
        q.put((rank, "unsup_estimator", bool(ok)))
        dist.destroy_process_group()
    except Exception:  # pragma: no cover
        import traceback

        q.put((rank, "error", traceback.format_exc()))


def test_estimator_sharded_unsup_two_ranks(tmp_path):
    res = _run(_worker_unsup_estimator, str(tmp_path))
    assert not [r for r in res if r[1] == "error"], res
    assert len(res) == 2 and all(r[2] for r in res), res
