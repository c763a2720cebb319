"""Synthetic graphs WITH learnable structure, for benchmark learning evidence.

The throughput benchmarks run on synthetic data of the reference configs' shapes (no
network, no dataset downloads).  Uniformly random edges carry nothing to learn, so a
held-out metric on them stays at chance; the generators here plant structure a model of
the benchmarked family can recover, so the committed bench JSONs can report a held-out
metric that must beat chance:

* :func:`lattice_kg` — entities on a 3-D integer lattice, every relation a fixed lattice
  translation: (h, r, t) holds iff pos(t) = pos(h) + off(r).  Exactly the TransE
  hypothesis (h + r = t); the FB15k-shaped config-5 bench trains R-GCN + TransE on it and
  reports tail-ranking MRR / hit@10 on held-out triples.
* :func:`community_graph` — a planted-partition graph (dense inside communities, sparse
  across): a node's walk neighbours share its community, so skip-gram embeddings
  (DeepWalk / LINE, config 4) separate held-out intra-community pairs from random pairs
  (link-prediction AUC).
* :func:`community_labels` — class = community (+ label noise): node classification on
  the same structure (GAT, config 3).

Reference counterparts: the datasets the reference examples train on (examples/TransX,
examples/deepwalk, examples/gat: FB15k, PPI/Cora, ...); these keep their shapes.
"""
from __future__ import annotations

import math

import torch

__all__ = ["synthetic_features", "synthetic_labels", "lattice_kg", "community_graph", "community_labels", "community_features", "tail_ranks", "rank_metrics",
           "auc"]


def lattice_kg(num_ent, num_rel, num_triples, num_test, seed=0, max_off=5):
    """(train (src, rel, dst), test (src, rel, dst)) int64 CPU tensors.  Relation
    frequencies follow a power law (few relations dominate, like FB15k)."""
    g = torch.Generator().manual_seed(int(seed))
    side = int(math.ceil(num_ent ** (1.0 / 3.0)))
    idx = torch.arange(num_ent)
    pos = torch.stack([idx // (side * side), (idx // side) % side, idx % side], 1)
    off = torch.randint(-max_off, max_off + 1, (num_rel, 3), generator=g)
    off[(off == 0).all(1)] = 1
    w = 1.0 / torch.arange(1, num_rel + 1, dtype=torch.float64) ** 1.1
    want = num_triples + num_test
    src_l, rel_l, dst_l, have = [], [], [], 0
    while have < want:
        m = 2 * (want - have) + 1024
        h = torch.randint(0, num_ent, (m,), generator=g)
        r = torch.multinomial(w, m, replacement=True, generator=g)
        p = pos[h] + off[r]
        ok = ((p >= 0) & (p < side)).all(1)
        t = p[:, 0] * side * side + p[:, 1] * side + p[:, 2]
        ok &= t < num_ent
        src_l.append(h[ok])
        rel_l.append(r[ok])
        dst_l.append(t[ok])
        have += int(ok.sum())
    src, rel, dst = (torch.cat(x)[:want] for x in (src_l, rel_l, dst_l))
    return (src[:num_triples], rel[:num_triples], dst[:num_triples]), (src[num_triples:], rel[num_triples:],
                                                                       dst[num_triples:])


def typed_kg(num_ent, num_rel, num_triples, num_types=50, p_in=0.9, cold_frac=0.1, seed=0):
    """Planted typed KG where an entity's type is carried by its neighbourhood.

    Entities 0..num_types-1 are type hubs; every other entity e has a type c(e) and one
    triple (e, rel 0 = "has_type", hub c(e)).  The other num_triples triples link entities
    through relations 1..num_rel-1 (power-law frequencies), the tail drawn from the head's
    type with probability p_in.  A cold_frac of the non-hub entities are *cold*: none of
    their triples is a training (loss) triple, but their link triples stay in the encoder
    graph; the test set is the cold entities' has_type triples — ranking the right hub
    needs the type inferred from the neighbours (message passing), a cold entity's own
    embedding never being trained.

    Returns (train (src, rel, dst), graph (src, rel, dst), test (src, rel, dst)) int64 CPU
    tensors: graph = every link triple (training + cold) + the warm has_type triples."""
    g = torch.Generator().manual_seed(int(seed))
    T = int(num_types)
    ent = torch.arange(T, num_ent)
    ctype = torch.randint(0, T, (num_ent,), generator=g)
    ctype[:T] = torch.arange(T)
    by_type = [ent[ctype[T:] == c] for c in range(T)]
    cold = torch.zeros(num_ent, dtype=torch.bool)
    cold[ent[torch.randperm(ent.numel(), generator=g)[: int(cold_frac * ent.numel())]]] = True
    w = 1.0 / torch.arange(1, num_rel, dtype=torch.float64) ** 1.1
    h = ent[torch.randint(0, ent.numel(), (num_triples,), generator=g)]
    r = 1 + torch.multinomial(w, num_triples, replacement=True, generator=g)
    inside = torch.rand(num_triples, generator=g) < p_in
    t = ent[torch.randint(0, ent.numel(), (num_triples,), generator=g)]
    for c in range(T):  # same-type tails
        sel = inside & (ctype[h] == c)
        k = int(sel.sum())
        if k:
            t[sel] = by_type[c][torch.randint(0, by_type[c].numel(), (k,), generator=g)]
    types = (ent, torch.zeros_like(ent), ctype[ent])
    link_cold = cold[h] | cold[t]
    warm_types = ~cold[ent]
    train = (torch.cat([h[~link_cold], types[0][warm_types]]), torch.cat([r[~link_cold], types[1][warm_types]]),
             torch.cat([t[~link_cold], types[2][warm_types]]))
    graph = (torch.cat([h, types[0][warm_types]]), torch.cat([r, types[1][warm_types]]),
             torch.cat([t, types[2][warm_types]]))
    test = (types[0][~warm_types], types[1][~warm_types], types[2][~warm_types])
    return train, graph, test


def community_graph(num_nodes, num_comm, avg_degree, p_in=0.9, seed=0):
    """(src, dst, comm): ``num_nodes * avg_degree`` directed edges, a fraction ``p_in``
    inside the source's community (community of node i = i % num_comm)."""
    g = torch.Generator().manual_seed(int(seed))
    m = int(num_nodes * avg_degree)
    src = torch.randint(0, num_nodes, (m,), generator=g)
    inside = torch.rand(m, generator=g) < p_in
    per = num_nodes // num_comm
    k = torch.randint(0, per, (m,), generator=g)
    dst_in = (k * num_comm + src % num_comm).clamp_max(num_nodes - 1)
    dst_out = torch.randint(0, num_nodes, (m,), generator=g)
    dst = torch.where(inside, dst_in, dst_out)
    return src, dst, torch.arange(num_nodes) % num_comm


def community_features(comm, dim, signal=0.5, seed=0):
    """[n, dim] node features = signal * (unit centroid of the node's community) + N(0, 1)
    noise / sqrt(dim): one node's own row is a weak community cue, the mean over its
    (mostly same-community) neighbours a strong one — the regime where aggregating the
    neighbourhood (GraphSAGE) beats the node's features alone."""
    g = torch.Generator().manual_seed(int(seed) + 7)
    k = int(comm.max()) + 1
    cent = torch.nn.functional.normalize(torch.randn(k, dim, generator=g), dim=1)
    return signal * cent[comm] + torch.randn(comm.numel(), dim, generator=g) / math.sqrt(dim)


def community_labels(comm, num_classes, noise=0.1, seed=0):
    g = torch.Generator().manual_seed(int(seed) + 1)
    y = comm % num_classes
    flip = torch.rand(comm.numel(), generator=g) < noise
    return torch.where(flip, torch.randint(0, num_classes, (comm.numel(),), generator=g), y)


@torch.no_grad()
def tail_ranks(ent, rel, src, ridx, dst, normalize=True, kind="l2", chunk=1024, cands=None):
    """Raw rank (1 = best) of the true tail among ALL entities (or among the candidate
    entities ``cands``, which must contain every true tail) for each test triple, TransE
    score -|h + r - t| (l1 / l2) on (optionally) l2-normalised rows; ties count against the
    true tail."""
    E = torch.nn.functional.normalize(ent.float(), dim=-1) if normalize else ent.float()
    R = torch.nn.functional.normalize(rel.float(), dim=-1) if normalize else rel.float()
    C = E if cands is None else E[cands]
    col = dst
    if cands is not None:
        pos = torch.full((E.shape[0],), -1, dtype=torch.long, device=E.device)
        pos[cands] = torch.arange(cands.numel(), device=E.device)
        col = pos[dst]
        if bool((col < 0).any()):
            raise ValueError("a true tail is not among the candidates")
    out = []
    for a in range(0, src.numel(), chunk):
        s, r, t = src[a:a + chunk], ridx[a:a + chunk], col[a:a + chunk]
        q = E[s] + R[r]                                        # [c, D]
        d = torch.cdist(q, C, p=1.0 if kind == "l1" else 2.0,
                        compute_mode="donot_use_mm_for_euclid_dist")  # [c, Nc]
        true = d.gather(1, t.view(-1, 1))
        out.append((d <= true).sum(1))
    return torch.cat(out)


def rank_metrics(ranks, ks=(1, 3, 10)):
    r = ranks.double()
    res = {"mrr": float((1.0 / r).mean())}
    for k in ks:
        res["hit@%d" % k] = float((r <= k).double().mean())
    return res


def auc(pos_scores, neg_scores):
    """ROC AUC = P(score(pos) > score(neg)) (ties count half), exact via ranks."""
    s = torch.cat([pos_scores.reshape(-1), neg_scores.reshape(-1)]).double()
    y = torch.cat([torch.ones(pos_scores.numel()), torch.zeros(neg_scores.numel())]).double()
    order = torch.argsort(s)
    ranks = torch.empty_like(s)
    ranks[order] = torch.arange(1, s.numel() + 1, dtype=torch.float64)
    # average ranks of ties
    su, inv, cnt = torch.unique(s, return_inverse=True, return_counts=True)
    rsum = torch.zeros(su.numel(), dtype=torch.float64).index_add_(0, inv, ranks)
    ranks = (rsum / cnt.double())[inv]
    n_pos, n_neg = pos_scores.numel(), neg_scores.numel()
    return float((ranks[y == 1].sum() - n_pos * (n_pos + 1) / 2) / (n_pos * n_neg))


def synthetic_labels(features: torch.Tensor, label_dim: int, chunk: int = 1 << 22) -> torch.Tensor:
    """Learnable synthetic labels: argmax of the first ``label_dim`` feature columns (the
    headline bench's node labels; int16 class ids, the device trainer's compact label mode)."""
    n = features.shape[0]
    out = torch.empty(n, dtype=torch.int16, device=features.device)
    for s in range(0, n, chunk):
        out[s:s + chunk] = features[s:s + chunk, :label_dim].float().argmax(1).to(torch.int16)
    return out


def synthetic_features(n: int, dim: int, seed: int, device, dtype=torch.bfloat16, chunk: int = 1 << 22):
    """[n, dim] random-normal feature table generated on ``device`` in chunks (no host copy of
    a 100M-row table)."""
    g = torch.Generator(device=device)
    g.manual_seed(seed)
    out = torch.empty((n, dim), dtype=dtype, device=device)
    for s in range(0, n, chunk):
        e = min(n, s + chunk)
        out[s:e] = torch.randn((e - s, dim), generator=g, device=device, dtype=torch.float32).to(dtype)
    return out
