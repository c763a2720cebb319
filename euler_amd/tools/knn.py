"""k-nearest-neighbour retrieval over inferred embeddings (reference ``knn/knn.py``).

The reference wraps faiss ``IndexIVFFlat`` (``ncent = 4 * sqrt(n)``, ``nprobe = 10``,
L2).  faiss is not available here; this module implements the same two index types
directly on torch tensors, so on an MI355X the k-means training, the coarse
assignment and the candidate scoring are GEMMs on the GPU (rocBLAS/hipBLASLt via
``torch.matmul``) and the top-k selections are device sorts:

* :class:`FlatIndex` — exact search, ``||q||^2 - 2 q.x + ||x||^2`` in query chunks;
* :class:`IVFFlatIndex` — Lloyd k-means coarse quantiser, padded inverted lists, search
  over the ``nprobe`` closest lists.

CLI (same flags as the reference)::

    python -m euler_amd.tools.knn --embedding_file embedding_0.npy --id_file ids_0.npy \
        [--query_file q.csv] [--index_type ivfflat|flat] [--k 10] [--out result.npz]

(the reference read the ids from ``embedding_file`` by mistake and pickled the result;
here ids come from ``id_file`` and the result is an ``.npz`` with ``distance`` / ``idx``.)
"""
from __future__ import annotations

import argparse
import math

import numpy as np
import torch

__all__ = ["FlatIndex", "IVFFlatIndex", "build_index", "kmeans"]


def _dev(device):
    if device is not None:
        return torch.device(device)
    return torch.device("cuda") if torch.cuda.is_available() else torch.device("cpu")


def _sqdist(q, x, x_norm=None):
    """squared L2 distances [nq, nx]"""
    qn = (q * q).sum(1, keepdim=True)
    xn = (x * x).sum(1) if x_norm is None else x_norm
    return (qn - 2.0 * (q @ x.t()) + xn.unsqueeze(0)).clamp_min_(0.0)


class FlatIndex:
    def __init__(self, d, device=None, chunk=8192):
        self.d, self.device, self.chunk = d, _dev(device), chunk
        self.xb = torch.zeros(0, d, device=self.device)
        self.xn = torch.zeros(0, device=self.device)

    def add(self, x):
        x = torch.as_tensor(x, dtype=torch.float32, device=self.device)
        self.xb = torch.cat([self.xb, x])
        self.xn = (self.xb * self.xb).sum(1)

    @property
    def ntotal(self):
        return self.xb.shape[0]

    def search(self, q, k):
        q = torch.as_tensor(q, dtype=torch.float32, device=self.device)
        k = min(int(k), self.ntotal)
        ds, ids = [], []
        for s in range(0, q.shape[0], self.chunk):
            d = _sqdist(q[s:s + self.chunk], self.xb, self.xn)
            v, i = torch.topk(d, k, dim=1, largest=False)
            ds.append(v)
            ids.append(i)
        return torch.cat(ds).cpu().numpy(), torch.cat(ids).cpu().numpy()


def kmeans(x, ncent, iters=20, seed=0, min_points_per_centroid=4):
    """Lloyd k-means on the device; empty clusters are re-seeded from random points."""
    n = x.shape[0]
    ncent = max(1, min(int(ncent), n // max(min_points_per_centroid, 1) or 1))
    g = torch.Generator(device="cpu").manual_seed(seed)
    cent = x[torch.randperm(n, generator=g)[:ncent].to(x.device)].clone()
    for _ in range(iters):
        assign = torch.cat([_sqdist(x[s:s + 65536], cent).argmin(1) for s in range(0, n, 65536)])
        sums = torch.zeros_like(cent).index_add_(0, assign, x)
        cnt = torch.bincount(assign, minlength=ncent).to(x.dtype)
        empty = cnt == 0
        cent = torch.where(empty.unsqueeze(1), cent, sums / cnt.clamp_min(1).unsqueeze(1))
        if bool(empty.any()):
            ridx = torch.randint(0, n, (int(empty.sum()),), generator=g).to(x.device)
            cent[empty] = x[ridx]
    return cent


class IVFFlatIndex:
    def __init__(self, d, ncent, nprobe=10, device=None, min_points_per_centroid=4, iters=20):
        self.d, self.ncent, self.nprobe = d, int(ncent), int(nprobe)
        self.device = _dev(device)
        self.min_pts, self.iters = min_points_per_centroid, iters
        self.cent = None
        self.xb = None

    def train(self, x):
        x = torch.as_tensor(x, dtype=torch.float32, device=self.device)
        self.cent = kmeans(x, self.ncent, self.iters, min_points_per_centroid=self.min_pts)
        self.ncent = self.cent.shape[0]

    def add(self, x):
        x = torch.as_tensor(x, dtype=torch.float32, device=self.device)
        self.xb = x if self.xb is None else torch.cat([self.xb, x])
        assign = torch.cat([_sqdist(self.xb[s:s + 65536], self.cent).argmin(1)
                            for s in range(0, self.xb.shape[0], 65536)])
        order = torch.argsort(assign, stable=True)
        counts = torch.bincount(assign, minlength=self.ncent)
        maxl = int(counts.max()) if counts.numel() else 0
        starts = torch.cumsum(counts, 0) - counts
        pos = torch.arange(order.numel(), device=self.device) - starts[assign[order]]
        lists = torch.full((self.ncent, max(maxl, 1)), -1, dtype=torch.long, device=self.device)
        lists[assign[order], pos] = order
        self.lists = lists
        self.xn = (self.xb * self.xb).sum(1)

    @property
    def ntotal(self):
        return 0 if self.xb is None else self.xb.shape[0]

    def search(self, q, k, chunk=1024):
        q = torch.as_tensor(q, dtype=torch.float32, device=self.device)
        nprobe = min(self.nprobe, self.ncent)
        ds, ids = [], []
        for s in range(0, q.shape[0], chunk):
            qq = q[s:s + chunk]
            probe = torch.topk(_sqdist(qq, self.cent), nprobe, dim=1, largest=False).indices  # [Q, nprobe]
            cand = self.lists[probe].reshape(qq.shape[0], -1)  # [Q, nprobe * maxl]
            valid = cand >= 0
            cz = cand.clamp_min(0)
            xc = self.xb[cz]  # [Q, C, d]
            d = ((qq * qq).sum(1, keepdim=True) - 2.0 * torch.einsum("qd,qcd->qc", qq, xc) + self.xn[cz])
            d = torch.where(valid, d.clamp_min(0.0), torch.full_like(d, float("inf")))
            kk = min(int(k), d.shape[1])
            v, i = torch.topk(d, kk, dim=1, largest=False)
            got = torch.gather(cand, 1, i)
            got = torch.where(torch.isinf(v), torch.full_like(got, -1), got)
            ds.append(v)
            ids.append(got)
        return torch.cat(ds).cpu().numpy(), torch.cat(ids).cpu().numpy()


def build_index(embedding, index_type="ivfflat", device=None):
    n, d = embedding.shape
    if index_type == "flat":
        idx = FlatIndex(d, device)
    elif index_type == "ivfflat":
        idx = IVFFlatIndex(d, int(4 * math.sqrt(n)), nprobe=10, device=device)
        idx.train(embedding)
    else:
        raise ValueError("unknown index_type %r (flat | ivfflat)" % index_type)
    idx.add(embedding)
    return idx


def main(argv=None):
    p = argparse.ArgumentParser(description="kNN over inferred embeddings")
    p.add_argument("--embedding_file", required=True)
    p.add_argument("--id_file", default=None)
    p.add_argument("--query_file", default=None, help="CSV of query vectors (default: first 25 embeddings)")
    p.add_argument("--index_type", default="ivfflat")
    p.add_argument("--k", type=int, default=10)
    p.add_argument("--out", default="result.npz")
    p.add_argument("--device", default=None)
    a = p.parse_args(argv)
    emb = np.load(a.embedding_file, allow_pickle=False).astype(np.float32)
    ids = np.load(a.id_file, allow_pickle=False).reshape(-1) if a.id_file else np.arange(len(emb))
    assert len(ids) == len(emb), "ids and embeddings differ in length"
    index = build_index(emb, a.index_type, a.device)
    query = np.loadtxt(a.query_file, dtype=np.float32, delimiter=",", ndmin=2) if a.query_file else emb[:25]
    D, I = index.search(query, a.k)
    res_ids = np.where(I >= 0, ids[np.clip(I, 0, None)], -1)
    np.savez(a.out, distance=D, idx=res_ids)
    print("wrote %s: %d queries x %d neighbours" % (a.out, D.shape[0], D.shape[1]))
    return D, res_ids


if __name__ == "__main__":
    main()
