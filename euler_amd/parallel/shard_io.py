"""Per-rank checkpoint files of ``mod``-sharded row tables, re-sharded on load.

The reference keeps its large embedding tables as parameter-server variables partitioned
by ``id % num_ps`` and every PS writes its own partition into the checkpoint
(``tf_euler/python/utils/embedding.py:24-68``, ``euler_estimator/python/base_estimator.py:
103-107``).  Here a table of ``num`` rows is row-sharded over ``world`` ranks (global row
``g`` on rank ``g % world`` at local row ``g // world``; ``parallel/sparse_table.py``,
``parallel/embedding.py``) and each rank writes ONLY its own rows, plus the row-sparse
optimizer slots of those rows, next to its ``model.ckpt-<step>-rank<r>.pt``:

    <ckpt stem>.<table>.<kind>.npy        kind in weight / m / v, [rows_of_rank, D] fp32

written in bounded chunks straight from HBM (a 100M x 128 table never has a whole-table
host copy, and no rank ever assembles the whole table).  The small ``.pt`` file keeps a
:func:`shard_meta` per table (``num``, ``world``, ``rank``, ``dim``, file names).

Loading for a run of ``world'`` ranks: every rank reads, for each kind, exactly the rows
``g = j * world' + rank'`` it owns from the old ranks' files (memory-mapped ``.npy``:
``numpy.load(mmap_mode="r")``, no pickle), ``CHUNK_ROWS`` rows at a time — so a
checkpoint written by W ranks restores on any W' with no collective and no all-gather.
"""
from __future__ import annotations

import logging
import os
import re
import time

import numpy as np
import torch

log = logging.getLogger("euler_amd.checkpoint")

__all__ = ["shard_meta", "save_rows", "read_rows", "sidecar_files", "CHUNK_ROWS"]

CHUNK_ROWS = 1 << 22  # 4M rows (2 GiB of 128-d fp32) per host transfer


def _safe(name: str) -> str:
    return re.sub(r"[^A-Za-z0-9_.-]", "_", name)


def sidecar_files(ckpt_path: str):
    """every shard file written next to checkpoint file ``ckpt_path``"""
    stem = ckpt_path[:-3] if ckpt_path.endswith(".pt") else ckpt_path
    d = os.path.dirname(stem) or "."
    base = os.path.basename(stem) + "."
    return [os.path.join(d, f) for f in os.listdir(d) if f.startswith(base) and f.endswith(".npy")]


def shard_meta(num: int, world: int, rank: int, dim: int, files: dict, extra=None) -> dict:
    m = {"num": int(num), "world": int(world), "rank": int(rank), "dim": int(dim), "files": dict(files)}
    m.update(extra or {})
    return m


def save_rows(ckpt_path: str, table: str, tensors: dict, num: int, world: int, rank: int, rows=None) -> dict:
    """Write this rank's rows of table ``table`` (``tensors``: kind -> [n_local, D] tensor
    whose local row j is global row ``j * world + rank``; only its first ``rows`` rows —
    default: every row of the rank below ``num`` — are written) into ``.npy`` files next
    to ``ckpt_path``; returns the :func:`shard_meta` to keep in the ``.pt`` file."""
    stem = ckpt_path[:-3] if ckpt_path.endswith(".pt") else ckpt_path
    n_rank = max(0, -(-(int(num) - int(rank)) // int(world)))  # rows g < num with g % world == rank
    n = n_rank if rows is None else min(int(rows), n_rank)
    files, dim = {}, None
    for kind, t in tensors.items():
        if t is None:
            continue
        t = t.detach()
        dim = int(t.shape[1])
        if t.shape[0] < n:
            raise ValueError(f"shard {table}.{kind}: {t.shape[0]} local rows < {n}")
        fn = "%s.%s.%s.npy" % (os.path.basename(stem), _safe(table), kind)
        path = os.path.join(os.path.dirname(stem) or ".", fn)
        tmp = path + ".tmp"
        # a plain .npy written sequentially: header, then CHUNK_ROWS rows per device->host
        # copy (no mapping of the whole file: host memory stays one chunk)
        t0 = time.time()
        with open(tmp, "wb") as f:
            np.lib.format.write_array_header_1_0(
                f, {"descr": np.lib.format.dtype_to_descr(np.dtype(np.float32)), "fortran_order": False,
                    "shape": (n, dim)})
            for s in range(0, n, CHUNK_ROWS):
                e = min(n, s + CHUNK_ROWS)
                f.write(np.ascontiguousarray(t[s:e].float().cpu().numpy()).tobytes())
        os.replace(tmp, path)
        files[kind] = fn
        log.info("wrote %s: %d rows, %.2f GiB in %.1f s", fn, n, n * dim * 4 / 2 ** 30, time.time() - t0)
    return shard_meta(num, world, rank, dim or 0, files)


def _open(dirname: str, meta: dict, kind: str):
    fn = meta["files"].get(kind)
    if fn is None:
        return None
    return np.load(os.path.join(dirname, fn), mmap_mode="r", allow_pickle=False)


def read_rows(dirname: str, metas, kind: str, rows: torch.Tensor, out: torch.Tensor) -> bool:
    """``out[k] = table[rows[k]]`` for the saved table described by ``metas`` (one
    :func:`shard_meta` per saved rank, any order) for ``kind``; rows outside [0, num) are
    left as they are.  Returns False when the checkpoint has no ``kind`` files (e.g. Adam
    slots restored into an SGD run)."""
    metas = sorted(metas, key=lambda m: m["rank"])
    W = int(metas[0]["world"])
    num = int(metas[0]["num"])
    if len(metas) != W:
        raise ValueError(f"shard checkpoint: {len(metas)} rank files for a world of {W}")
    arrays = [_open(dirname, m, kind) for m in metas]
    if any(a is None for a in arrays):
        return False
    rows = rows.reshape(-1).long().cpu()
    t0 = time.time()
    for s in range(0, rows.numel(), CHUNK_ROWS):
        r = rows[s: s + CHUNK_ROWS]
        ok = (r >= 0) & (r < num)
        owner = torch.remainder(r, W)
        for w, a in enumerate(arrays):
            sel = ok & (owner == w)
            if not bool(sel.any()):
                continue
            local = torch.div(r[sel], W, rounding_mode="floor").numpy()
            if local.size > 1 and np.all(np.diff(local) == 1):
                data = np.asarray(a[int(local[0]): int(local[-1]) + 1])  # one contiguous read
            else:
                data = a[local]
            idx = torch.nonzero(sel).reshape(-1) + s
            out[idx.to(out.device)] = torch.from_numpy(np.array(data, dtype=np.float32)).to(out.device, out.dtype)
    log.info("read %d rows of %s (and its %d-rank siblings) in %.1f s", rows.numel(), metas[0]["files"][kind], W,
             time.time() - t0)
    return True
