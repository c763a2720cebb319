"""JSON graph -> Euler on-disk format (meta + partitioned Node/Edge data + indexes).

Same inputs and the same byte layout as the reference's offline tools
(``euler/tools/generate_euler_data.py:28-50``, ``json2meta.py``, ``json2partdat.py``,
``json2partindex.py``; format in SURVEY §2.9), so directories written here load in
either engine.  Deliberate fixes:

* every (node, edge type) neighbor group is sorted by neighbor id;
* in-neighbor lists are filled (the reference converter left them empty, so
  ``inV`` / in-neighbor sampling returned nothing).

JSON input: ``{"nodes": [{id, type, weight, features: [{name, type, value}]}],
"edges": [{src, dst, type, weight, features}]}``.  Index meta (optional) uses the
reference's ``"name:valuetype:idtype:hash_index|range_index|neighbor_index"`` strings.
"""
from __future__ import annotations

import json
import os
import shutil
import struct
from collections import OrderedDict, defaultdict

__all__ = ["EulerGenerator", "convert_json", "edge_id_hash"]

_TYPE_CODES = ["int8_t", "int16_t", "int32_t", "int64_t", "uint8_t", "uint16_t", "uint32_t", "uint64_t",
               "float", "double", "bool", "string"]
_FMT = {"int8_t": "b", "int16_t": "h", "int32_t": "i", "int64_t": "q", "uint8_t": "B", "uint16_t": "H",
        "uint32_t": "I", "uint64_t": "Q", "float": "f", "double": "d", "bool": "?"}
_FTYPE = {"sparse": 0, "dense": 1, "binary": 2}


def _s(x) -> bytes:
    if not isinstance(x, bytes):
        x = str(x).encode()
    return struct.pack("<I", len(x)) + x


def _vec(fmt: str, v) -> bytes:
    v = list(v)
    return struct.pack("<I", len(v)) + (struct.pack("<%d%s" % (len(v), fmt), *v) if v else b"")


def _val(vtype: str, v) -> bytes:
    if vtype == "string":
        return _s(v)
    return struct.pack("<" + _FMT[vtype], v)


def edge_id_hash(src: int, dst: int, etype: int) -> int:
    """MurmurHash3-x64 based edge id (reference data_types.h:48-56), via the C++ engine."""
    from euler_amd.ops._native import engine

    return int(engine().edge_id_hash(int(src), int(dst), int(etype)))


class _Meta:
    def __init__(self, partitions: int):
        self.partitions = partitions
        self.node_types = OrderedDict()
        self.edge_types = OrderedDict()
        self.node_meta = OrderedDict()  # name -> (ftype, idx)
        self.edge_meta = OrderedDict()
        self.node_dim = {}
        self.edge_dim = {}
        self.counts = {"node": {"sparse": 0, "dense": 0, "binary": 0}, "edge": {"sparse": 0, "dense": 0, "binary": 0}}
        self.node_count = 0
        self.edge_count = 0

    def _feat(self, kind, f):
        name = f["type"] + "_" + f["name"]
        meta = self.node_meta if kind == "node" else self.edge_meta
        dims = self.node_dim if kind == "node" else self.edge_dim
        t, v = f["type"], f["value"]
        if name not in dims:
            dims[name] = 0
        if t == "sparse":
            for i in v:
                dims[name] = max(int(i), dims[name])
        elif t == "dense":
            dims[name] = len(v)
        if name not in meta:
            self.counts[kind][t] += 1
            meta[name] = (t, self.counts[kind][t] - 1)

    def parse(self, data):
        self.node_count = len(data["nodes"])
        self.edge_count = len(data["edges"])
        for n in data["nodes"]:
            t = str(n["type"])
            if t not in self.node_types:
                self.node_types[t] = len(self.node_types)
            for f in n.get("features", []):
                self._feat("node", f)
        for e in data["edges"]:
            t = str(e["type"])
            if t not in self.edge_types:
                self.edge_types[t] = len(self.edge_types)
            for f in e.get("features", []):
                self._feat("edge", f)

    def write(self) -> bytes:
        s = _s("graph") + _s("2.0") + struct.pack("<QQI", self.node_count, self.edge_count, self.partitions)
        for meta, dims in ((self.node_meta, self.node_dim), (self.edge_meta, self.edge_dim)):
            s += struct.pack("<I", len(meta))
            for name, (t, idx) in meta.items():
                s += _s(name) + struct.pack("<iiq", _FTYPE[t], idx, dims[name])
        for types in (self.node_types, self.edge_types):
            s += struct.pack("<I", len(types))
            for name, idx in types.items():
                s += _s(name) + struct.pack("<I", idx)
        return s


def _features_block(meta, feats) -> bytes:
    by = {"sparse": {}, "dense": {}, "binary": {}}
    for f in feats:
        name = f["type"] + "_" + f["name"]
        t, idx = meta[name]
        by[t][idx] = f["value"]
    out = b""
    for t, fmt in (("sparse", "Q"), ("dense", "f"), ("binary", None)):
        n = max([i for (tt, i) in meta.values() if tt == t], default=-1) + 1
        idx_list, vals = [], []
        acc = 0
        for i in range(n):
            v = by[t].get(i, [] if t != "binary" else "")
            if t == "binary":
                v = v.encode() if isinstance(v, str) else bytes(v)
                vals.append(v)
            else:
                vals.extend(v)
            acc += len(v)
            idx_list.append(acc)
        out += _vec("i", idx_list)
        if t == "binary":
            out += _s(b"".join(vals))
        else:
            out += _vec(fmt, [int(x) for x in vals] if t == "sparse" else [float(x) for x in vals])
    return out


def _neighbor_block(groups, n_types) -> bytes:
    """groups: etype -> [(nbr, w)] ; weights stored as prefix sums running across groups."""
    group_ids, group_w, groups_idx, nbrs, cum = [], [], [], [], []
    acc_idx, acc_w = 0, 0.0
    for t in range(n_types):
        lst = sorted(groups.get(t, []), key=lambda x: x[0])
        acc_idx += len(lst)
        groups_idx.append(acc_idx)
        tw = 0.0
        for nb, w in lst:
            nbrs.append(int(nb))
            acc_w += float(w)
            tw += float(w)
            cum.append(acc_w)
        group_ids.append(t)
        group_w.append(tw)
    return (_vec("i", group_ids) + _vec("f", group_w) + _vec("i", groups_idx) + _vec("Q", nbrs) + _vec("f", cum))


class EulerGenerator:
    """``EulerGenerator(graph_json, index_meta, out_dir, partition_num).do()`` (reference API)."""

    def __init__(self, graph_json, index_meta, out_dir, partition_num=1, prefix="graph", partition_fn=None):
        self.graph_json = graph_json
        self.index_meta = index_meta
        self.out_dir = out_dir
        self.partition_num = int(partition_num)
        # node id -> partition (edges follow their source); default id % partition_num, the
        # layout remote mode routes by.  Any other assignment (a min-cut partitioner's) is
        # served by mode=graph_partition.
        P = self.partition_num
        self.partition_fn = partition_fn if partition_fn is not None else (lambda i: int(i) % P)
        self.prefix = prefix

    def _load(self, x):
        if isinstance(x, dict):
            return x
        with open(x) as f:
            return json.load(f)

    def do(self):
        data = self._load(self.graph_json)
        P = self.partition_num
        if os.path.exists(self.out_dir):
            shutil.rmtree(self.out_dir)
        os.makedirs(os.path.join(self.out_dir, "Node"))
        os.makedirs(os.path.join(self.out_dir, "Edge"))
        meta = _Meta(P)
        meta.parse(data)
        with open(os.path.join(self.out_dir, "euler.meta"), "wb") as f:
            f.write(meta.write())
        n_et = max(len(meta.edge_types), 1)
        out_nb = defaultdict(lambda: defaultdict(list))
        in_nb = defaultdict(lambda: defaultdict(list))
        for e in data["edges"]:
            t = meta.edge_types[str(e["type"])]
            out_nb[e["src"]][t].append((e["dst"], e["weight"]))
            in_nb[e["dst"]][t].append((e["src"], e["weight"]))
        node_files = [bytearray() for _ in range(P)]
        for n in data["nodes"]:
            rec = struct.pack("<Qif", int(n["id"]), meta.node_types[str(n["type"])], float(n["weight"]))
            rec += _neighbor_block(out_nb.get(n["id"], {}), n_et)
            rec += _neighbor_block(in_nb.get(n["id"], {}), n_et)
            rec += _features_block(meta.node_meta, n.get("features", []))
            node_files[self._part(n["id"])] += struct.pack("<I", len(rec)) + rec
        edge_files = [bytearray() for _ in range(P)]
        for e in data["edges"]:
            rec = struct.pack("<QQif", int(e["src"]), int(e["dst"]), meta.edge_types[str(e["type"])], float(e["weight"]))
            rec += _features_block(meta.edge_meta, e.get("features", []))
            edge_files[self._part(e["src"])] += struct.pack("<I", len(rec)) + rec
        for p in range(P):
            with open(os.path.join(self.out_dir, "Node", "%s_%d.dat" % (self.prefix, p)), "wb") as f:
                f.write(node_files[p])
            with open(os.path.join(self.out_dir, "Edge", "%s_%d.dat" % (self.prefix, p)), "wb") as f:
                f.write(edge_files[p])
        if self.index_meta:
            _write_indexes(data, self._load(self.index_meta), meta, self.out_dir, P, self._part)
        return self.out_dir

    def _part(self, node_id):
        p = int(self.partition_fn(int(node_id)))
        if not 0 <= p < self.partition_num:
            raise ValueError(f"partition_fn({node_id}) = {p} is not in [0, {self.partition_num})")
        return p


def _index_keys(spec):
    """all 'name:vtype:idtype:kind' strings inside an index meta dict."""
    out = []
    stack = [spec]
    while stack:
        v = stack.pop()
        if isinstance(v, str):
            out.append(v)
        elif isinstance(v, dict):
            stack.extend(v.values())
    return out


def _write_indexes(data, spec, meta, out_dir, P, part_of=None):
    part_of = part_of or (lambda i: int(i) % P)
    per_part = [defaultdict(list) for _ in range(P)]  # key -> [(value, id, weight)] or neighbor dict
    nbr_node_vals = defaultdict(dict)  # neighbor-index key -> node id -> (value, id, w)
    edge_nbr = defaultdict(lambda: defaultdict(list))  # key -> src -> [(value, dst, w)]

    def add(key, value, iid, w, part):
        if key.endswith("neighbor_index"):
            nbr_node_vals[key][iid] = (value, iid, w)
        else:
            per_part[part][key].append((value, iid, w))

    node_spec = spec.get("node", {})
    for n in data["nodes"]:
        part = part_of(n["id"])
        fs = node_spec.get("features", {})
        for f in n.get("features", []):
            if f["name"] in fs:
                sel = fs[f["name"]]
                if isinstance(sel, dict):
                    for vidx, key in sel.items():
                        add(key, f["value"][int(vidx)], n["id"], n["weight"], part)
                else:
                    add(sel, f["value"], n["id"], n["weight"], part)
        for k, key in node_spec.items():
            if k != "features" and k in n:
                add(key, n[k], n["id"], n["weight"], part)
    edge_spec = spec.get("edge", {})
    for e in data["edges"]:
        part = part_of(e["src"])
        etno = meta.edge_types[str(e["type"])]
        iid = edge_id_hash(e["src"], e["dst"], etno)
        fs = edge_spec.get("features", {})
        for f in e.get("features", []):
            if f["name"] in fs:
                for vidx, key in fs[f["name"]].items():
                    v = f["value"][int(vidx)]
                    if key.endswith("neighbor_index"):
                        edge_nbr[key][e["src"]].append((v, e["dst"], e["weight"]))
                    else:
                        per_part[part][key].append((v, iid, e["weight"]))
        for k, key in edge_spec.items():
            if k != "features" and k in e:
                v = e[k]  # raw JSON value, like the reference (json2partindex.py parse_edge)
                if key.endswith("neighbor_index"):
                    edge_nbr[key][e["src"]].append((v, e["dst"], e["weight"]))
                else:
                    per_part[part][key].append((v, iid, e["weight"]))
    # node neighbor index: per edge src, the values of its destinations
    nbr_data = [defaultdict(lambda: defaultdict(list)) for _ in range(P)]
    for key, vals in nbr_node_vals.items():
        for e in data["edges"]:
            if e["dst"] in vals:
                nbr_data[part_of(e["src"])][key][e["src"]].append(vals[e["dst"]])
    for key, d in edge_nbr.items():
        for src, lst in d.items():
            nbr_data[part_of(src)][key][src].extend(lst)

    for key in _index_keys(spec):
        name, vtype, idtype, kind = key.split(":")
        d = os.path.join(out_dir, "Index", name)
        os.makedirs(d, exist_ok=True)
        kcode = {"hash_index": 0, "range_index": 1, "neighbor_index": 2}[kind]
        with open(os.path.join(d, "meta"), "wb") as f:
            f.write(struct.pack("<iii", kcode, _TYPE_CODES.index(idtype), _TYPE_CODES.index(vtype)))
        for p in range(P):
            if kind == "hash_index":
                groups = OrderedDict()
                for v, iid, w in per_part[p].get(key, []):
                    groups.setdefault(v, ([], []))
                    groups[v][0].append(iid)
                    groups[v][1].append(w)
                blob = b"".join(_val(vtype, v) + struct.pack("<I", len(ids)) + b"".join(_val(idtype, i) for i in ids)
                                + _vec("f", ws) for v, (ids, ws) in groups.items())
            elif kind == "range_index":
                blob = _range_blob(per_part[p].get(key, []), vtype, idtype)
            else:
                blob = b"".join(_val(idtype, root) + _range_blob(lst, vtype, idtype)
                                for root, lst in nbr_data[p].get(key, {}).items())
            with open(os.path.join(d, "index_%d.dat" % p), "wb") as f:
                f.write(blob)


def _range_blob(items, vtype, idtype):
    items = sorted(items, key=lambda x: x[0])
    out = struct.pack("<I", len(items)) + b"".join(_val(idtype, i) for _, i, _ in items)
    out += struct.pack("<I", len(items)) + b"".join(_val(vtype, v) for v, _, _ in items)
    cum, acc = [], 0.0
    for _, _, w in items:
        acc += w
        cum.append(acc)
    return out + _vec("f", cum)


def convert_json(graph_json, out_dir, partition_num=1, index_meta=None, partition_fn=None):
    return EulerGenerator(graph_json, index_meta, out_dir, partition_num, partition_fn=partition_fn).do()
