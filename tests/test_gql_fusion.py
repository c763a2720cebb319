"""REMOTE fusion pass of the distribute-mode compiler (csrc/gql/gql.cc FuseRemoteNodes;
reference DAGDef::FusionNodes, euler/core/dag_def/dag_def.cc:128-203)."""
import pytest

eng = pytest.importorskip("euler_amd._engine")


def _topological(nodes):
    seen = set()
    for name, _op, _shard, inputs, _inner in nodes:
        for ref in inputs:
            src = ref.split(":")[0]
            if src.startswith(("REMOTE,", "LOCAL,")):
                assert src in seen, f"{name} reads {src} before it is defined"
        seen.add(name)


def test_independent_remotes_of_a_shard_fuse():
    spec = [("REMOTE", 1, ["ids"], 0), ("REMOTE", 2, ["ids"], 0), ("REMOTE", 3, ["ids"], 1)]
    out = eng.fuse_remote_nodes(spec)
    _topological(out)
    by_shard = {}
    for _name, op, shard, _in, inner in out:
        if op == "REMOTE":
            by_shard.setdefault(shard, []).append(inner)
    assert by_shard[0] == [["INNER_1", "INNER_2"]]
    assert by_shard[1] == [["INNER_3"]]


def test_asymmetric_cross_shard_pattern_stays_acyclic():
    """a1(s0), b1(s1), X(local, reads a1), a2(s0, reads b1), b2(s1, reads X).  a2 joins a1's
    group, which then depends on b1's group; b2 depends on that group through X, so it
    must NOT join b1's group (that would be a cycle A -> B -> X -> A)."""
    spec = [
        ("REMOTE", 1, ["ids"], 0),
        ("REMOTE", 2, ["ids"], 1),
        ("LOCAL", 3, ["REMOTE,1:0"], -1),
        ("REMOTE", 4, ["REMOTE,2:0"], 0),
        ("REMOTE", 5, ["LOCAL,3:0"], 1),
    ]
    out = eng.fuse_remote_nodes(spec)
    _topological(out)
    inners = sorted(tuple(x[4]) for x in out if x[1] == "REMOTE")
    assert ("INNER_1", "INNER_4") in inners
    assert ("INNER_2",) in inners and ("INNER_5",) in inners
    assert len(out) == 4


def test_chain_through_local_node_is_not_fused():
    spec = [("REMOTE", 1, ["ids"], 0), ("LOCAL", 2, ["REMOTE,1:0"], -1), ("REMOTE", 3, ["LOCAL,2:0"], 0)]
    out = eng.fuse_remote_nodes(spec)
    _topological(out)
    assert sum(1 for x in out if x[1] == "REMOTE") == 2
