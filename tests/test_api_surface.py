"""The reference's public Python surface (SURVEY §2.3, §7.4 "API compatibility surface"):
every name a tf_euler / euler_estimator user reaches for exists here, with the same
call contract where it is cheap to check.  Names are the reference's (tf_euler/python/
euler_ops/*.py, convolution/, dataflow/, graph_pool/, solution/, utils/, dataset/,
euler_estimator/)."""
import importlib

import pytest

GRAPH_OPS = [
    # euler_ops/base.py
    "initialize_graph", "initialize_embedded_graph", "initialize_shared_graph",
    # feature_ops.py
    "get_sparse_feature", "get_edge_sparse_feature", "get_dense_feature", "get_edge_dense_feature",
    "get_binary_feature", "get_edge_binary_feature",
    # neighbor_ops.py
    "sparse_get_adj", "sample_neighbor", "get_top_k_neighbor", "sample_fanout_with_feature",
    "sample_neighbor_layerwise", "get_full_neighbor", "get_sorted_full_neighbor", "sample_fanout",
    "sample_fanout_layerwise_each_node", "sample_fanout_layerwise", "get_multi_hop_neighbor",
    # sample_ops.py
    "sample_node", "sample_edge", "sample_node_with_src", "get_graph_by_label", "sample_graph_label",
    "sample_n_with_types",
    # type_ops.py
    "get_node_type_id", "get_edge_type_id", "get_node_type",
    # walk_ops.py / util_ops.py
    "random_walk", "gen_pair", "inflate_idx", "sparse_gather",
    # mp_ops.py
    "gather", "scatter_add", "scatter_max", "scatter_mean", "scatter_", "scatter_softmax",
    # euler.start (service launcher)
    "start",
]

MODULES = {
    "euler_amd.convolution": ["Conv", "GCNConv", "SAGEConv", "GATConv", "GINConv", "GraphConv", "AGNNConv",
                              "APPNPConv", "ARMAConv", "DNAConv", "SGCNConv", "TAGConv", "GatedConv",
                              "RelationConv"],
    "euler_amd.dataflow": ["DataFlow", "Block", "NeighborDataFlow", "UniqueDataFlow", "SageDataFlow",
                           "GCNDataFlow", "FastGCNDataFlow", "LayerwiseDataFlow", "LayerwiseEachDataFlow",
                           "WholeDataFlow", "RelationDataFlow"],
    "euler_amd.graph_pool": ["Pooling", "AttentionPool", "Set2SetPool"],
    "euler_amd.solution": ["SuperviseSolution", "UnsuperviseSolution", "SuperviseSampleSolution",
                           "UnsuperviseSampleSolution", "DenseLogits", "PosNegLogits", "CosineLogits",
                           "GetLabelFromFea", "SamplePosWithTypes", "SampleNegWithTypes"],
    "euler_amd.estimator": ["BaseEstimator", "NodeEstimator", "EdgeEstimator", "GraphEstimator", "GaeEstimator",
                            "SampleEstimator"],
    "euler_amd.dataset": ["get_dataset"],
    "euler_amd.utils.encoders": ["ShallowEncoder", "GCNEncoder", "GenieEncoder", "ScalableGCNEncoder",
                                 "SageEncoder", "ShuffleSageEncoder", "SageEncoderNew", "ScalableSageEncoder",
                                 "LayerEncoder", "SparseSageEncoder", "LGCEncoder"],
    "euler_amd.mp_utils": ["BaseGNNNet", "JKGNNNet", "SuperviseModel", "UnsuperviseModel"],
}


@pytest.mark.parametrize("name", GRAPH_OPS)
def test_graph_op_names(name):
    import euler_amd as ea

    assert callable(getattr(ea, name)), name


@pytest.mark.parametrize("module", sorted(MODULES))
def test_library_names(module):
    m = importlib.import_module(module)
    missing = [n for n in MODULES[module] if not hasattr(m, n)]
    assert not missing, missing


@pytest.mark.parametrize("module", ["layers", "metrics", "encoders", "aggregators", "sparse_aggregators",
                                    "optimizers", "embedding", "hooks", "flags", "to_dense_adj",
                                    "to_dense_batch"])
def test_utils_modules(module):
    """tf_euler.utils.{encoders, aggregators, layers, metrics, optimizers, embedding, hooks, flags}"""
    importlib.import_module("euler_amd.utils." + module)


def test_estimator_params_contract(tmp_path):
    """params keys of the reference runners are accepted (run_graphsage.py:67-75)."""
    from euler_amd.estimator import NodeEstimator

    params = {"train_node_type": 0, "batch_size": 8, "optimizer": "adam", "learning_rate": 0.01, "log_steps": 5,
              "model_dir": str(tmp_path), "id_file": "", "infer_dir": str(tmp_path), "total_step": 1,
              "infer_type": "node", "label": ["label"], "num_classes": 2, "epoch": 1}
    est = NodeEstimator(lambda x: x, params)
    assert est.model_dir == str(tmp_path)
