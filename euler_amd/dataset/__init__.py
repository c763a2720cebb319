"""Datasets (reference ``tf_euler/python/dataset/*.py``).

``get_dataset(name).load_graph()`` prepares ``<data_dir>/euler`` (the partitioned binary
format) and initialises the embedded graph, like the reference.  The reference
downloads the raw files; this environment has no network, so each dataset

1. converts raw files that are already present in ``data_dir`` (the same file names
   the reference downloads: ``cora.content``/``cora.cites``, ``train.txt`` /
   ``valid.txt`` / ``test.txt`` triples, the TU ``MUTAG_*.txt`` files, GraphSAGE
   ``*-G.json`` / ``*-feats.npy`` / ``*-class_map.json``, ``ratings.dat``), or
2. otherwise builds a **synthetic graph of the same schema and shape** (node/edge
   types, feature names and dims, label dims, split types, relation ids), flagged by
   ``dataset.synthetic = True``.  ``scale`` shrinks the synthetic size for tests.

Every dataset exposes the attributes the reference runners read (``max_node_id``,
``train_node_type``, ``train_edge_type``, ``all_edge_type``, ``total_size``,
``id_file``, ``feature_idx``, ``feature_dim``, ``label_idx``, ``label_dim``,
``num_classes`` ...).
"""
from euler_amd.dataset.base import DataSet, get_dataset, dataset_names  # noqa: F401

__all__ = ["DataSet", "get_dataset", "dataset_names"]
