"""Model zoo (reference ``examples/*``) plus the fused GraphSAGE
flagship used by ``bench.py``.

* :mod:`~euler_amd.models.node_classification` — GraphSAGE, GCN, GAT, FastGCN,
  AdaptiveGCN, AGNN, APPNP, ARMA, DNA, SGCN, TAGCN, GeniePath, LGCN;
* :mod:`~euler_amd.models.unsupervised` — GraphSAGE-unsup, DeepWalk / Node2Vec, LINE,
  DGI, GAE, VGAE, RGCN;
* :mod:`~euler_amd.models.knowledge_graph` — TransE, TransH, TransR, TransD, DistMult;
* :mod:`~euler_amd.models.graph_classification` — GIN, GatedGraph, GraphGCN, Set2Set;
* :mod:`~euler_amd.models.fused_sage` — the device-resident fused GraphSAGE.
"""
from euler_amd.models.graph_classification import GIN, GatedGraph, GraphGCN, Set2SetModel  # noqa: F401
from euler_amd.models.knowledge_graph import DistMult, TransD, TransE, TransH, TransR  # noqa: F401
from euler_amd.models.node_classification import (  # noqa: F401
    AGNN, APPNP, ARMA, DNA, GAT, LGCN, SGCN, TAGCN, AdaptiveGCN, FastGCN, GeniePath, SupervisedGCN,
    SupervisedGNN, SupervisedGraphSage)
from euler_amd.models.unsupervised import (  # noqa: F401
    DGI, DeepWalk, GraphAutoEncoder, Line, Node2Vec, UnsupervisedGraphSage, UnsupervisedRGCN,
    VariationalGraphAutoEncoder)
