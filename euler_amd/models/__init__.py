"""Model zoo (reference ``examples/*``) plus the device-path trainers
(:mod:`~euler_amd.models.sage_trainer` — the fused GraphSAGE step ``bench.py`` measures,
:mod:`~euler_amd.models.sage_tower` — unsupervised GraphSAGE).

* :mod:`~euler_amd.models.node_classification` — GraphSAGE, GCN, GAT, FastGCN,
  AdaptiveGCN, AGNN, APPNP, ARMA, DNA, SGCN, TAGCN, GeniePath, LGCN;
* :mod:`~euler_amd.models.unsupervised` — GraphSAGE-unsup, DeepWalk / Node2Vec, LINE,
  DGI, GAE, VGAE, RGCN;
* :mod:`~euler_amd.models.knowledge_graph` — TransE, TransH, TransR, TransD, DistMult;
* :mod:`~euler_amd.models.graph_classification` — GIN, GatedGraph, GraphGCN, Set2Set;
"""
from euler_amd.models.graph_classification import GIN, GatedGraph, GraphGCN, Set2SetModel  # noqa: F401
from euler_amd.models.knowledge_graph import DistMult, TransD, TransE, TransH, TransR  # noqa: F401
from euler_amd.models.node_classification import (  # noqa: F401
    AGNN, APPNP, ARMA, DNA, GAT, LGCN, SGCN, TAGCN, AdaptiveGCN, FastGCN, GeniePath, ScalableGCN, ScalableSage,
    SupervisedGCN, SupervisedGNN, SupervisedGraphSage)
from euler_amd.models.unsupervised import (  # noqa: F401
    DGI, DeepWalk, GraphAutoEncoder, Line, Node2Vec, UnsupervisedGraphSage, UnsupervisedRGCN,
    VariationalGraphAutoEncoder)
