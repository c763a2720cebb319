"""Graph-captured training step for the engine-path GraphSAGE estimator loop.

With the native batch pipeline in static mode (dataflow/native_loader.py) every batch
arrives in one set of fixed-capacity device tensors, and a model whose convolutions all
run the fused fixed-fanout SAGE kernel (SAGEConv.fused_relu, csrc/hip/sage.hip) has no
data-dependent shapes or host syncs left in forward, backward or the fused Adam update.
The whole step — forward, sigmoid-CE loss, device metric accumulation, backward, Adam —
is then captured once into a hipGraph and replayed: one launch per step instead of ~70
PyTorch kernel launches whose host cost (≈1.4 ms) dominated the step.

Steps: the first ``warm`` steps run eagerly on a side stream over the static inputs
(they allocate the optimizer state, the metric accumulators and the BLAS workspaces,
and are real training steps), the next step is captured and replayed, every later step
only replays.  Capacity padding rows carry -1 neighbour / self indices (the kernel's
zero row) and never reach the roots, so results are exact for the valid rows.

Reference mechanics replaced: the reference estimator runs each step as one
tf.estimator session.run over the static TF graph it built
(euler_estimator/python/base_estimator.py:123-142); here the static graph is the
captured hipGraph.
"""
from __future__ import annotations

import logging
import os

import torch

log = logging.getLogger("euler_amd")

__all__ = ["GraphedTrainStep", "graph_step_blocker"]


def graph_step_blocker(est, feat_dim):
    """None when the estimator's step (native pipeline inputs of ``feat_dim`` input
    features) can be captured, else the reason it cannot."""
    from euler_amd.convolution.convs import SAGEConv
    from euler_amd.mp_utils.models import BaseGNNNet, SuperviseModel

    if est.params.get("cuda_graph", "auto") in (False, "0", "false", "off"):
        return "disabled (params cuda_graph)"
    if est.device.type != "cuda":
        return "not on a GPU"
    if est.world != 1:
        return "multi-rank gradient sync is not captured"
    if est.params.get("amp"):
        return "autocast"
    if os.environ.get("EULER_AMD_FUSED_CONV", "1") == "0":
        return "fused SAGE conv disabled"
    m = est.model
    if type(m).forward is not SuperviseModel.forward:
        return "custom model forward"
    gnn = getattr(m, "gnn", None)
    if not isinstance(gnn, BaseGNNNet) or type(gnn).forward is not BaseGNNNet.forward or gnn.whole_graph:
        return "model is not a fixed-fanout BaseGNNNet"
    if not all(isinstance(c, SAGEConv) and type(c).fused_relu is SAGEConv.fused_relu for c in gnn.convs):
        return "a convolution without the fused fixed-fanout kernel"
    widths = [int(feat_dim)] + [c.self_fc.weight.shape[0] for c in gnn.convs]
    if max(widths) > 512:
        return "layer width above the fused kernel's 512"
    opt = est.optimizer
    if not isinstance(opt, torch.optim.Adam) or not opt.defaults.get("fused"):
        return "optimizer is not the fused Adam"
    if est._extra_losses() is not None or any(callable(getattr(x, "after_backward", None))
                                              for x in m.modules() if x is not m):
        return "extra losses / after-backward hooks"
    return None


class GraphedTrainStep:
    def __init__(self, est, loader, warm=3):
        self.est = est
        self.loader = loader
        self.warm = int(warm)
        self.graph = None
        self.loss = self.metric_name = self.metric = None
        for g in est.optimizer.param_groups:
            g["capturable"] = True
        for st in est.optimizer.state.values():
            if torch.is_tensor(st.get("step")) and not st["step"].is_cuda:
                st["step"] = st["step"].to(est.device, torch.float32)

    def _eager(self, source):
        est = self.est
        _, loss, name, metric = est._run_model(source)
        est.optimizer.zero_grad(set_to_none=True)
        loss.backward()
        est.optimizer.step()
        # detached: a live autograd graph keeps its AccumulateGrad nodes (bound to the
        # stream they were created on) alive into the capture, which then breaks
        return loss.detach(), name, metric

    def step(self, source):
        """One training step over the static inputs ``source`` (already filled for this
        step on the current stream); returns (loss tensor, metric name, metric).  The
        caller must not hold any autograd graph of an earlier step."""
        cur = torch.cuda.current_stream()
        if self.graph is None and self.warm > 0:
            self.warm -= 1
            side = torch.cuda.Stream()
            side.wait_stream(cur)
            with torch.cuda.stream(side):
                out = self._eager(source)
            cur.wait_stream(side)
            return out
        if self.graph is None:
            self.est.optimizer.zero_grad(set_to_none=True)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, capture_error_mode="thread_local"):
                _, loss, name, metric = self.est._run_model(source)
                loss.backward()
                self.est.optimizer.step()
            self.graph, self.loss, self.metric_name, self.metric = g, loss, name, metric
            log.info("training step captured into a hipGraph (replayed from now on)")
        self.graph.replay()
        return self.loss, self.metric_name, self.metric
