"""Device-step driver shared by the FCOS / RetinaNet / CenterNet trainers.

A trainer provides `_fwd_bwd(hook)` (targets, forward, fused loss, backward; the backward calls
hook(name) as each of the model's `grad_groups()` becomes final) and `_update()` (clip, optimizer,
weight re-pack).  The step is replayed from HIP graphs: with data parallelism the fwd+bwd graph is
captured in SEGMENTS split at the hook points, and between segment replays dist.GradSync launches
the finished groups' RCCL all-reduces (async, on ProcessGroupNCCL's own HIP stream), so the
collectives of the late layers overlap the backward of the early ones; the update graph is queued
behind GradSync.finish() (a stream wait, no host sync).  Without a graph the same hooks fire
eagerly.
"""
import warnings

import torch

from . import dist


class GraphStepper(object):
    def _init_stepper(self, net, world, use_graph):
        self.world = world
        self.use_graph = use_graph
        self.sync = (dist.GradSync(net.store, net.grad_groups())
                     if world > 1 or (dist.force_sync() and torch.distributed.is_initialized()) else None)
        self.segs = None
        self.g_up = None

    def _hook(self, name):
        if self.sync is not None:
            self.sync.ready(name)

    def capture(self):
        """Warm the allocator on a side stream, then capture fwd+bwd (in hook-split segments when
        data-parallel, sharing one memory pool) and the update into HIP graphs."""
        from .checkpoint import model_bns
        # the warm-up forwards must not move the BatchNorm moving statistics: snapshot / restore
        # (the captured graph itself applies exactly one EMA update per replayed step)
        bns = model_bns(self.net)
        snap = [(bn.run_mean.clone(), bn.run_var.clone()) for bn in bns]
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                self._fwd_bwd(None)
        torch.cuda.current_stream().wait_stream(s)
        torch.cuda.synchronize()
        for bn, (m, v) in zip(bns, snap):
            bn.run_mean.copy_(m)
            bn.run_var.copy_(v)
        pool = torch.cuda.graph_pool_handle()
        segs = []
        cap = torch.cuda.Stream()
        with torch.cuda.stream(cap):
            g = torch.cuda.CUDAGraph()
            g.capture_begin(pool=pool)

            def split(name):
                nonlocal g
                if not self.sync.is_boundary(name):      # merged into a later group's launch
                    return
                g.capture_end()
                segs.append((g, name))
                g = torch.cuda.CUDAGraph()
                g.capture_begin(pool=pool)
            self._fwd_bwd(split if self.sync is not None else None)
            with warnings.catch_warnings(record=True) as w:      # the backward may end on a hook:
                warnings.simplefilter("always")                  # then this last graph is empty
                g.capture_end()
            if not any("empty" in str(x.message) for x in w):
                segs.append((g, None))
        torch.cuda.synchronize()
        self.segs = segs
        self.g_up = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_up):
            self._update()
        torch.cuda.synchronize()

    def run_fwd_bwd(self):
        """Forward + backward only (targets, loss and the parameter gradients), replayed from the
        captured segments: the shape-bucketed step (train_fcos.JitterFCOSTrainer) sums several
        buckets' gradients before one update.  No data-parallel hooks on this path."""
        assert self.sync is None, "bucketed gradient accumulation runs without the all-reduce hooks"
        if self.use_graph:
            if self.segs is None:
                self.capture()
            for g, _ in self.segs:
                g.replay()
        else:
            self._fwd_bwd(None)
        return self.losses

    def invalidate(self):
        self.segs = None
        self.g_up = None

    def step(self):
        if self.use_graph:
            if self.segs is None:
                self.capture()
            for g, name in self.segs:
                g.replay()
                if name is not None:
                    self._hook(name)
        else:
            self._fwd_bwd(self._hook)
        if self.sync is not None:
            self.sync.finish()
        if self.use_graph:
            self.g_up.replay()
        else:
            self._update()
        return self.losses
