"""Data parallelism over RCCL/xGMI (one process per GPU, torch.distributed backend "nccl" = RCCL).

The reference trains on one device (FCOS/train_fcos.py:128-185); SURVEY.md §8e: images are
independent and BatchNorm statistics are per image, so sharding the batch across ranks changes no
training-mode math.  Rank r processes its own bs images; the step's gradient is
    g = (sum over all ranks' images of grad loss_i) / (world * bs)
= one SUM all-reduce of the flat fp32 gradient buffer, then every rank runs the identical fused
clip + SGD update (the global norm is computed from the reduced gradient, so no extra collective).
"""
import os

import torch
import torch.distributed as tdist
from . import _lib

# 64 MiB buckets: few, large collectives (each RCCL ring step is xGMI-link bound; ~146 MB of fp32
# gradients per FCOS-R50 step -> 3 buckets)
BUCKET_BYTES = 64 << 20
# consecutive gradient groups smaller than this are launched together at the last one's ready point
# (one graph segment boundary and one collective fewer each); the FCOS step's six groups become four
# (heads + towers with the FPN, conv5, conv4, conv3 with conv2 + stem): each cut costs a graph
# launch boundary (~1/3 of the measured one-rank overhead), while the later launch of a small group
# costs no overlap (the collectives finish within ~60 us of their ready point, profiles r05c)
MIN_GROUP_BYTES = 24 << 20


def force_sync():
    """CVL_DISPATCH=dp_force_sync: run the gradient all-reduce path even at world size 1 (a one-rank RCCL
    group exercises ProcessGroupNCCL's stream ordering against the HIP-graph segments on a 1-GPU
    box; the SUM over one rank is the identity, so the step must be bit-identical)."""
    return bool(_lib.dispatch("dp_force_sync"))


def init_from_env(backend=None):
    """torchrun-style env (RANK, WORLD_SIZE, LOCAL_RANK, MASTER_ADDR/PORT).  Returns (rank, world, local)."""
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if (world > 1 or (force_sync() and "MASTER_ADDR" in os.environ)) and not tdist.is_initialized():
        if backend is None:
            backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        tdist.init_process_group(backend=backend)
    return rank, world, local


def bucket_views(flat, bucket_bytes=BUCKET_BYTES):
    n = flat.numel()
    per = max(1, bucket_bytes // flat.element_size())
    return [flat[i:i + per] for i in range(0, n, per)]


def allreduce_grads(flat_grad, group=None, bucket_bytes=BUCKET_BYTES):
    """SUM all-reduce of the flat gradient buffer in large buckets (in place)."""
    if not tdist.is_initialized() or tdist.get_world_size(group) == 1:
        return flat_grad
    works = [tdist.all_reduce(v, op=tdist.ReduceOp.SUM, group=group, async_op=True)
             for v in bucket_views(flat_grad, bucket_bytes)]
    for w in works:
        w.wait()
    return flat_grad


def param_ranges(store, names, bucket_bytes=BUCKET_BYTES):
    """Contiguous [start, end) element ranges of the flat buffer covering `names` (alignment gaps
    between neighbouring tensors are included: their gradients stay 0), split at bucket_bytes."""
    spans = sorted((store.offsets[n][0], store.offsets[n][0] + store.offsets[n][1]) for n in names)
    merged = []
    for a, b in spans:
        if merged and a <= (merged[-1][1] + 15) // 16 * 16:
            merged[-1][1] = max(merged[-1][1], b)
        else:
            merged.append([a, b])
    per = max(1, bucket_bytes // 4)
    out = []
    for a, b in merged:
        for s in range(a, b, per):
            out.append((s, min(s + per, b)))
    return out


class GradSync(object):
    """All-reduce of the flat fp32 gradient buffer overlapped with the backward pass.

    `groups` = [(name, [param names])] in the order the backward pass finalises them; the model's
    backward calls `ready(name)` as soon as a group's gradients are final, which launches that
    group's buckets as async RCCL all-reduces (ProcessGroupNCCL runs them on its own HIP stream,
    ordered after the work already queued on the compute stream), so the collectives of the late
    layers run while the backward of the early layers computes.  `finish()` makes the compute
    stream wait for all of them (no host sync) before the optimizer step.  HIP-graph trainers
    capture the backward in segments split at the ready points and call ready() between replays.
    With world size 1 every call is a no-op."""

    def __init__(self, store, groups, group=None, bucket_bytes=BUCKET_BYTES, min_group_bytes=MIN_GROUP_BYTES):
        self.grad = store.grad
        self.pg = group
        self.order = [n for n, _ in groups]
        names = [k for _, ns in groups for k in ns]
        assert len(names) == len(set(names)) == len(store.offsets), \
            "gradient groups must cover every parameter exactly once"
        # merge consecutive small groups: a merged group is launched at its LAST member's ready point,
        # its ranges coalesced where they touch (one all-reduce for adjacent tensors)
        self.launch_at = {}                     # last member -> the merged group's ranges
        pend, pend_bytes = [], 0
        for i, (n, ns) in enumerate(groups):
            pend += ns
            pend_bytes += sum(store.offsets[k][1] for k in ns) * self.grad.element_size()
            if pend_bytes >= min_group_bytes or i == len(groups) - 1:
                self.launch_at[n] = param_ranges(store, pend, bucket_bytes)
                pend, pend_bytes = [], 0
        self.works = []
        self._cursor = -1                       # ready(): the last group reported this step (order check)
        self.active = tdist.is_initialized() and (tdist.get_world_size(group) > 1 or force_sync())
        # measurement hook (one rank only): keep the segmented graphs, issue no collective -- the
        # segmentation's share of the one-rank overhead (tools/dp_overhead.sh)
        self.segments_only = bool(_lib.dispatch("dp_segments_only")) and self.active and \
            tdist.get_world_size(group) == 1
        self.trace = None

    def is_boundary(self, name):
        """True where ready(name) launches collectives (a graph segment ends only there)."""
        return name in self.launch_at

    def plan(self):
        """[(merged group, [bucket bytes])] in enqueue order (bench.py's dist block)."""
        return [(n, [(b - a) * self.grad.element_size() for a, b in self.launch_at[n]]) for n in self.order
                if n in self.launch_at]

    def begin_trace(self):
        """Time the next step's enqueue points: a HIP event on the compute stream at step start and
        at each group's ready point, and one after the group's all-reduces (recorded on a side
        stream made to wait for RCCL's, so the compute stream is not held).  Read by end_trace()."""
        self.trace = {"t0": torch.cuda.Event(enable_timing=True), "groups": []}
        self.trace["t0"].record()

    def end_trace(self):
        """Per group: (name, bucket bytes, ready ms, all-reduce done ms) from the traced step's start."""
        tr, self.trace = self.trace, None
        torch.cuda.synchronize()
        t0 = tr["t0"]
        return [(n, by, t0.elapsed_time(r), t0.elapsed_time(d) if d is not None else None)
                for n, by, r, d in tr["groups"]]

    def ready(self, name):
        # a merged group launches at its LAST member's ready point, which is only right when the
        # backward reports groups in grad_groups() order: check it (the cursor resets in finish())
        i = self.order.index(name)
        assert i > self._cursor, "gradient group %r reported out of grad_groups() order (after %r)" % (
            name, self.order[self._cursor])
        self._cursor = i
        if not self.active or name not in self.launch_at or self.segments_only:
            return
        ev_r = ev_d = None
        if self.trace is not None:
            ev_r = torch.cuda.Event(enable_timing=True)
            ev_r.record()
        new = [tdist.all_reduce(self.grad[a:b], op=tdist.ReduceOp.SUM, group=self.pg, async_op=True)
               for a, b in self.launch_at[name]]
        self.works += new
        if self.trace is not None:
            side = self.trace.setdefault("side", torch.cuda.Stream())
            with torch.cuda.stream(side):
                for w in new:
                    w.wait()
                ev_d = torch.cuda.Event(enable_timing=True)
                ev_d.record()
            self.trace["groups"].append((name, [(b - a) * self.grad.element_size() for a, b in self.launch_at[name]],
                                         ev_r, ev_d))

    def finish(self):
        for w in self.works:
            w.wait()
        self.works = []
        self._cursor = -1


def max_over_ranks(value, device):
    if not tdist.is_initialized():
        return value
    t = torch.tensor([float(value)], dtype=torch.float64, device=device)
    tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
    return float(t.item())


def barrier():
    if tdist.is_initialized():
        tdist.barrier()
