"""Data-parallel step on the GPU box: two ranks on cuda:0 (gloo process group: one GPU per box), each
training 2 of 4 images through FCOSTrainer's HIP-graph segments with the overlapped per-group
gradient all-reduce (dist.GradSync, cvlite/stepper.py), must update the weights as one process
that computes the same two shard gradients with the same kernels, sums them and applies the
trainer's clip + SGD (per-image BN: sharding changes no math) -> rel-L2 of the update <= 1e-5."""
import os
import socket
import sys
import tempfile

import pytest
import torch
import torch.multiprocessing as mp

from conftest import PKG, ROOT

pytestmark = pytest.mark.gpu

C, D, BS = 20, 256, 2


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dp_delta(rank, world):
    """This rank's share of a DP step: its 2 images through the segmented graphs + GradSync."""
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    net = FCOSNet(C, device=torch.device("cuda", 0), seed=0)
    w0 = net.store.flat.clone()
    tr = FCOSTrainer(net, BS, (D, D), world=world, use_graph=True)
    imgs, boxes, nbox = synthetic_batch(world * BS, D, D, C, seed=5, device="cuda")
    sl = slice(rank * BS, (rank + 1) * BS)
    tr.load_batch(imgs[sl].contiguous(), boxes[sl].contiguous(), nbox[sl].contiguous())
    tr.step()
    torch.cuda.synchronize()
    return (net.store.flat - w0).cpu(), len(tr.segs)


def _serial_delta(world):
    """The same step in one process: each shard's gradient from the same kernels (same batch
    composition, so bit-identical per shard), summed, then the trainer's own clip + SGD update
    with inv_bs = 1/(world*bs).  (A single 4-image batch is NOT a valid reference: its split-K
    plans differ, and the random-init graph amplifies 1-ulp differences chaotically.)"""
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    net = FCOSNet(C, device=torch.device("cuda", 0), seed=0)
    w0 = net.store.flat.clone()
    tr = FCOSTrainer(net, BS, (D, D), world=world, use_graph=False)
    imgs, boxes, nbox = synthetic_batch(world * BS, D, D, C, seed=5, device="cuda")
    acc = torch.zeros_like(net.store.grad)
    for r in range(world):
        sl = slice(r * BS, (r + 1) * BS)
        tr.load_batch(imgs[sl].contiguous(), boxes[sl].contiguous(), nbox[sl].contiguous())
        tr._fwd_bwd(None)
        acc += net.store.grad
    net.store.grad.copy_(acc)
    tr._update()
    torch.cuda.synchronize()
    return (net.store.flat - w0).cpu()


def _worker(rank, world, port, out):
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as tdist
    from cvlite import dist
    torch.cuda.set_device(0)
    dist.init_from_env(backend="gloo")
    d, nseg = _dp_delta(rank, world)
    if rank == 0:
        torch.save({"delta": d, "nseg": nseg}, out)
    tdist.barrier()
    tdist.destroy_process_group()


def test_dp_overlapped_allreduce_matches_single_process():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "dp.pt")
        mp.start_processes(_worker, args=(world, _port(), out), nprocs=world, join=True, start_method="spawn")
        got = torch.load(out, weights_only=True)
    ref = _serial_delta(world)
    assert got["nseg"] == 4      # 6 gradient groups, small ones merged (dist.MIN_GROUP_BYTES) -> 4 graph segments
    e = float((got["delta"] - ref).norm() / ref.norm())
    print("DP (2 ranks x 2 images, overlapped all-reduce) vs serial shards: weight-update rel-L2 %.2e" % e)
    assert e < 1e-5


def _nccl_worker(rank, port, out, D=D, BS=BS):
    """One rank on an RCCL ("nccl") process group with the gradient all-reduce forced on: the
    trainer captures its backward in hook-split graph segments and GradSync queues async RCCL
    all-reduces on ProcessGroupNCCL's stream between the segment replays (the N>1 bench path)."""
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1",
                      CVL_DISPATCH="dp_force_sync")
    import torch.distributed as tdist
    from cvlite import dist
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    torch.cuda.set_device(0)
    dist.init_from_env(backend="nccl")
    assert tdist.get_backend() == "nccl"
    net = FCOSNet(C, device=torch.device("cuda", 0), seed=0)
    w0 = net.store.flat.clone()
    tr = FCOSTrainer(net, BS, (D, D), world=1, use_graph=True)
    assert tr.sync is not None and tr.sync.active
    for i in range(2):
        tr.load_batch(*synthetic_batch(BS, D, D, C, seed=11 + i, device="cuda"))
        tr.step()
    torch.cuda.synchronize()
    torch.save({"delta": (net.store.flat - w0).cpu(), "nseg": len(tr.segs)}, out)
    tdist.barrier()
    tdist.destroy_process_group()


@pytest.mark.parametrize("D,BS", [(D, BS), (512, 16)], ids=["256_bs2", "512_bs16"])
def test_rccl_segmented_allreduce_matches_plain_step(D, BS):
    """The RCCL branch of dist.init_from_env + GradSync against HIP-graph segment replay (one GPU per
    box, so one rank: the SUM all-reduce is the identity and the two steps must be bit-identical to
    the same trainer without the collective path).  512 / bs 16 is configs[2]'s per-rank workload:
    the production dispatch (split-K plans, X32 tower segments, deferred weight-gradient reductions
    flushed at each group's hook) under the segmented DP graphs."""
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "nccl.pt")
        mp.start_processes(_nccl_worker, args=(_port(), out, D, BS), nprocs=1, join=True, start_method="spawn")
        got = torch.load(out, weights_only=True)
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import FCOSTrainer, synthetic_batch
    net = FCOSNet(C, device=torch.device("cuda", 0), seed=0)
    w0 = net.store.flat.clone()
    tr = FCOSTrainer(net, BS, (D, D), world=1, use_graph=True)
    assert tr.sync is None
    for i in range(2):
        tr.load_batch(*synthetic_batch(BS, D, D, C, seed=11 + i, device="cuda"))
        tr.step()
    torch.cuda.synchronize()
    assert got["nseg"] == 4
    ref = (net.store.flat - w0).cpu()
    assert torch.equal(got["delta"], ref), float((got["delta"] - ref).abs().max())


def _train_api_worker(rank, world, port, out):
    """cvlite.train_fcos.train (the reference's loop API, FCOS/train_fcos.py:87-251) with world=2:
    each rank trains its shard of the same global sample; the ranks must end bit-identical."""
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import numpy as np
    import torch.distributed as tdist
    from cvlite import dist
    from cvlite.fcos_net import FCOSNet
    from cvlite.train_fcos import SGD, synthetic_batch, train
    torch.cuda.set_device(0)
    dist.init_from_env(backend="gloo")
    D2 = 128
    imgs, boxes, nbox = synthetic_batch(8, D2, D2, C, seed=3, device="cpu")
    data = [dict(image=imgs[i].numpy(), bbox=boxes[i, :int(nbox[i]), :4].numpy(),
                 label=boxes[i, :int(nbox[i]), 4].numpy()) for i in range(8)]
    net = FCOSNet(C, device=torch.device("cuda", 0), seed=0)
    w0 = net.store.flat.clone()
    np.random.seed(123)                      # the same global sample on every rank
    with tempfile.TemporaryDirectory() as td:
        train(data, [], net, 2, SGD(5e-4, 0.9), None, None, 0, 3, display_step=1, step_save=100,
              step_cool=1000, weight_decay=0.0, save_loss_file=os.path.join(td, "l.csv"), world=world)
    torch.cuda.synchronize()
    w = net.store.flat.cpu()
    other = w.clone()
    tdist.broadcast(other, src=0)
    if rank == 1:
        torch.save({"equal": bool(torch.equal(w, other)), "moved": float((w - w0.cpu()).norm()),
                    "finite": bool(torch.isfinite(w).all())}, out)
    tdist.barrier()
    tdist.destroy_process_group()


def test_train_api_data_parallel_world2():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "train.pt")
        mp.start_processes(_train_api_worker, args=(world, _port(), out), nprocs=world, join=True,
                           start_method="spawn")
        got = torch.load(out, weights_only=True)
    assert got["equal"] and got["finite"] and got["moved"] > 0
