"""Data-parallel semantics on CPU with the gloo backend (world_size 2): the bucketed SUM all-reduce
of cvlite.dist and the DP step (per-rank image shards, all-reduced gradient / (world*bs), global-norm
clip, Keras SGD) equal the single-process reference step over the union of the shards
(FCOS/train_fcos.py:128-185 restated by oracle/model_ref.py)."""
import os
import socket
import tempfile

import numpy as np
import torch
import torch.distributed as tdist
import torch.multiprocessing as mp

from conftest import PKG, ROOT

C = 20
D = 128
BS = 2          # images per rank


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(n, seed):
    from oracle import fcos_ref
    from cvlite.train_fcos import synthetic_batch
    imgs, boxes, nbox = synthetic_batch(n, D, D, C, seed=seed, device="cpu")
    tg = []
    for b in range(n):
        outs, _ = fcos_ref.format_data(boxes[b, :int(nbox[b])].numpy(), np.array([D, D], np.float32), C,
                                       img_pad=(D, D))
        tg.append(torch.from_numpy(fcos_ref.pack_targets(outs)))
    return imgs, torch.stack(tg)


def _worker(rank, world, port, out_path):
    import sys
    sys.path[:0] = [ROOT, PKG]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    from cvlite import dist
    from cvlite.fcos_net import FCOSNet
    from oracle import model_ref
    dist.init_from_env(backend="gloo")
    # 1) bucketed all-reduce
    x = torch.arange(1000, dtype=torch.float32) * (rank + 1)
    dist.allreduce_grads(x, bucket_bytes=256)
    assert torch.equal(x, torch.arange(1000, dtype=torch.float32) * 3)
    # 2) overlapped per-group all-reduce (GradSync) over the real FCOS parameter layout, fired in
    #    backward order, equals one all-reduce of the whole flat buffer
    from cvlite.layers import ParamStore
    net = FCOSNet.__new__(FCOSNet)
    st = ParamStore()
    net._build_layers(st, C)
    st.finalize("cpu", 0)
    g = torch.Generator().manual_seed(100 + rank)
    for k in st.offsets:
        st.g(k).copy_(torch.randn(st.g(k).shape, generator=g))
    expect = st.grad.clone()
    dist.allreduce_grads(expect)
    sync = dist.GradSync(st, net.grad_groups(), bucket_bytes=1 << 20)
    assert sync.order == ["heads_towers", "fpn", "conv5", "conv4", "conv3", "conv2_stem"]
    for name in sync.order:
        sync.ready(name)
    sync.finish()
    assert torch.equal(st.grad, expect)
    # the plan bench.py's dist block prints: groups in enqueue order, buckets within the cap, the
    # whole flat buffer covered up to alignment gaps
    plan = sync.plan()
    assert [n for n, _ in plan] == ["fpn", "conv5", "conv4", "conv2_stem"]    # heads+fpn, conv3+conv2
    assert all(0 < b <= 1 << 20 for _, bs in plan for b in bs)
    used = sum(st.offsets[k][1] for k in st.offsets) * 4
    assert used <= sum(b for _, bs in plan for b in bs) <= st.grad.numel() * 4
    # 3) DP training step
    params = FCOSNet.param_dict(C, seed=0)                 # identical init on every rank
    imgs, tg = _batch(world * BS, seed=11)
    shard = slice(rank * BS, (rank + 1) * BS)
    names = sorted(params)
    acc = {k: torch.zeros_like(v) for k, v in params.items()}
    for b in range(rank * BS, (rank + 1) * BS):            # per-image grads (batch-1, as the reference)
        _, g, _, _ = model_ref.fcos_loss_and_grads(params, imgs[b:b + 1], tg[b:b + 1], C)
        for k, v in g.items():
            acc[k] += v
    flat = torch.cat([acc[k].reshape(-1) for k in names])
    dist.allreduce_grads(flat)
    flat /= world * BS                                      # divide_no_nan(acc, bs) over the global batch
    norm = float(flat.double().norm())
    flat *= 1.0 / max(norm, 1.0)                            # clip_by_global_norm(., 1.0)
    lr, mom = 5e-4, 0.9
    o = 0
    for k in names:
        n = params[k].numel()
        params[k] -= lr * flat[o:o + n].view_as(params[k])  # first step: v = -lr g, w += v
        o += n
    del shard
    if rank == 0:
        torch.save({k: params[k] for k in names[:40]}, out_path)
    tdist.barrier()
    tdist.destroy_process_group()


def test_dp_step_equals_single_process_reference():
    world = 2
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "dp.pt")
        mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
        got = torch.load(out, weights_only=True)
    from cvlite.fcos_net import FCOSNet
    from oracle import model_ref
    params = FCOSNet.param_dict(C, seed=0)
    moms = {k: torch.zeros_like(v) for k, v in params.items()}
    imgs, tg = _batch(world * BS, seed=11)
    model_ref.train_step_reference(params, moms, imgs, tg, C, 5e-4)
    for k, v in got.items():
        torch.testing.assert_close(v, params[k], rtol=1e-5, atol=1e-7)
