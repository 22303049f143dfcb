"""End-to-end parity of the FCOS ResNet-50-FPN forward / loss / backward on the GPU (bf16 MFMA
convs, fp32 accumulation and master weights) against the torch-CPU restatement
(oracle/model_ref.py) on identical weights, images and reference targets, with the oracle storing
activations/gradients in bf16 at the same points (fp32 arithmetic).  At random init this graph is
chaotic (a 0.4% per-layer perturbation grows to ~55% at C5 — measured on the oracle alone, fp32
vs bf16 storage), so the bf16 path is compared with the bf16-storage oracle; the per-block test
below compares each block against the plain fp32 oracle with synchronised inputs.
Tolerances (bf16 activations through ~70 conv+BN layers): predictions and losses rel-L2 <= 3e-2;
gradients rel-L2 <= 6e-2 over all parameters, <= 0.2 per tensor (tensors with non-negligible
gradient; the conv biases in front of a BatchNorm have a mathematically-zero gradient)."""
import numpy as np
import pytest
import torch

from oracle import fcos_ref, model_ref

pytestmark = pytest.mark.gpu


def synth_batch(B, D, C, seed):
    rng = np.random.default_rng(seed)
    nmax = 6
    boxes = np.zeros((B, nmax, 5), np.float32)
    nbox = np.zeros(B, np.int32)
    for b in range(B):
        n = int(rng.integers(1, nmax + 1))
        nbox[b] = n
        for i in range(n):
            h, w = np.exp(rng.uniform(np.log(8 / D), np.log(0.9), 2))
            boxes[b, i] = [rng.uniform(h / 2, 1 - h / 2), rng.uniform(w / 2, 1 - w / 2), h, w, rng.integers(0, C)]
    x = (rng.uniform(-1, 1, size=(B, D, D, 3))).astype(np.float32)
    return x, boxes, nbox


def rel(a, b):
    return float((a - b).norm() / max(b.norm(), 1e-30))


def _run_gpu(net, x, boxes, nbox, C, B, D):
    from cvlite import ops_targets as ot
    xg = torch.from_numpy(x).cuda()
    dims = torch.full((B, 2), float(D), device="cuda")
    tg, _ = ot.fcos_assign(torch.from_numpy(boxes).cuda(), torch.from_numpy(nbox).cuda(), dims, (D, D), C)
    for b in range(B):   # device targets are the reference's (bit-exact)
        outs, _ = fcos_ref.format_data(boxes[b, :nbox[b]], np.array([D, D], np.float32), C, img_pad=(D, D))
        np.testing.assert_array_equal(tg[b].cpu().numpy(), fcos_ref.pack_targets(outs))
    reg, cls = net.forward(xg)
    P = reg.shape[1]
    d_reg = torch.zeros((B, P, 32), dtype=torch.bfloat16, device="cuda")
    d_cls = torch.zeros((B, P, 32), dtype=torch.bfloat16, device="cuda")
    losses, _, _ = ot.fcos_loss(reg, cls, tg, C, grad_scale=1.0 / B, d_reg=d_reg, d_cls=d_cls)
    net.backward(d_reg, d_cls)
    torch.cuda.synchronize()
    return tg.cpu(), reg[..., :5].cpu(), cls[..., :C].cpu(), losses.cpu().double()


def _damp_residual_gammas(net, factor):
    for k in net.store.offsets:
        if k.endswith("_3_bn/gamma"):
            net.store.p(k).mul_(factor)


def test_fcos_train_graph_matches_cpu_oracle():
    """Damped residual-branch gammas (x0.25, so the forward is not chaotic).  Forward, loss and
    backward of the whole graph vs the oracle: predictions/losses within 2e-2 of the bf16-storage
    oracle; every gradient tensor no further from the fp32 oracle than bf16 storage moves the
    oracle itself (ReLU-mask flips from bf16-level forward differences dominate gradient error:
    a single isolated block already shows 5-10% on random upstream gradients).  A wiring error
    (wrong buffer, missing accumulation) shows up as an O(1) excess on specific tensors."""
    from cvlite.fcos_net import FCOSNet
    C, B, D = 20, 2, 256
    net = FCOSNet(C, seed=1)
    _damp_residual_gammas(net, 0.25)
    params = net.store.state_dict()
    x, boxes, nbox = synth_batch(B, D, C, 3)
    tg, reg, cls, losses = _run_gpu(net, x, boxes, nbox, C, B, D)
    with model_ref.emulate_bf16():
        l16, g16, reg16, cls16 = model_ref.fcos_loss_and_grads(params, torch.from_numpy(x), tg, C, grad_scale=1.0 / B)
    l32, g32, reg32, cls32 = model_ref.fcos_loss_and_grads(params, torch.from_numpy(x), tg, C, grad_scale=1.0 / B)
    print("reg %.4f cls %.4f loss %.4f | bf16-oracle vs fp32: reg %.4f cls %.4f" % (
        rel(reg, reg16), rel(cls, cls16), rel(losses, l16.double()), rel(reg16, reg32), rel(cls16, cls32)))
    # 2e-2, or 1.5x the distance bf16 storage alone puts between the oracle and itself (summation
    # order differences, e.g. split-K, are the same size as one bf16 rounding)
    assert rel(reg, reg16) < max(2e-2, 1.5 * rel(reg16, reg32))
    assert rel(cls, cls16) < max(2e-2, 1.5 * rel(cls16, cls32))
    assert rel(losses, l16.double()) < 2e-2
    big = max(float(v.norm()) for v in g32.values())
    excess = []
    for k, gr in g32.items():
        if float(gr.norm()) < 1e-3 * big or k.endswith("_conv/bias"):
            continue      # conv biases in front of BatchNorm: true gradient is zero (pure noise)
        e_gpu, e_emu = rel(net.store.g(k).cpu(), gr), rel(g16[k], gr)
        excess.append((e_gpu - (1.5 * e_emu + 0.03), e_gpu, e_emu, k))
    excess.sort(reverse=True)
    print("worst (excess, gpu, bf16-oracle, tensor):", excess[:4])
    assert excess[0][0] <= 0, excess[:4]


def test_reference_init_deviation_bounded_by_bf16_storage():
    """Reference (Keras glorot) init: the graph is chaotic, so compare how far the GPU result is
    from the fp32 oracle with how far bf16 storage alone moves the oracle itself."""
    from cvlite.fcos_net import FCOSNet
    C, B, D = 20, 2, 256
    net = FCOSNet(C, seed=1)
    params = net.store.state_dict()
    x, boxes, nbox = synth_batch(B, D, C, 3)
    tg, reg, cls, _ = _run_gpu(net, x, boxes, nbox, C, B, D)
    with torch.no_grad():
        reg32, cls32 = model_ref.fcos_forward(torch.from_numpy(x), params, C)
        with model_ref.emulate_bf16():
            reg16, cls16 = model_ref.fcos_forward(torch.from_numpy(x), params, C)
    for g, r32, r16 in ((reg, reg32, reg16), (cls, cls32, cls16)):
        e_gpu, e_emu = rel(g, r32), rel(r16, r32)
        print("gpu-vs-fp32 %.4f  bf16-oracle-vs-fp32 %.4f" % (e_gpu, e_emu))
        assert e_gpu <= 1.5 * e_emu + 0.02


def test_backbone_inference_uses_moving_stats():
    """Keras training=False (infer_fcos / image_detections): every BN normalises with its moving
    mean / variance, not the image's own statistics, and the moving statistics are not updated.
    Non-trivial moving statistics; each block vs the fp32 oracle with moving-statistics BN, fed
    the oracle's own input."""
    import torch.nn.functional as F
    from cvlite.fcos_net import FCOSNet
    C, B, D = 20, 2, 128
    net = FCOSNet(C, seed=2)
    p = net.store.state_dict()
    g = torch.Generator().manual_seed(4)
    moving = {}
    for bn in net.backbone.bns():
        rm = torch.randn(bn.c, generator=g) * 0.3
        rv = torch.rand(bn.c, generator=g) * 2.0 + 0.2
        bn.run_mean.copy_(rm)
        bn.run_var.copy_(rv)
        moving[bn.name] = (rm, rv)

    def bn_inf(x, name, eps=1.001e-5):
        rm, rv = moving[name]
        gm, bt = p[name + "/gamma"].view(1, -1, 1, 1), p[name + "/beta"].view(1, -1, 1, 1)
        return (x - rm.view(1, -1, 1, 1)) / torch.sqrt(rv.view(1, -1, 1, 1) + eps) * gm + bt

    rng = np.random.default_rng(5)
    x = torch.from_numpy(rng.uniform(-1, 1, size=(B, D, D, 3)).astype(np.float32))
    pool, _ = net.backbone.stem.forward(x.cuda(), train=False)
    pool_train, _ = net.backbone.stem.forward(x.cuda(), train=True)
    xn = x.permute(0, 3, 1, 2)
    hr = F.max_pool2d(F.pad(F.relu(bn_inf(model_ref.conv(xn, p, "conv1_conv", 2, pad=3), "conv1_bn")),
                            (1, 1, 1, 1)), 3, 2)
    assert rel(pool.float().cpu().permute(0, 3, 1, 2), hr) < 1e-2
    assert rel(pool_train.float().cpu().permute(0, 3, 1, 2), hr) > 0.1     # the two modes differ
    for bn in net.backbone.bns():                                           # restore (train=True moved them)
        bn.run_mean.copy_(moving[bn.name][0])
        bn.run_var.copy_(moving[bn.name][1])
    H = W = hr.shape[2]
    for si, stage in enumerate(net.backbone.stages):
        for bi, blk in enumerate(stage):
            n = "conv%d_block%d" % (si + 2, bi + 1)
            s = blk.c1.conv.stride
            hin = hr.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda()
            out, H, W, _ = blk.forward(hin, B, H, W, train=False)
            hb = hin.float().cpu().permute(0, 3, 1, 2)
            sc = bn_inf(model_ref.conv(hb, p, n + "_0_conv", s), n + "_0_bn") if bi == 0 else hb
            y = F.relu(bn_inf(model_ref.conv(hb, p, n + "_1_conv", s), n + "_1_bn"))
            y = F.relu(bn_inf(model_ref.conv(y, p, n + "_2_conv"), n + "_2_bn"))
            hr = F.relu(bn_inf(model_ref.conv(y, p, n + "_3_conv"), n + "_3_bn") + sc)
            e = rel(out.float().cpu().permute(0, 3, 1, 2), hr)
            assert e < 1.5e-2, (n, e)
    for bn in net.backbone.bns():
        assert torch.equal(bn.run_mean.cpu(), moving[bn.name][0]) and torch.equal(bn.run_var.cpu(), moving[bn.name][1])


@pytest.mark.parametrize("backbone", ["resnet50", "resnet101"])
def test_backbone_blocks_match_fp32_oracle_with_synced_inputs(backbone):
    """Every ResNet-50 / ResNet-101 block (conv + per-image BN + residual + ReLU, fwd) vs the plain
    fp32 oracle, each fed the oracle's own input: isolates kernel error from the graph's chaotic
    amplification.  (ResNet-101: retinanet_module.py:39-45, the backbone of
    train_retinanet_coco.py:347; taps conv4_block23_out.)"""
    import torch.nn.functional as F
    from cvlite.retina_net import RetinaNetNet
    C, B, D = 20, 2, 256
    net = RetinaNetNet(C, seed=1, backbone_model=backbone)       # retinanet_module.py:30-45
    assert len(net.backbone.stages[2]) == (23 if backbone == "resnet101" else 6)
    p = net.store.state_dict()
    rng = np.random.default_rng(3)
    x = torch.from_numpy(rng.uniform(-1, 1, size=(B, D, D, 3)).astype(np.float32))
    pool, _ = net.backbone.stem.forward(x.cuda())
    xn = x.permute(0, 3, 1, 2)
    hr = F.max_pool2d(F.pad(F.relu(model_ref.bn(model_ref.conv(xn, p, "conv1_conv", 2, pad=3), p, "conv1_bn")),
                            (1, 1, 1, 1)), 3, 2)
    assert rel(pool.float().cpu().permute(0, 3, 1, 2), hr) < 1e-2
    H = W = hr.shape[2]
    for si, stage in enumerate(net.backbone.stages):
        for bi, blk in enumerate(stage):
            n = "conv%d_block%d" % (si + 2, bi + 1)
            s = blk.c1.conv.stride
            hin = hr.permute(0, 2, 3, 1).contiguous().to(torch.bfloat16).cuda()
            out, H, W, _ = blk.forward(hin, B, H, W)
            hb = hin.float().cpu().permute(0, 3, 1, 2)
            sc = model_ref.bn(model_ref.conv(hb, p, n + "_0_conv", s), p, n + "_0_bn") if bi == 0 else hb
            y = F.relu(model_ref.bn(model_ref.conv(hb, p, n + "_1_conv", s), p, n + "_1_bn"))
            y = F.relu(model_ref.bn(model_ref.conv(y, p, n + "_2_conv"), p, n + "_2_bn"))
            hr = F.relu(model_ref.bn(model_ref.conv(y, p, n + "_3_conv"), p, n + "_3_bn") + sc)
            e = rel(out.float().cpu().permute(0, 3, 1, 2), hr)
            assert e < 1.5e-2, (n, e)
