"""Diagnostic: CenterNet s8 forward (GPU) vs the bf16-storage oracle for C = 1 / 2, eager vs graph."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import numpy as np  # noqa: E402
import torch  # noqa: E402

from cvlite import ops_targets as ot  # noqa: E402
from cvlite.centernet_s8_net import CenterNetS8Net  # noqa: E402
from cvlite.train_centernet_s8 import S8Trainer  # noqa: E402
from oracle import centernet_s8_ref as s8  # noqa: E402
from oracle.model_ref import emulate_bf16  # noqa: E402


def rel(a, b):
    a, b = a.double().cpu(), b.double().cpu()
    return float((a - b).norm() / max(float(b.norm()), 1e-30))


for C, seed in ((2, 1), (1, 2), (2, 2), (1, 1)):
    B, D, ns = 2, 128, 5
    net = CenterNetS8Net(C, n_scales=ns, seed=seed)
    for k in net.store.offsets:
        if k.endswith("_3_bn/gamma"):
            net.store.p(k).mul_(0.25)
    net.pack()
    params = net.store.state_dict()
    x = torch.rand(B, D, D, 3, generator=torch.Generator().manual_seed(8)) * 2 - 1
    reg, cls = net.forward(x.cuda())
    with emulate_bf16():
        _, _, _, (or16, oc16) = s8.loss_and_grads(params, x, torch.zeros(B, 16, 16, ns, 4 + C), C, ns)
    S = D // 8
    print("C=%d seed=%d eager: reg %.4f cls %.4f" % (C, seed, rel(reg.cpu().view(B, S, S, ns, 4), or16),
                                                     rel(cls.cpu().view(B, S, S, ns, C), oc16)), flush=True)
    tr = S8Trainer(net, B, D, n_max=8, init_lr=0.0)
    tr.skip_assign = True
    tr.images.copy_(x.cuda())
    tr.step()
    r2, c2 = tr.outputs
    print("   graph: reg %.4f cls %.4f | graph vs eager cls %.2e" % (
        rel(r2.cpu().view(B, S, S, ns, 4), or16), rel(c2.cpu().view(B, S, S, ns, C), oc16), rel(c2, cls)), flush=True)
