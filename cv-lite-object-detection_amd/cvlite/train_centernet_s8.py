"""CenterNet ResNet stride-8 training on MI355X — mirrors CenterNet/train_centernet_crowdhuman.py
(img_dims 512, batch 16, sub_batch 1, box_scales [32..512], SGD momentum 0.9, lr 0.01 / 10 / 100
at steps 20000 / 25000, floor min_lr) over tf_centernet_resnet_s8.train_step (:387-444).

`S8Trainer` runs a whole step on the device: targets (cvl_centernet_s8_assign), forward (per-image
BN), the fused model_loss forward + backward (cls_lambda = reg_lambda = 1), backward, (RCCL
all-reduce), divide_no_nan(g, batch), clip_by_global_norm(1.0), Keras SGD, head assembly + bf16
re-pack — captured into HIP graphs and replayed.
"""
import torch

from . import ops_nn as nn
from . import ops_targets as ot
from .stepper import GraphStepper

BOX_SCALES = (32.0, 64.0, 128.0, 256.0, 512.0)     # train_centernet_crowdhuman.py:225


def crowdhuman_lr(step, init_lr=0.01, min_lr=1.0e-5):
    """train_centernet_crowdhuman.py:39-45."""
    if step < 20000:
        lr = init_lr
    elif step < 25000:
        lr = init_lr / 10.0
    else:
        lr = init_lr / 100.0
    return max(lr, min_lr)


class S8Trainer(GraphStepper):
    def __init__(self, net, batch_size, img_dims, n_max=64, box_scales=BOX_SCALES, momentum=0.9, grad_clip=1.0,
                 cls_lambda=1.0, reg_lambda=1.0, init_lr=0.01, world=1, use_graph=True):
        self.net = net
        self.B = batch_size
        self.img = int(img_dims)
        self.C = net.C
        self.scales = tuple(float(v) for v in box_scales)
        assert len(self.scales) == net.ns
        self.momentum, self.clip = momentum, grad_clip
        self.cls_lambda, self.reg_lambda = cls_lambda, reg_lambda
        dev = net.device
        B = self.B
        self.S = self.img // 8
        self.P = self.S * self.S
        self.images = torch.zeros((B, self.img, self.img, 3), dtype=torch.float32, device=dev)
        self.boxes = torch.zeros((B, n_max, 5), dtype=torch.float32, device=dev)
        self.nbox = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.img_dim = torch.full((B, 2), float(self.img), dtype=torch.float32, device=dev)
        self.targets = torch.zeros((B, self.S, self.S, net.ns, 4 + self.C), dtype=torch.float32, device=dev)
        self.d_reg = torch.zeros((B, self.P, net.reg_ld), dtype=torch.bfloat16, device=dev)
        self.d_cls = torch.zeros((B, self.P, net.cls_ld), dtype=torch.bfloat16, device=dev)
        self.losses = torch.zeros((B, 2), dtype=torch.float32, device=dev)
        self.lr = torch.tensor([init_lr], dtype=torch.float32, device=dev)
        self.sumsq = torch.zeros(nn.SUMSQ_WS, dtype=torch.float64, device=dev)
        self._init_stepper(net, world, use_graph)

    skip_assign = False         # True: targets are loaded pre-formatted (train_step's `bboxes`)

    def _fwd_bwd(self, hook=None):
        if not self.skip_assign:
            ot.centernet_s8_assign(self.boxes, self.nbox, self.img_dim, (self.img, self.img), self.C, self.scales,
                                   out=self.targets)
        reg, cls = self.net.forward(self.images)
        self.outputs = (reg, cls)
        ot.centernet_s8_loss(reg, cls, self.targets.view(self.B, self.P, self.net.ns, -1), self.C, self.net.ns,
                             self.cls_lambda, self.reg_lambda, d_reg=self.d_reg, d_cls=self.d_cls, losses=self.losses)
        self.net.backward(self.d_reg, self.d_cls, hook=hook)

    def _update(self):
        st = self.net.store
        nn.sgd_clip_update(st.flat, st.grad, st.mom, self.lr, self.momentum, 1.0 / (self.B * self.world), self.clip,
                           ws=self.sumsq)
        self.net.pack()

    def set_lr(self, lr):
        self.lr.fill_(float(lr))

    def load_batch(self, images, boxes, nbox, raw_dims=None):
        """images [B,img,img,3] (resized to raw_dims and padded), boxes [B,n,5] normalised to the
        raw image (y, x, h, w, cls); raw_dims None = img_dims."""
        self.images.copy_(images, non_blocking=True)
        self.boxes.zero_()
        self.boxes[:, :boxes.shape[1]].copy_(boxes, non_blocking=True)
        self.nbox.copy_(nbox, non_blocking=True)
        self.img_dim.fill_(float(self.img if raw_dims is None else raw_dims))
