"""CenterNet hourglass training step on MI355X — mirrors CenterNet/tf_centernet_hourglass.py
`train_step` (:507-564) with the optimizer the hourglass trainers use (tf.keras.optimizers.Adam(),
CenterNet/train_hourglass_voc.py:330).

`CenterNetTrainer` runs one whole step on the device: centroid targets (cvl_centernet_assign, the
reference's `format_data` :379-456 at the model's stride 4), forward with BatchNorm statistics per
sub-batch of `sub_batch_sz` images (one Keras training forward per sub-batch), the fused
model_loss forward + backward (2.5 cls + 1.0 reg), backward, (RCCL gradient all-reduce),
divide_no_nan(g, batch_size), clip_by_global_norm, Keras Adam, then the separable-conv fold and
bf16 re-pack — captured into two HIP graphs (fwd+bwd, update) and replayed.
"""
import numpy as np
import torch

from . import dist
from .stepper import GraphStepper
from . import ops_nn as nn
from . import ops_targets as ot


class Adam(object):
    """tf.keras.optimizers.Adam(learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-07):
    the moment buffers live on the device next to the flat parameter buffer; `iterations` is a
    device int32 (Keras optimizer.iterations)."""

    def __init__(self, learning_rate=0.001, beta_1=0.9, beta_2=0.999, epsilon=1e-7):
        self.lr = float(learning_rate)
        self.beta_1, self.beta_2, self.epsilon = float(beta_1), float(beta_2), float(epsilon)
        self.m = self.v = self.iterations = self.lr_dev = self.ws = None
        # slots restored from a checkpoint before the optimizer met its parameters (the reference
        # restores tf.train.Checkpoint before training starts, train_hourglass_voc.py:332-344):
        # applied by bind()
        self.pending_state = None

    def bind(self, store):
        if self.m is None:
            dev = store.flat.device
            self.m = torch.zeros_like(store.flat)
            self.v = torch.zeros_like(store.flat)
            self.iterations = torch.zeros(1, dtype=torch.int32, device=dev)
            self.lr_dev = torch.tensor([self.lr], dtype=torch.float32, device=dev)
            self.ws = torch.zeros(1, dtype=torch.float64, device=dev)
        if self.pending_state is not None:
            s, self.pending_state = self.pending_state, None
            if s["m"].numel() != self.m.numel():
                raise ValueError("restored Adam slots do not match the parameter layout")
            self.load_state(s)
        return self

    def load_state(self, s):
        self.m.copy_(s["m"])
        self.v.copy_(s["v"])
        self.iterations.copy_(s["iterations"])

    def apply(self, store, inv_bs, clip):
        nn.adam_clip_update(store.flat, store.grad, self.m, self.v, self.lr_dev, self.iterations, self.beta_1,
                            self.beta_2, self.epsilon, inv_bs, clip, ws=self.ws)


class CenterNetTrainer(GraphStepper):
    def __init__(self, net, batch_size, image_hw, sub_batch_sz=2, n_max=64, optimizer=None, cls_lambda=2.5,
                 reg_lambda=1.0, grad_clip=1.0, world=1, use_graph=True):
        self.net = net
        self.B = batch_size
        self.H, self.W = image_hw
        self.C = net.C
        self.group = max(1, min(int(sub_batch_sz), batch_size))
        self.world = world
        self.cls_lambda, self.reg_lambda, self.clip = cls_lambda, reg_lambda, grad_clip
        self.opt = (optimizer or Adam()).bind(net.store)
        dev = net.device
        B, H, W = self.B, self.H, self.W
        self.Ho, self.Wo = net.out_hw(H, W)
        self.stride = H // self.Ho
        self.P = self.Ho * self.Wo
        self.images = torch.zeros((B, H, W, 3), dtype=torch.float32, device=dev)
        self.boxes = torch.zeros((B, n_max, 5), dtype=torch.float32, device=dev)
        self.nbox = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.img_dim = torch.tensor([[float(H), float(W)]] * B, dtype=torch.float32, device=dev)
        self.targets = torch.zeros((B, self.Ho, self.Wo, 4 + self.C), dtype=torch.float32, device=dev)
        self.d_out = torch.zeros((B, self.Ho, self.Wo, net.cout_ld), dtype=torch.bfloat16, device=dev)
        self.losses = torch.zeros((B, 2), dtype=torch.float32, device=dev)
        self.assign = True
        self._init_stepper(net, world, use_graph)

    def _fwd_bwd(self, hook=None):
        if self.assign:
            ot.centernet_assign(self.boxes, self.nbox, self.img_dim, (self.H, self.W), self.C, stride=self.stride,
                                out=self.targets)
        out = self.net.forward(self.images, group=self.group)
        ot.centernet_loss(out.view(self.B, self.P, -1), self.targets.view(self.B, self.P, -1), self.C,
                          self.cls_lambda, self.reg_lambda, d_pred=self.d_out.view(self.B, self.P, -1),
                          losses=self.losses)
        self.out = out
        self.net.backward(self.d_out, hook=hook)

    def _update(self):
        self.opt.apply(self.net.store, 1.0 / (self.B * self.world), self.clip)
        self.net.pack()

    def load_batch(self, images, boxes, nbox):
        self.images.copy_(images, non_blocking=True)
        self.boxes[:, :boxes.shape[1]].copy_(boxes, non_blocking=True)
        self.nbox.copy_(nbox, non_blocking=True)

    def load_targets(self, images, targets):
        """Pre-formatted target maps (the reference train_step's `bboxes` argument)."""
        self.images.copy_(images, non_blocking=True)
        self.targets.copy_(targets, non_blocking=True)
        if self.assign:
            self.assign = False
            self.invalidate()                     # re-capture without the assign launch



def synthetic_batch(B, H, W, n_classes, n_max=64, seed=1234, device="cuda", mean_boxes=2.4):
    """VOC-shaped synthetic batch (SURVEY.md §8d generator): images U[-1,1), 1+Poisson boxes with
    log-uniform sides in [12, 480] px and distinct areas; normalised (yc, xc, h, w, cls)."""
    rng = np.random.default_rng(seed)
    g = torch.Generator(device="cpu").manual_seed(seed)
    images = (torch.rand((B, H, W, 3), generator=g) * 2 - 1).to(device)
    boxes = np.zeros((B, n_max, 5), np.float32)
    nbox = np.zeros(B, np.int32)
    for b in range(B):
        n = int(min(max(1 + rng.poisson(mean_boxes - 1.0), 1), n_max))
        areas = set()
        k = 0
        while k < n:
            h = float(np.exp(rng.uniform(np.log(12.0), np.log(min(480.0, H)))))
            w = float(np.exp(rng.uniform(np.log(12.0), np.log(min(480.0, W)))))
            a = round(h * w, 3)
            if a in areas:
                continue
            areas.add(a)
            yc, xc = rng.uniform(h / 2, H - h / 2), rng.uniform(w / 2, W - w / 2)
            boxes[b, k] = [yc / H, xc / W, h / H, w / W, rng.integers(0, n_classes)]
            k += 1
        nbox[b] = n
    return images, torch.from_numpy(boxes).to(device), torch.from_numpy(nbox).to(device)
