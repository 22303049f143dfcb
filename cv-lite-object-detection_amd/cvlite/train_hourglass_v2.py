"""CenterNet v2 training on MI355X — mirrors CenterNet/train_hourglass_voc.py (the loop, its inline
target builder :96-160 and the jittered batch size :99-106) over tf_hourglass_net.train_step
(:415-447) with tf.keras.optimizers.Adam() (:330).

`HourglassV2Trainer` owns one image size (the reference jitters img_dims over multiples of 64 per
step: one trainer / captured graph per size, `train` keeps a dict of them).  A step: the batch's
targets (cvl_hourglass_v2_assign, launched when the batch is loaded: raw_dims changes every step
and is a kernel argument), then the captured graph — forward with BN statistics per sub-batch of
`sub_batch_sz` images, the fused model_loss forward + backward (cls_lambda 2.5, reg_lambda 1.0),
backward, (RCCL all-reduce), divide_no_nan(g, batch_size), clip_by_global_norm(1.0), Keras Adam,
separable-conv fold and bf16 re-pack.
Out of scope (data pipeline / visualisation): JPEG decode, image_augment's
brightness / contrast / flip / transpose, obj_detect_results plotting.
"""
import time

import numpy as np
import torch

from . import ops_targets as ot
from .stepper import GraphStepper
from .train_centernet import Adam


def jitter_dims(rnd_scale, base=320):
    """train_hourglass_voc.py:99-105: raw_dims = int(rnd * 320); img_dims = raw_dims rounded up to
    a multiple of 64 (the reference's own formula); returns (raw_dims, img_dims, pad_dims)."""
    raw = int(rnd_scale * base)
    if raw % 64 == 0:
        img = int(rnd_scale * base / 64) * 64
    else:
        img = (int(rnd_scale * base / 64) + 1) * 64
    return raw, img, int((img - raw) / 2.0)


class HourglassV2Trainer(GraphStepper):
    def __init__(self, net, batch_size, img_dims, sub_batch_sz=2, n_max=64, optimizer=None, cls_lambda=2.5,
                 reg_lambda=1.0, grad_clip=1.0, loss_type="focal", world=1, use_graph=True):
        self.net = net
        self.B = batch_size
        self.img = int(img_dims)
        self.C = net.C
        self.group = max(1, min(int(sub_batch_sz), batch_size))
        self.cls_lambda, self.reg_lambda, self.clip = cls_lambda, reg_lambda, grad_clip
        self.loss_type = loss_type
        self.opt = (optimizer or Adam()).bind(net.store)
        dev = net.device
        B = self.B
        self.S = self.img // 8
        self.P = self.S * self.S
        self.images = torch.zeros((B, self.img, self.img, 3), dtype=torch.float32, device=dev)
        self.boxes = torch.zeros((B, n_max, 5), dtype=torch.float32, device=dev)
        self.nbox = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.targets = torch.zeros((B, self.S, self.S, 4, 5 + self.C), dtype=torch.float32, device=dev)
        self.d_out = torch.zeros((B, self.S, self.S, net.cout_ld), dtype=torch.bfloat16, device=dev)
        self.losses = torch.zeros((B, 2), dtype=torch.float32, device=dev)
        self._init_stepper(net, world, use_graph)

    def _fwd_bwd(self, hook=None):
        out = self.net.forward(self.images, group=self.group)
        ot.hourglass_v2_loss(out.view(self.B, self.P, -1), self.targets.view(self.B, self.P, 4, -1), self.C,
                             self.loss_type, self.cls_lambda, self.reg_lambda,
                             d_pred=self.d_out.view(self.B, self.P, -1), losses=self.losses)
        self.out = out
        self.net.backward(self.d_out, hook=hook)

    def _update(self):
        self.opt.apply(self.net.store, 1.0 / (self.B * self.world), self.clip)
        self.net.pack()

    def set_lr(self, lr):
        """optimizer.lr.assign(learning_rate) (tf_hourglass_net.train_step :418)."""
        self.opt.lr_dev.fill_(float(lr))

    def load_batch(self, images, boxes, nbox, raw_dims):
        """images [B,img,img,3] (already resized to raw_dims and padded), boxes [B,n,5] dataset corner
        rows + label, nbox [B]: copies into the static buffers and builds the targets."""
        self.images.copy_(images, non_blocking=True)
        self.boxes.zero_()
        self.boxes[:, :boxes.shape[1]].copy_(boxes, non_blocking=True)
        self.nbox.copy_(nbox, non_blocking=True)
        ot.hourglass_v2_assign(self.boxes, self.nbox, raw_dims, self.img, self.C, out=self.targets)

    def load_targets(self, images, targets):
        """Pre-formatted [B,S,S,4,5+C] maps (the reference train_step's `bboxes` argument)."""
        self.images.copy_(images, non_blocking=True)
        self.targets.copy_(targets, non_blocking=True)


def train(net, n_classes, sub_batch_sz, batch_size, train_data, training_loss, st_step, max_steps, optimizer=None,
          init_lr=1.0e-3, min_lr=1.0e-6, decay=0.75, display_step=100, base_rows=320, seed=None, use_graph=True,
          print_fn=print):
    """train_hourglass_voc.train (:69-270) on pre-decoded samples: train_data[i] = {"image": float32
    [h, w, 3] in [0, 1], "objects": {"bbox": [n, 4] corner rows, "label": [n]}}.  Keeps the
    reference's sampling (np.random.choice without replacement, rnd_scale ~ U(0.6, 1.3), raw /
    img / pad dims), lr = max(decay ** epoch * init_lr, min_lr), per-step average cls / reg losses
    and the display cadence.  Images whose size differs from the step's raw_dims are resized on
    the host by nearest sampling (the reference's JPEG decode + tf.image.resize are outside this
    tier).  Returns training_loss."""
    if seed is not None:
        np.random.seed(seed)
    n_data = len(train_data)
    opt = (optimizer or Adam()).bind(net.store)
    trainers = {}
    tot_cls = tot_reg = 0.0
    t0 = time.time()
    for step in range(st_step, max_steps):
        sample = np.random.choice(n_data, size=batch_size, replace=False)
        raw, img, pad = jitter_dims(np.random.uniform(low=0.6, high=1.3), base_rows)
        tr = trainers.get(img)
        if tr is None:
            n_max = max(max(len(d["objects"]["label"]) for d in train_data), 1)
            tr = trainers[img] = HourglassV2Trainer(net, batch_size, img, sub_batch_sz, n_max=n_max, optimizer=opt,
                                                    use_graph=use_graph)
        imgs = np.zeros((batch_size, img, img, 3), np.float32)
        boxes = np.zeros((batch_size, tr.boxes.shape[1], 5), np.float32)
        nbox = np.zeros(batch_size, np.int32)
        for j, k in enumerate(sample):
            d = train_data[k]
            im = np.asarray(d["image"], np.float32)
            if im.shape[0] != raw or im.shape[1] != raw:
                yi = (np.arange(raw) * im.shape[0] // raw).clip(0, im.shape[0] - 1)
                xi = (np.arange(raw) * im.shape[1] // raw).clip(0, im.shape[1] - 1)
                im = im[yi][:, xi]
            imgs[j, pad:pad + raw, pad:pad + raw] = im
            o = d["objects"]
            n = len(o["label"])
            boxes[j, :n, :4] = np.asarray(o["bbox"], np.float32)
            boxes[j, :n, 4] = np.asarray(o["label"])
            nbox[j] = n
        tr.load_batch(torch.from_numpy(imgs).to(net.device), torch.from_numpy(boxes).to(net.device),
                      torch.from_numpy(nbox).to(net.device), raw)
        epoch = int(step * batch_size / n_data)
        tr.set_lr(max(decay ** epoch * init_lr, min_lr))
        losses = tr.step().double().sum(0).cpu().numpy() / batch_size
        tot_cls += float(losses[0])
        tot_reg += float(losses[1])
        if (step + 1) % display_step == 0:
            training_loss.append((step + 1, tot_cls / display_step, tot_reg / display_step))
            print_fn("Step", str(step + 1), "Summary:")
            print_fn("Learning Rate:", str(float(opt.lr_dev)))
            print_fn("Average Epoch Cls. Loss:", str(tot_cls / display_step) + ".")
            print_fn("Average Epoch Reg. Loss:", str(tot_reg / display_step) + ".")
            print_fn("Elapsed time:", str((time.time() - t0) / 60.0), "mins.")
            tot_cls = tot_reg = 0.0
            t0 = time.time()
    return training_loss
