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
`image_augment` (:24-67: brightness / contrast / flip / 90- and 270-degree rotation of the padded
image and its target map) runs on the GPU over the whole batch (cvl_image_augment), the per-image
draws made on the host in the reference's np.random order (`draw_augment`).
Out of scope (data pipeline / visualisation): JPEG decode, obj_detect_results plotting.
"""
import time

import numpy as np
import torch

from . import _lib
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


NONE, BRIGHTNESS, CONTRAST, FLIP_LR, TRANSPOSE, ROT270 = range(6)


def draw_augment(p=0.5, rng=np.random, tf_rng=None):
    """The branch draws of one image_augment(img, bbox, p) call (train_hourglass_voc.py:25-56): the
    reference's np.random.uniform() calls in its order (apply if u >= p; u <= 0.333 brightness /
    contrast by a third draw; <= 0.667 flip left-right; else transpose, 270 degrees when a third
    draw is >= 0.5); the brightness delta ~ U[-0.25, 0.25) and contrast factor ~ U[0.75, 1.25) --
    tf.random draws in the reference -- from `tf_rng` (default: a generator of its own, so the
    numpy stream the loop samples batches from advances exactly as the reference's).
    Returns (op code, param) for cvl_image_augment."""
    tf_rng = _TF_RNG if tf_rng is None else tf_rng
    if rng.uniform() >= p:
        p_tmp = rng.uniform()
        if p_tmp <= 0.333:
            if rng.uniform() <= 0.50:
                return BRIGHTNESS, float(np.float32(tf_rng.uniform(-0.25, 0.25)))
            return CONTRAST, float(np.float32(tf_rng.uniform(0.75, 1.25)))
        if p_tmp <= 0.667:
            return FLIP_LR, 0.0
        return (ROT270 if rng.uniform() >= 0.50 else TRANSPOSE), 0.0
    return NONE, 0.0


_TF_RNG = np.random.RandomState(12345)


def augment_batch(images, targets, ops, params, out_images=None, out_targets=None):
    """cvl_image_augment: images [B,N,N,3] f32 (CUDA), targets [B,S,S,4,5+C] f32 or None, ops / params
    per image (host sequences or device tensors) -> (out_images, out_targets), new buffers unless
    given (they must not overlap the inputs).  Two launches on the current stream."""
    _lib.require_cuda(images)
    B, N = int(images.shape[0]), int(images.shape[1])
    assert images.dtype == torch.float32 and tuple(images.shape) == (B, N, N, 3) and images.is_contiguous()
    dev = images.device
    ops = torch.as_tensor(ops, dtype=torch.int32).to(dev, non_blocking=True)
    params = torch.as_tensor(params, dtype=torch.float32).to(dev, non_blocking=True)
    assert ops.shape == (B,) and params.shape == (B,)
    out_images = torch.empty_like(images) if out_images is None else out_images
    assert out_images.shape == images.shape and out_images.data_ptr() != images.data_ptr()
    S = T = 0
    if targets is not None:
        assert targets.dtype == torch.float32 and targets.is_contiguous() and targets.shape[0] == B
        S, T = int(targets.shape[1]), int(targets.shape[4])
        assert tuple(targets.shape) == (B, S, S, 4, T)
        out_targets = torch.empty_like(targets) if out_targets is None else out_targets
        assert out_targets.shape == targets.shape and out_targets.data_ptr() != targets.data_ptr()
    ws_n = int(_lib.load().cvl_image_augment_workspace_size(B, N))
    ws = torch.empty(ws_n, dtype=torch.uint8, device=dev)
    _lib.call("cvl_image_augment", _lib.ptr(images), _lib.ptr(out_images),
              _lib.ptr(targets) if targets is not None else None,
              _lib.ptr(out_targets) if targets is not None else None, _lib.ptr(ops), _lib.ptr(params),
              B, N, S, T, _lib.ptr(ws), ws_n, _lib.stream())
    return out_images, (out_targets if targets is not None else None)


def image_augment(img_in, img_bbox, p=0.5):
    """train_hourglass_voc.image_augment(img_in, img_bbox, p) for one CUDA image [N,N,3] and its
    target map [S,S,4,5+C]: returns the (possibly) transformed pair as new tensors."""
    op, prm = draw_augment(p)
    im, bb = augment_batch(img_in.unsqueeze(0).contiguous(), img_bbox.float().unsqueeze(0).contiguous(), [op], [prm])
    return im[0], bb[0]


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

    def load_batch(self, images, boxes, nbox, raw_dims, augment=None):
        """images [B,img,img,3] (already resized to raw_dims and padded), boxes [B,n,5] dataset corner
        rows + label, nbox [B]: copies into the static buffers and builds the targets.  augment =
        (ops, params) per image (draw_augment): the batch's image_augment runs on the GPU between
        the target build and the step (train_hourglass_voc.py:209-211)."""
        self.boxes.zero_()
        self.boxes[:, :boxes.shape[1]].copy_(boxes, non_blocking=True)
        self.nbox.copy_(nbox, non_blocking=True)
        if augment is None:
            self.images.copy_(images, non_blocking=True)
            ot.hourglass_v2_assign(self.boxes, self.nbox, raw_dims, self.img, self.C, out=self.targets)
            return
        if getattr(self, "_aug_in", None) is None:
            self._aug_in = (torch.empty_like(self.images), torch.empty_like(self.targets))
        img_in, tgt_in = self._aug_in
        img_in.copy_(images, non_blocking=True)
        ot.hourglass_v2_assign(self.boxes, self.nbox, raw_dims, self.img, self.C, out=tgt_in)
        augment_batch(img_in, tgt_in, augment[0], augment[1], out_images=self.images, out_targets=self.targets)

    def load_targets(self, images, targets):
        """Pre-formatted [B,S,S,4,5+C] maps (the reference train_step's `bboxes` argument)."""
        self.images.copy_(images, non_blocking=True)
        self.targets.copy_(targets, non_blocking=True)


def train(net, n_classes, sub_batch_sz, batch_size, train_data, training_loss, st_step, max_steps, optimizer=None,
          init_lr=1.0e-3, min_lr=1.0e-6, decay=0.75, display_step=100, base_rows=320, seed=None, use_graph=True,
          print_fn=print, augment=True):
    """train_hourglass_voc.train (:69-270) on pre-decoded samples: train_data[i] = {"image": float32
    [h, w, 3] in [0, 1], "objects": {"bbox": [n, 4] corner rows, "label": [n]}}.  Keeps the
    reference's sampling (np.random.choice without replacement, rnd_scale ~ U(0.6, 1.3), raw /
    img / pad dims), lr = max(decay ** epoch * init_lr, min_lr), per-step average cls / reg losses
    and the display cadence.  Images whose size differs from the step's raw_dims are resized on
    the host by nearest sampling (the reference's JPEG decode + tf.image.resize are outside this
    tier).  augment: image_augment per image as the reference (its np.random draws in the
    reference's order, after the batch's targets; augment=False skips it).  Returns training_loss."""
    if seed is not None:
        np.random.seed(seed)
    # the brightness / contrast amounts (tf.random draws in the reference, which tf.random.set_seed
    # controls): a generator owned by this call, seeded from `seed`, so two train() calls with one
    # seed draw the same amounts; the numpy branch-draw stream stays np.random, as the reference's
    tf_rng = np.random.RandomState(None if seed is None else (int(seed) * 1000003 + 12345) % (1 << 32))
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
        aug = None
        if augment:
            d = [draw_augment(0.5, tf_rng=tf_rng) for _ in range(batch_size)]
            aug = ([o for o, _ in d], [p for _, p in d])
        tr.load_batch(torch.from_numpy(imgs).to(net.device), torch.from_numpy(boxes).to(net.device),
                      torch.from_numpy(nbox).to(net.device), raw, augment=aug)
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
