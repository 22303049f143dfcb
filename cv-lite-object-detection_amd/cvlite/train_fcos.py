"""FCOS training step and loop on MI355X — mirrors FCOS/train_fcos.py.

`FCOSTrainer` is the MI355X-native step: target assignment, forward, fused loss, backward,
(RCCL gradient all-reduce), global-norm clip + Keras SGD and the bf16 weight re-pack, with the
whole device part captured once into two HIP graphs (fwd+bwd, update) and replayed, so a step
costs two graph launches instead of ~700 Python-side kernel launches.  Reference semantics kept
(FCOS/train_fcos.py:107-185): per-image BatchNorm statistics (the reference runs batch-1 forwards),
loss = cls + reg + cen summed over images (cls_lambda unused, Q11), g = sum_i grad_i / bs
(divide_no_nan), clip_by_global_norm(g, gradient_clip), SGD momentum v = m v - lr g, w += v,
lr = max(init * rate^floor(step / decay_step), min_lr) computed on the device.

`train(...)` keeps the reference's keyword surface and printing/checkpoint cadence for
pre-decoded samples (JPEG decode / resize / flip are outside this tier).
"""
import math
import os
import time

import numpy as np
import torch

from . import dist
from .stepper import GraphStepper
from . import ops_nn as nn
from . import ops_targets as ot

BF16 = torch.bfloat16


class SGD(object):
    """Stand-in for tf.optimizers.SGD(learning_rate, momentum) (train_fcos.py:284-285)."""

    def __init__(self, learning_rate=0.01, momentum=0.0):
        self.lr = float(learning_rate)
        self.momentum = float(momentum)


class FCOSTrainer(GraphStepper):
    def __init__(self, net, batch_size, image_hw, n_max=16, init_lr=5e-4, min_lr=1e-5, decay_step=1000,
                 decay_rate=0.9, momentum=0.9, gradient_clip=1.0, reg_type="l1", weight_decay=0.0,
                 world=1, use_graph=True, st_step=0, targets="fcos", center_only=True, optimizer=None,
                 max_decays=None):
        self.net = net
        # optimizer: None or SGD -> Keras SGD with `momentum` (train_fcos.py:284-285); an Adam
        # (cvlite.train_centernet.Adam, the tf.optimizers.Adam() stand-in) -> Keras Adam, what the
        # centre variant trains with (train_fcos_center_voc.py:327).  The scheduled learning rate
        # is written into the optimizer's device lr either way.  max_decays caps the decay
        # exponent (the centre loops' step schedule, train_fcos_center_voc.py:150-157: init_lr,
        # then init_lr / 10 from step 8000 on = decay_rate 0.1, decay_step 8000, max_decays 1).
        self.adam = optimizer.bind(net.store) if hasattr(optimizer, "bind") else None
        if optimizer is not None and self.adam is None:
            momentum = float(getattr(optimizer, "momentum", momentum))
        self.max_decays = max_decays
        # weight_decay * l2_params_reg (train_fcos.py:118-120, 160-164): the reference computes the
        # regulariser OUTSIDE the GradientTape, so it is added to each image's reported loss and
        # contributes nothing to the gradient; it is evaluated on the device at the start of the
        # step (before the update), as the reference does
        self.weight_decay = float(weight_decay)
        self.l2 = nn.L2Reg(net.store) if self.weight_decay > 0.0 else None
        self.B = batch_size
        self.H, self.W = image_hw
        self.C = net.C
        self.world = world
        self.momentum, self.clip = momentum, gradient_clip
        self.sched = (init_lr, min_lr, decay_rate, decay_step)
        self.reg_type = reg_type
        # targets="center": fcos_center.format_data (train_fcos_center_voc.py:184-187, center_only);
        # "center_v1": fcos_center_v1.format_data (train_fcos_center_v1_voc.py)
        if targets not in ("fcos", "center", "center_v1"):
            raise ValueError("targets must be 'fcos', 'center' or 'center_v1'")
        self.target_kind, self.center_only = targets, center_only
        # the centre networks (cvlite.fcos_center_net): focal centerness from the cls-tower head in
        # class column cen_col (train_fcos_center_voc.py:194-195), v1's sigmoid regression head
        centre = hasattr(net, "cen_heads")
        self.loss_flags = dict(cen_type="focal" if centre else "l1", cen_in_cls=centre,
                               reg_sigmoid=bool(getattr(net, "v1", False)))
        dev = net.device
        B, H, W = self.B, self.H, self.W
        _, _, self.P = net.layout(B, H, W)
        self.images = torch.zeros((B, H, W, 3), dtype=torch.float32, device=dev)
        self.boxes = torch.zeros((B, n_max, 5), dtype=torch.float32, device=dev)
        self.nbox = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.img_dim_pad = torch.tensor([[float(H), float(W)]] * B, dtype=torch.float32, device=dev)
        self.img_dim = self.img_dim_pad.clone()
        self._custom_dim = False
        self.targets = torch.zeros((B, self.P, 5 + self.C), dtype=torch.float32, device=dev)
        self.ntgt = torch.zeros((B, 5), dtype=torch.int32, device=dev)
        act = net.store.act                   # bf16, or fp32 in the parity mode
        self.d_reg = torch.zeros((B, self.P, 32), dtype=act, device=dev)
        self.d_cls = torch.zeros((B, self.P, net.cls_ld), dtype=act, device=dev)
        self.losses = torch.zeros((B, 3), dtype=torch.float32, device=dev)
        # the heads' fp32 outputs, zeroed once (FCOSNet writes only the used columns; see
        # FCOSNet._heads_forward) -- lent to the network for the step's forward only
        self._head_out = ((torch.zeros((B, self.P, net.reg_ld), dtype=torch.float32, device=dev),
                           torch.zeros((B, self.P, net.cls_ld), dtype=torch.float32, device=dev))
                          if hasattr(net, "reg_ld") and not centre else None)
        if self.adam is not None:
            self.lr = self.adam.lr_dev
            self.lr.fill_(init_lr)
        else:
            self.lr = torch.tensor([init_lr], dtype=torch.float32, device=dev)
        self.step_dev = torch.tensor([st_step], dtype=torch.int32, device=dev)
        self.sumsq = torch.zeros(nn.SUMSQ_WS, dtype=torch.float64, device=dev)
        self._init_stepper(net, world, use_graph)

    # ---- the two device phases -------------------------------------------------------------------
    def _fwd_bwd(self, hook=None):
        if self.l2 is not None:
            self.l2.run()
        if self.target_kind == "center":
            tg, _ = ot.fcos_center_assign(self.boxes, self.nbox, self.img_dim, (self.H, self.W), self.C,
                                          center_only=self.center_only, out=self.targets, num_targets=self.ntgt)
        elif self.target_kind == "center_v1":
            tg, _ = ot.fcos_center_v1_assign(self.boxes, self.nbox, self.img_dim, (self.H, self.W), self.C,
                                             out=self.targets, num_targets=self.ntgt)
        else:
            tg, _ = ot.fcos_assign(self.boxes, self.nbox, self.img_dim, (self.H, self.W), self.C,
                                   out=self.targets, num_targets=self.ntgt)
        self.net.head_out = self._head_out
        try:
            reg, cls = self.net.forward(self.images)
        finally:
            self.net.head_out = None
        self.outputs = (reg, cls)                 # head outputs of the last step (graph memory)
        ot.fcos_loss(reg, cls, tg, self.C, reg_type=self.reg_type, grad_scale=1.0, d_reg=self.d_reg,
                     d_cls=self.d_cls, losses=self.losses, **self.loss_flags)
        self.net.backward(self.d_reg, self.d_cls, hook=hook)

    def _update(self):
        init_lr, min_lr, rate, dstep = self.sched
        nn.lr_schedule(self.step_dev, self.lr, init_lr, min_lr, rate, dstep, max_decays=self.max_decays)
        st = self.net.store
        if self.adam is not None:
            self.adam.apply(st, 1.0 / (self.B * self.world), self.clip)
        else:
            nn.sgd_clip_update(st.flat, st.grad, st.mom, self.lr, self.momentum, 1.0 / (self.B * self.world),
                               self.clip, ws=self.sumsq)
        self.net.pack()

    def load_batch(self, images, boxes, nbox, img_dim=None):
        """Device-to-device copy of one batch into the static input buffers.  img_dim [B,2]: the
        unpadded resized [h, w] of each image (data_preprocess.resize_and_pad_image's new_shape,
        passed to format_data as img_dim while img_pad is the padded batch size,
        train_fcos.py:131-143); None = the padded size."""
        self.images.copy_(images, non_blocking=True)
        self.boxes.copy_(boxes, non_blocking=True)
        self.nbox.copy_(nbox, non_blocking=True)
        if img_dim is not None:
            self.img_dim.copy_(torch.as_tensor(img_dim, dtype=torch.float32).reshape(self.B, 2), non_blocking=True)
            self._custom_dim = True
        elif self._custom_dim:
            self.img_dim.copy_(self.img_dim_pad)
            self._custom_dim = False

    @property
    def l2_params_reg(self):
        """The device l2_params_reg of the last step (None without weight decay)."""
        return None if self.l2 is None else self.l2.out



class JitterFCOSTrainer(object):
    """The FCOS step over a batch whose images have different padded sizes (FCOS/train_fcos.py:
    128-176 preprocesses every image with its own jittered size and runs it as a batch-1 forward).
    Per-image BatchNorm makes a group of equal-size images one batch with the same math, so the
    batch is split into shape BUCKETS: one FCOSTrainer (its own HIP graphs) per (padded size,
    image count), created on first use and kept in an LRU of `max_buckets`; each bucket's
    forward + backward runs from its graphs, the parameter gradients are summed across buckets,
    then ONE clip + SGD update with 1 / batch_size (train_fcos.py:179-185)."""

    def __init__(self, net, batch_size, n_max=16, init_lr=5e-4, min_lr=1e-5, decay_step=1000, decay_rate=0.9,
                 momentum=0.9, gradient_clip=1.0, reg_type="l1", weight_decay=0.0, st_step=0, use_graph=True,
                 max_buckets=12, world=1, optimizer=None, max_decays=None):
        # world > 1: data-parallel (dist.py) -- each rank runs its own bs images through its buckets,
        # the summed gradient is all-reduced (one bucketed SUM over RCCL) before the shared update
        # with 1 / (world * bs); the buckets differ per rank, so there is no overlap with the backward
        self.net, self.B, self.n_max, self.world = net, batch_size, n_max, int(world)
        self.momentum, self.clip = momentum, gradient_clip
        self.adam = optimizer.bind(net.store) if hasattr(optimizer, "bind") else None    # Keras Adam
        self.max_decays = max_decays
        self.sched = (init_lr, min_lr, decay_rate, decay_step)
        self.reg_type, self.use_graph, self.max_buckets = reg_type, use_graph, max_buckets
        self.weight_decay = float(weight_decay)
        self.l2 = nn.L2Reg(net.store) if self.weight_decay > 0.0 else None
        dev = net.device
        self.buckets = {}
        self.acc = torch.zeros_like(net.store.grad)
        if self.adam is not None:
            self.lr = self.adam.lr_dev
            self.lr.fill_(init_lr)
        else:
            self.lr = torch.tensor([init_lr], dtype=torch.float32, device=dev)
        self.step_dev = torch.tensor([st_step], dtype=torch.int32, device=dev)
        self.sumsq = torch.zeros(nn.SUMSQ_WS, dtype=torch.float64, device=dev)
        self.losses = torch.zeros((batch_size, 3), dtype=torch.float32, device=dev)
        self.ntgt = torch.zeros((batch_size, 5), dtype=torch.int32, device=dev)

    def bucket(self, size, count):
        key = (int(size), int(count))
        tr = self.buckets.pop(key, None)
        if tr is None:
            if len(self.buckets) >= self.max_buckets:          # evict the least recently used
                self.buckets.pop(next(iter(self.buckets)))
            tr = FCOSTrainer(self.net, count, (size, size), n_max=self.n_max, reg_type=self.reg_type,
                             use_graph=self.use_graph)
        self.buckets[key] = tr
        return tr

    def step(self, images, boxes, nbox, img_dim):
        """images: list of bs device [S_i, S_i, 3] fp32 (preprocess_data outputs); boxes [bs, n_max, 5]
        (yc, xc, h, w, cls) normalised to img_dim; nbox [bs]; img_dim [bs, 2] = unpadded sizes.
        Returns the per-image (cls, reg, cen) losses [bs, 3] in the input order."""
        bs = len(images)
        assert bs == self.B
        dev = self.net.device
        boxes = torch.as_tensor(boxes, dtype=torch.float32, device=dev)
        nbox = torch.as_tensor(nbox, dtype=torch.int32, device=dev)
        img_dim = torch.as_tensor(img_dim, dtype=torch.float32, device=dev)
        if self.l2 is not None:
            self.l2.run()
        sizes = [int(t.shape[0]) for t in images]
        first = True
        for S in sorted(set(sizes)):
            idx = [i for i in range(bs) if sizes[i] == S]
            tr = self.bucket(S, len(idx))
            it = torch.tensor(idx, device=dev)
            bsel = boxes.index_select(0, it)
            nmax = tr.boxes.shape[1]
            if bsel.shape[1] < nmax:       # the batch's box arrays may be narrower than the trainer's
                bsel = torch.cat([bsel, bsel.new_zeros((bsel.shape[0], nmax - bsel.shape[1], 5))], 1)
            elif bsel.shape[1] > nmax:
                if int(nbox.max()) > nmax:
                    raise ValueError("an image has %d boxes, the trainer holds %d" % (int(nbox.max()), nmax))
                bsel = bsel[:, :nmax]
            tr.load_batch(torch.stack([images[i] for i in idx]), bsel.contiguous(), nbox.index_select(0, it),
                          img_dim=img_dim.index_select(0, it))
            tr.run_fwd_bwd()
            if first:
                self.acc.copy_(self.net.store.grad)
                first = False
            else:
                self.acc.add_(self.net.store.grad)
            self.losses.index_copy_(0, it, tr.losses)
            self.ntgt.index_copy_(0, it, tr.ntgt)
        st = self.net.store
        st.grad.copy_(self.acc)
        if self.world > 1:
            dist.allreduce_grads(st.grad)
        init_lr, min_lr, rate, dstep = self.sched
        nn.lr_schedule(self.step_dev, self.lr, init_lr, min_lr, rate, dstep, max_decays=self.max_decays)
        if self.adam is not None:
            self.adam.apply(st, 1.0 / (bs * self.world), self.clip)
        else:
            nn.sgd_clip_update(st.flat, st.grad, st.mom, self.lr, self.momentum, 1.0 / (bs * self.world), self.clip,
                               ws=self.sumsq)
        self.net.pack()
        return self.losses

    @property
    def l2_params_reg(self):
        return None if self.l2 is None else self.l2.out


def _raw_batch(train_data, idx, rng):
    """preprocess_data (data_preprocess.py:98-133) of each chosen raw sample: device images of their
    own padded sizes + boxes / counts / unpadded sizes for the bucketed step."""
    from .data_preprocess import preprocess_data
    imgs, boxes, dims = [], [], []
    for i in idx:
        img, bbox, cls, shp = preprocess_data(train_data[i], rng=rng)
        imgs.append(img)
        boxes.append(np.concatenate([bbox, cls.astype(np.float32)[:, None]], 1))
        dims.append(shp)
    n_max = max(16, max(len(b) for b in boxes))
    bx = np.zeros((len(idx), n_max, 5), np.float32)
    nb = np.zeros(len(idx), np.int32)
    for k, b in enumerate(boxes):
        bx[k, :len(b)] = b
        nb[k] = len(b)
    return imgs, bx, nb, np.stack(dims)


# -------------------------------------------------------------------------------------------------
# synthetic VOC-shaped batches
# -------------------------------------------------------------------------------------------------
def synthetic_batch(B, H, W, n_classes, n_max=16, seed=1234, device="cuda"):
    """Images U[-1,1) (post /127.5-1), 1+Poisson(1.4) boxes (<= n_max) with log-uniform sides in
    [12, 480] px, class U{0..C-1}, normalised (yc, xc, h, w, cls); distinct areas."""
    rng = np.random.default_rng(seed)
    g = torch.Generator(device="cpu").manual_seed(seed)
    images = (torch.rand((B, H, W, 3), generator=g) * 2 - 1).to(device)
    boxes = np.zeros((B, n_max, 5), np.float32)
    nbox = np.zeros(B, np.int32)
    for b in range(B):
        n = int(min(max(1 + rng.poisson(1.4), 1), n_max))
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


# -------------------------------------------------------------------------------------------------
# reference-shaped training loop (FCOS/train_fcos.py:87-251)
# -------------------------------------------------------------------------------------------------
def _batch_from_samples(train_data, idx, n_max):
    """Host batch from pre-processed samples dict(image=[Hp,Wp,3], bbox=[N,4] (yc,xc,h,w)
    normalised, label=[N], optional img_dim=[h,w] unpadded resized size)."""
    bs = len(idx)
    imgs = np.stack([np.asarray(train_data[i]["image"], np.float32) for i in idx])
    bx = np.zeros((bs, n_max, 5), np.float32)
    nb = np.zeros(bs, np.int32)
    dims = np.zeros((bs, 2), np.float32)
    for k, i in enumerate(idx):
        s = train_data[i]
        n = len(s["label"])
        bx[k, :n, :4] = s["bbox"]
        bx[k, :n, 4] = s["label"]
        nb[k] = n
        dims[k] = s.get("img_dim", imgs.shape[1:3])
    return imgs, bx, nb, dims


def train(train_data, training_loss, model, batch_size, optimizer, ckpt, ck_manager, st_step, max_steps,
          init_lr=1.0e-3, min_lr=1.0e-5, decay_step=1000, decay_rate=0.99, display_step=50, step_save=100,
          step_cool=1000, weight_decay=1.0e-4, gradient_clip=1.0, save_loss_file="train_losses.csv", world=None,
          max_decays=None):
    """Same keywords and defaults as FCOS/train_fcos.py:87-93.
    * `model`: what cvlite.fcos.build_model returns (or its FCOSNet).
    * `train_data`: either the reference's raw samples dict(image = a JPEG / PNG file name (decoded
      on the host, data_preprocess._parse_image) or a decoded [H,W,3] image, objects = {bbox,
      label}, l_jitter, u_jitter, min_side, max_side) -- each chosen image then runs
      data_preprocess.preprocess_data (flip + jittered resize + pad) on the GPU and the
      batch trains as shape buckets (JitterFCOSTrainer) -- or pre-processed samples
      dict(image=[Hp,Wp,3] in [-1,1], bbox=[N,4] normalised (yc,xc,h,w), label=[N], optional
      img_dim=[h,w]) of one padded size.
    * `ckpt` / `ck_manager`: cvlite.checkpoint.Checkpoint / CheckpointManager (tf.train.*
      semantics: ckpt.step += 1 per step, ck_manager.save() every step_save steps), or a path
      prefix string (torch checkpoint at <prefix>.pt) and None.
    * weight_decay > 0 adds weight_decay * l2_params_reg to every image's reported loss and not to
      the gradient, exactly as the reference (the regulariser is computed outside the tape).
    * world (cvlite extension; the reference is single-device): data-parallel over the initialised
      torch.distributed group (None = its world size, 1 without one).  Rank 0 draws the global
      sample of world * batch_size indices from np.random and broadcasts it, so the shards
      partition it whatever the ranks' seeds; each rank trains its own batch_size shard; gradients are all-reduced, the
      reported losses are averaged over all world * batch_size images, and only rank 0 prints and
      saves.
    * `optimizer`: the SGD stand-in (momentum read from it, train_fcos.py:284-285) or
      cvlite.train_centernet.Adam (Keras Adam, what train_fcos_center_voc.py:327 trains with);
      max_decays caps the decay exponent (the centre loops' step schedule, :150-157).  A string
      ckpt prefix saves the optimizer's slots too (SGD momentum or Adam m / v / iterations).
    The reference's thermal "Cooling GPU" sleep runs only with CVL_COOLING=1.  Returns None."""
    from . import checkpoint as ck
    import torch.distributed as tdist
    net = getattr(model, "net", model)
    n_data = len(train_data)
    raw = "objects" in train_data[0]
    dist_on = tdist.is_available() and tdist.is_initialized()
    if world is None:
        world = tdist.get_world_size() if dist_on else 1
    world = int(world)
    rank = tdist.get_rank() if (dist_on and world > 1) else 0
    if world > 1 and not (dist_on and tdist.get_world_size() == world):
        raise ValueError("train(world=%d) needs an initialised process group of that size" % world)
    if n_data < world * batch_size:
        raise ValueError("train_data holds %d samples, fewer than world * batch_size" % n_data)
    say = print if rank == 0 else (lambda *a, **k: None)
    momentum = float(getattr(optimizer, "momentum", 0.9))
    if raw:          # reference-format samples: per-image jittered sizes, shape-bucketed step
        n_max = max(16, max(len(s["objects"]["label"]) for s in train_data))
        trainer = JitterFCOSTrainer(net, batch_size, n_max=n_max, init_lr=init_lr, min_lr=min_lr,
                                    decay_step=decay_step, decay_rate=decay_rate, momentum=momentum,
                                    gradient_clip=gradient_clip, weight_decay=weight_decay, st_step=st_step,
                                    world=world, optimizer=optimizer, max_decays=max_decays)
        rng = np.random.default_rng()
    else:
        H, W = np.asarray(train_data[0]["image"]).shape[:2]
        n_max = max(16, max(len(s["label"]) for s in train_data))
        trainer = FCOSTrainer(net, batch_size, (H, W), n_max=n_max, init_lr=init_lr, min_lr=min_lr,
                              decay_step=decay_step, decay_rate=decay_rate, momentum=momentum,
                              gradient_clip=gradient_clip, weight_decay=weight_decay, st_step=st_step,
                              world=world, optimizer=optimizer, max_decays=max_decays)
    dev = net.device
    start = time.time()
    elapsed = 0.0
    batch_objs = total_loss = trend_loss = 0.0
    tot = np.zeros(3)
    for step in range(st_step, max_steps):
        idx = np.random.choice(n_data, size=world * batch_size, replace=False)   # train_fcos.py:112
        if world > 1:        # rank 0's draw for every rank: the shards partition one global sample
            t = torch.from_numpy(idx.astype(np.int64))
            t = t.to(dev) if tdist.get_backend() == "nccl" else t
            tdist.broadcast(t, 0)
            idx = t.cpu().numpy()
        idx = idx[rank * batch_size:(rank + 1) * batch_size]
        if raw:
            imgs, bx, nb, dims = _raw_batch(train_data, idx, rng)
            per_img = trainer.step(imgs, bx, nb, dims).detach().double()
        else:
            imgs, bx, nb, dims = _batch_from_samples(train_data, idx, n_max)
            trainer.load_batch(torch.from_numpy(imgs).to(dev), torch.from_numpy(bx).to(dev),
                               torch.from_numpy(nb).to(dev), img_dim=torch.from_numpy(dims).to(dev))
            per_img = trainer.step().detach().double()     # [bs, 3] (cls, reg, cen)
        ntgt = trainer.ntgt.sum(1)
        for k in np.nonzero(ntgt.cpu().numpy() == 0)[0]:
            say("No targets at index", str(idx[k]) + ".")
        if world > 1:        # report over the global batch: sums of every rank's images
            red = torch.cat([per_img.sum(0), ntgt.sum().double().view(1)])
            tdist.all_reduce(red)
            per_img = (red[:3] / world).view(1, 3).cpu().numpy()
            ntgt = np.array([float(red[3]) / world])
        else:
            per_img = per_img.cpu().numpy()
            ntgt = ntgt.cpu().numpy()
        wd_term = weight_decay * float(trainer.l2_params_reg.item()) if weight_decay > 0.0 else 0.0
        acc = per_img.sum() + batch_size * wd_term
        if isinstance(ckpt, ck.Checkpoint):
            ckpt.step.assign_add(1)
        batch_objs += float(ntgt.sum()) / batch_size
        tot += per_img.sum(0) / batch_size
        total_loss += acc / batch_size
        trend_loss += acc / batch_size
        if (step + 1) % display_step == 0:
            avg_loss = total_loss / display_step
            avg = tot / display_step
            avg_objs = batch_objs / display_step
            batch_objs = total_loss = 0.0
            tot[:] = 0.0
            elapsed = (time.time() - start) / 60.0
            start = time.time()
            say("Iteration:", str(step + 1))
            say("Learning Rate:", str(float(trainer.lr.item())))
            say("Average Objs:", str(avg_objs))
            say("Average Loss:", str(round(avg_loss, 5)))
            say("Average Reg Loss:", str(round(avg[1], 5)))
            say("Average Cls Loss:", str(round(avg[0], 5)))
            say("Average Cen Loss:", str(round(avg[2], 5)))
            if (step + 1) % step_save == 0:
                training_loss.append((step + 1, avg_loss))
                if rank == 0:
                    with open(save_loss_file, "w") as f:
                        f.write("step,train_loss\n")
                        for a, b in training_loss:
                            f.write("%d,%s\n" % (a, b))
                say("")
                if rank != 0:
                    pass
                elif ck_manager is not None and hasattr(ck_manager, "save"):
                    say("Saved model to {}".format(ck_manager.save()))
                elif isinstance(ckpt, str) and ckpt:
                    save_checkpoint(ckpt, net, trainer, step + 1)
                    say("Saved model to {}".format(ckpt + ".pt"))
            if (step + 1) % step_cool != 0:
                say("Elapsed Time:", str(elapsed), "mins.")
                say("-" * 50)
        if (step + 1) % step_cool == 0:
            say("Trend Loss:", str(round(trend_loss / step_cool, 5)))
            trend_loss = 0.0
            say("Elapsed Time:", str(elapsed), "mins.")
            if os.environ.get("CVL_COOLING") == "1":
                say("Cooling GPU for 2 minutes.")
                time.sleep(120)
            say("-" * 50)
    return None


def save_checkpoint(prefix, model, trainer, step):
    """{step, params, SGD momentum, BN running stats, parameter layout[, Adam m / v / iterations]}
    at <prefix>.pt."""
    from . import checkpoint as ck
    net = getattr(model, "net", model)
    st = ck.net_state(net)
    st["step"] = int(step)
    adam = getattr(trainer, "adam", None)
    if adam is not None:
        st["adam"] = {"m": adam.m.detach().cpu().clone(), "v": adam.v.detach().cpu().clone(),
                      "iterations": adam.iterations.detach().cpu().clone()}
    torch.save(st, prefix + ".pt")


def load_checkpoint(path, model, trainer=None):
    from . import checkpoint as ck
    net = getattr(model, "net", model)
    s = torch.load(path, weights_only=True)
    ck.load_net_state(net, s)
    if trainer is not None:
        trainer.step_dev.fill_(int(s["step"]))
        adam = getattr(trainer, "adam", None)
        if adam is not None and "adam" in s:
            adam.load_state({k: v.to(adam.m.device) for k, v in s["adam"].items()})
    return int(s["step"])
