"""RetinaNet training step and loop on MI355X -- mirrors RetinaNet/train_retinanet_coco.py:145-308.

`RetinaTrainer` runs the reference step semantics on the device, captured into HIP graphs:
* the reference draws 3*batch_size candidate images, skips those whose `format_data` finds no
  (box, anchor) match and trains on the first batch_size usable ones (Q27); here the targets of
  all candidates are assigned in one launch (cvl_retina_assign), cvl_select_first_nonzero picks
  the first batch_size candidates with matches (empty slots weight 0) and cvl_gather_rows moves
  their images / targets into the batch buffers -- no host round trip;
* loss = cls + reg summed over the 45 (level, anchor) terms (cvl_retina_loss, fwd+bwd fused);
* gradients summed over the images, / batch_size (even when fewer were usable), clipped by
  global norm, Keras SGD momentum 0.9 (`tf.optimizers.SGD(momentum=0.9)`, :345);
* lr = max(init_lr, min_lr) for step < 60000 and max(init_lr / 10, min_lr) for every step after
  (:164-171; the 80000 branch is unreachable in the reference) = the device schedule
  max(init * 0.1^floor(step / 60000), max(init / 10, min_lr)).
BN statistics are per image (the reference forwards one image at a time).
"""
import numpy as np
import torch

from . import dist
from .stepper import GraphStepper
from . import ops_nn as nn
from . import ops_targets as ot
from .retina_net import RetinaNetNet

BF16 = torch.bfloat16


class RetinaTrainer(GraphStepper):
    def __init__(self, net, anchors, batch_size, img_size, n_max=64, init_lr=0.01, min_lr=1e-5,
                 momentum=0.9, gradient_clip=1.0, candidates=3, world=1, use_graph=True, st_step=0):
        assert isinstance(net, RetinaNetNet)
        self.net, self.anchors = net, anchors
        self.B, self.S = batch_size, img_size
        self.nc = candidates * batch_size
        self.C, self.A = net.C, net.A
        self.world = world
        self.momentum, self.clip = momentum, gradient_clip
        # the floor max(init/10, min_lr) stops the decay after the first drop (:164-171)
        self.sched = (init_lr, max(init_lr / 10.0, min_lr), 0.1, 60000)
        dev = net.device
        B, S = self.B, self.S
        shapes, off, self.P = net.layout(B, S, S)
        self.level_cells = [h * w for h, w in shapes]
        T = self.A * self.P
        self.cand_images = torch.zeros((self.nc, S, S, 3), dtype=torch.float32, device=dev)
        self.cand_boxes = torch.zeros((self.nc, n_max, 5), dtype=torch.float32, device=dev)
        self.cand_nbox = torch.zeros((self.nc,), dtype=torch.int32, device=dev)
        self.cand_dim = torch.tensor([[float(S), float(S)]] * self.nc, dtype=torch.float32, device=dev)
        self.cand_targets = torch.zeros((self.nc, T, 4 + self.C), dtype=torch.float32, device=dev)
        self.cand_counts = torch.zeros((self.nc,), dtype=torch.int32, device=dev)
        self.sel = torch.zeros((B,), dtype=torch.int32, device=dev)
        self.img_w = torch.zeros((B,), dtype=torch.float32, device=dev)
        self.images = torch.zeros((B, S, S, 3), dtype=torch.float32, device=dev)
        self.targets = torch.zeros((B, T, 4 + self.C), dtype=torch.float32, device=dev)
        # padding channels of the head gradients must stay zero: written once, never touched
        self.d_reg = torch.zeros((B, self.P, net.reg_ld), dtype=net.store.act, device=dev)   # bf16 | fp32 parity
        self.d_cls = torch.zeros((B, self.P, net.cls_ld), dtype=net.store.act, device=dev)
        self.losses = torch.zeros((B, 2), dtype=torch.float32, device=dev)
        self.lr = torch.tensor([init_lr], dtype=torch.float32, device=dev)
        self.step_dev = torch.tensor([st_step], dtype=torch.int32, device=dev)
        self.sumsq = torch.zeros(nn.SUMSQ_WS, dtype=torch.float64, device=dev)
        self._init_stepper(net, world, use_graph)

    def _fwd_bwd(self, hook=None):
        self.anchors.format_data_batched(self.cand_boxes, self.cand_nbox, self.cand_dim, self.S,
                                         out=self.cand_targets, num_targets=self.cand_counts)
        nn.select_first_nonzero(self.cand_counts, self.B, self.sel, self.img_w)
        nn.gather_rows(self.cand_images, self.sel, self.images)
        nn.gather_rows(self.cand_targets, self.sel, self.targets)
        reg, cls = self.net.forward(self.images)
        self.outputs = (reg, cls)
        ot.retina_loss(reg, cls, self.targets, self.level_cells, self.A, self.C, img_weight=self.img_w,
                       d_reg=self.d_reg, d_cls=self.d_cls, losses=self.losses)
        self.net.backward(self.d_reg, self.d_cls, hook=hook)

    def _update(self):
        init_lr, min_lr, rate, dstep = self.sched
        nn.lr_schedule(self.step_dev, self.lr, init_lr, min_lr, rate, dstep)
        st = self.net.store
        nn.sgd_clip_update(st.flat, st.grad, st.mom, self.lr, self.momentum, 1.0 / (self.B * self.world),
                           self.clip, ws=self.sumsq)
        self.net.pack()

    def load_candidates(self, images, boxes, nbox):
        """Device-to-device copy of the 3*bs candidate images and their boxes."""
        self.cand_images.copy_(images, non_blocking=True)
        self.cand_boxes.zero_()
        self.cand_boxes[:, :boxes.shape[1]].copy_(boxes, non_blocking=True)
        self.cand_nbox.copy_(nbox, non_blocking=True)



def synthetic_coco_batch(n, S, n_classes=80, n_max=50, seed=1234, device="cuda"):
    """images U[-1,1) at S x S, 1+Poisson(6.3) boxes (<= n_max), log-uniform
    sides in [12, 0.94 S] px, class U{0..C-1}, normalised (yc, xc, h, w, cls); distinct areas."""
    rng = np.random.default_rng(seed)
    g = torch.Generator(device="cpu").manual_seed(seed)
    images = (torch.rand((n, S, S, 3), generator=g) * 2 - 1).to(device)
    boxes = np.zeros((n, n_max, 5), np.float32)
    nbox = np.zeros(n, np.int32)
    hi = 0.9375 * S
    for b in range(n):
        k_n = int(min(max(1 + rng.poisson(6.3), 1), n_max))
        areas, k = set(), 0
        while k < k_n:
            h = float(np.exp(rng.uniform(np.log(12.0), np.log(hi))))
            w = float(np.exp(rng.uniform(np.log(12.0), np.log(hi))))
            a = round(h * w, 3)
            if a in areas:
                continue
            areas.add(a)
            yc, xc = rng.uniform(h / 2, S - h / 2), rng.uniform(w / 2, S - w / 2)
            boxes[b, k] = [yc / S, xc / S, h / S, w / S, rng.integers(0, n_classes)]
            k += 1
        nbox[b] = k_n
    return images, torch.from_numpy(boxes).to(device), torch.from_numpy(nbox).to(device)


# -------------------------------------------------------------------------------------------------
# reference-shaped training loop (RetinaNet/train_retinanet_coco.py:145-308)
# -------------------------------------------------------------------------------------------------
def train(train_data, training_loss, model, batch_size, optimizer, ckpt, ck_manager, st_step, max_steps,
          init_lr=1e-3, min_lr=1e-5, decay_step=1000, decay_rate=0.99, img_dims=512, display_step=50,
          step_save=100, step_cool=1000, gradient_clip=1.0, save_loss_file="train_losses.csv"):
    """Same keywords as train_retinanet_coco.py:145-150.  `model` is a cvlite.retinanet.RetinaNet;
    `train_data` a list of pre-processed samples dict(image=[S,S,3] in [-1,1], bbox=[N,4] normalised
    (yc,xc,h,w), label=[N]) of one square size S (decode/resize are outside this tier).  Per step
    3*batch_size candidates are drawn without replacement; the device picks the first batch_size
    with anchor matches.  Prints the reference's progress lines.  `ckpt` / `ck_manager`:
    cvlite.checkpoint.Checkpoint / CheckpointManager (tf.train semantics), or a path prefix string
    and None (torch checkpoint with parameters, momentum and BN moving statistics)."""
    import os
    import time
    from . import checkpoint as ck
    n_data = len(train_data)
    S = int(train_data[0]["image"].shape[0])
    n_max = max(16, max(len(s["label"]) for s in train_data))
    trainer = RetinaTrainer(model.model, model, batch_size, S, n_max=n_max, init_lr=init_lr, min_lr=min_lr,
                            momentum=optimizer.momentum, gradient_clip=gradient_clip, st_step=st_step)
    dev = model.model.device
    start = time.time()
    batch_objs = total_loss = trend_loss = 0.0
    tot = np.zeros(2)
    nc = 3 * batch_size
    for step in range(st_step, max_steps):
        idx = np.random.choice(n_data, size=nc, replace=False)
        imgs = torch.from_numpy(np.stack([train_data[i]["image"] for i in idx]).astype(np.float32))
        bx = np.zeros((nc, n_max, 5), np.float32)
        nb = np.zeros(nc, np.int32)
        for k, i in enumerate(idx):
            s = train_data[i]
            n = len(s["label"])
            bx[k, :n, :4] = s["bbox"]
            bx[k, :n, 4] = s["label"]
            nb[k] = n
        trainer.load_candidates(imgs.to(dev), torch.from_numpy(bx).to(dev), torch.from_numpy(nb).to(dev))
        losses = trainer.step().detach().double().sum(0).cpu().numpy()
        if isinstance(ckpt, ck.Checkpoint):
            ckpt.step.assign_add(1)
        sel_w = trainer.img_w.cpu().numpy()
        used = trainer.cand_counts.cpu().numpy()[trainer.sel.cpu().numpy()] * sel_w
        batch_objs += float(used.sum()) / batch_size
        tot += losses / batch_size
        total_loss += losses.sum() / batch_size
        trend_loss += losses.sum() / batch_size
        if (step + 1) % display_step == 0:
            avg = tot / display_step
            training_loss.append((step + 1, total_loss / display_step, avg[0], avg[1]))
            elapsed = (time.time() - start) / 60.0
            start = time.time()
            print("Iteration:", str(step + 1))
            print("Learning Rate:", str(float(trainer.lr.item())))
            print("Average Objs:", str(batch_objs / display_step))
            print("Average Loss:", str(round(total_loss / display_step, 5)))
            print("Average Reg Loss:", str(round(avg[1], 5)))
            print("Average Cls Loss:", str(round(avg[0], 5)))
            batch_objs = total_loss = 0.0
            tot[:] = 0.0
            if (step + 1) % step_save == 0:
                with open(save_loss_file, "w") as f:
                    f.write("step,train_loss,cls_loss,reg_loss\n")
                    for row in training_loss:
                        f.write(",".join(str(v) for v in row) + "\n")
                if ck_manager is not None and hasattr(ck_manager, "save"):
                    print("Saved model to {}".format(ck_manager.save()))
                elif isinstance(ckpt, str) and ckpt:
                    st = ck.net_state(model.model)
                    st["step"] = step + 1
                    torch.save(st, ckpt + ".pt")
            if (step + 1) % step_cool != 0:
                print("Elapsed Time:", str(elapsed), "mins.")
                print("-" * 50)
        if (step + 1) % step_cool == 0:
            print("Trend Loss:", str(round(trend_loss / step_cool, 5)))
            trend_loss = 0.0
            if os.environ.get("CVL_COOLING") == "1":
                print("Cooling GPU for 2 minutes.")
                time.sleep(120)
    return None
