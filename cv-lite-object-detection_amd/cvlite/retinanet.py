"""Drop-in mirror of RetinaNet/retinanet_module.py's `RetinaNet` target interface on MI355X.

`RetinaNet(n_classes, id_2_label, aspect_ratios, anchor_scales, anchor_sizes, backbone_model)`
keeps the reference attributes (`anchor_sizes`, `aspect_ratios`, `anchor_scales`, `strides`,
`n_anchors`, `box_areas`, `anchor_boxes`) and methods `get_anchors`, `format_data` (device kernel
cvl_retina_assign: anchor generation + IoU matching per output cell), `focal_loss`,
`smooth_l1_loss`, and the inference decode `prediction_to_corners`, `cpu_nms`,
`image_detections` (kernels cvl_retina_corners / cvl_retina_decode / cvl_retina_nms, batched
form `decode_detections`).  The anchor dimensions are the 45 numbers of retinanet_module.py:205-219,
computed once on the host with the reference's fp32 operation order.
"""
import ctypes

import numpy as np
import torch

from . import _lib
from . import ops_targets as ot

f32 = np.float32


class RetinaNet(object):
    def __init__(self, n_classes, id_2_label, aspect_ratios=None, anchor_scales=None, anchor_sizes=None,
                 backbone_model="resnet50", **kwargs):
        if anchor_sizes is None:
            self.anchor_sizes = [32.0, 64.0, 128.0, 256.0, 512.0]
        elif len(anchor_sizes) != 5:
            raise ValueError("anchor_sizes must be of dimension 5.")
        else:
            self.anchor_sizes = anchor_sizes
        self.aspect_ratios = [0.5, 1.0, 2.0] if aspect_ratios is None else aspect_ratios
        if anchor_scales is None:
            self.anchor_scales = [2 ** x for x in [0, 1 / 3, 2 / 3]]
        elif len(anchor_scales) != 3:
            raise ValueError("anchor_scales must be of dimension 3.")
        else:
            self.anchor_scales = anchor_scales
        self.n_class = n_classes
        self.strides = [8, 16, 32, 64, 128]
        self.n_anchors = len(self.anchor_scales) * len(self.aspect_ratios)
        self.box_areas = list(sorted([x ** 2 for x in self.anchor_sizes]))
        self.id_2_label = id_2_label
        self.backbone_model = backbone_model
        # retinanet_module.py:205-216: h = sqrt(area / ratio), w = area / h (fp32 tensor ops),
        # scale * (h, w) (fp32); ratio outer loop, scale inner loop (Q22)
        boxes = []
        for area in self.box_areas:
            lev = []
            for ratio in self.aspect_ratios:
                h = np.sqrt(f32(area / ratio))
                w = f32(f32(area) / h)
                for sc in self.anchor_scales:
                    lev.append(np.array([f32(f32(sc) * h), f32(f32(sc) * w)], dtype=f32))
            boxes.append(lev)
        self.anchor_boxes = boxes
        self._dims_dev = None
        self._model = None

    @property
    def model(self):
        """retinanet_module.py:199-200 `self.model = build_model(...)`: the MI355X network
        (built on first use, so target-only users need no weights)."""
        if self._model is None:
            from .retina_net import RetinaNetNet
            _lib.require_cuda()
            self._model = RetinaNetNet(self.n_class, n_anchors=self.n_anchors, backbone_model=self.backbone_model)
        return self._model

    def train_loss(self, x_image, x_label, img_weight=None):
        """retinanet_module.py:403-426: forward (training-mode BN, per-image statistics) and
        (cls, reg) summed over levels, anchors and images.  x_image [B,H,W,3] (square);
        x_label: the device targets [B, A*P, 4+C] of format_data_batched, or (B = 1) the nested
        [5][A] list format_data returns.  Returns float32 scalars; gradients come from the
        trainer (cvlite.train_retinanet.RetinaTrainer), which runs the same fused loss."""
        net = self.model
        x = torch.as_tensor(x_image, dtype=torch.float32, device="cuda")
        if x.dim() == 3:
            x = x.unsqueeze(0)
        B, H, W = int(x.shape[0]), int(x.shape[1]), int(x.shape[2])
        if isinstance(x_label, (list, tuple)):
            flat = [torch.as_tensor(np.asarray(m, np.float32)).reshape(-1, 4 + self.n_class)
                    for lev in x_label for m in lev]
            x_label = torch.cat(flat, 0).unsqueeze(0).cuda()
        shapes, _, _ = net.layout(B, H, W)
        reg, cls = net.forward(x.contiguous())
        losses = ot.retina_loss(reg, cls, x_label.contiguous(), [h * w for h, w in shapes], self.n_anchors,
                                self.n_class, img_weight=img_weight)
        s = losses.sum(0)
        return s[0], s[1]

    def anchor_dims_device(self):
        if self._dims_dev is None:
            _lib.require_cuda()
            self._dims_dev = torch.tensor(np.array(self.anchor_boxes, dtype=f32), device="cuda")
        return self._dims_dev

    def get_anchors(self, cnn_shape, level):
        """retinanet_module.py:221-246 (host helper): 9 arrays [S0, S1, 4] = (col, row, h, w)."""
        if level >= 5 or level < 0:
            raise ValueError("level has to be between 0 and 4.")
        gx, gy = np.meshgrid(np.arange(cnn_shape[1], dtype=f32), np.arange(cnn_shape[0], dtype=f32))
        base = np.stack([gx, gy, np.ones_like(gx), np.ones_like(gx)], -1).astype(np.float64)
        return [base * np.array([1, 1, d[0], d[1]], np.float64).reshape(1, 1, 4) for d in self.anchor_boxes[level]]

    def format_data_batched(self, boxes, nbox, img_dim, pad, iou_thresh=0.50, out=None, num_targets=None):
        """Device form: boxes [B,Nmax,5], nbox [B], img_dim [B,2] -> targets [B, P, 4+C], counts [B]."""
        return ot.retina_assign(boxes, nbox, img_dim, pad, self.anchor_dims_device(), self.n_class,
                                iou_thresh=iou_thresh, strides=self.strides, out=out, num_targets=num_targets)

    def format_data(self, gt_labels, img_dim, iou_thresh=0.50, img_pad=None):
        """retinanet_module.py:251-365 -> (nested [5][A] float32 [S,S,4+C] maps, num_targets)."""
        if img_pad is None:
            img_pad = img_dim
        pad = int(float(np.asarray(img_pad, dtype=np.float32)[0]))
        if int(float(np.asarray(img_pad, dtype=np.float32)[1])) != pad:
            raise ValueError("the reference's transposed anchor grid is consistent only for square maps")
        gt = np.asarray(gt_labels, dtype=f32).reshape(-1, 5)
        n = len(gt)
        boxes = np.zeros((1, max(n, 1), 5), f32)
        boxes[0, :n] = gt
        dev = "cuda"
        tg, nt = self.format_data_batched(torch.tensor(boxes, device=dev), torch.tensor([n], dtype=torch.int32, device=dev),
                                          torch.tensor(np.asarray(img_dim, f32).reshape(1, 2), device=dev), pad,
                                          iou_thresh)
        tg = tg[0].cpu().numpy()
        outs, o = [], 0
        for s in self.strides:
            S = pad // s
            lev = []
            for _ in range(self.n_anchors):
                lev.append(tg[o:o + S * S].reshape(S, S, 4 + self.n_class))
                o += S * S
            outs.append(lev)
        return outs, int(nt[0].item())

    def focal_loss(self, labels, logits, alpha=0.25, gamma=2.0):
        from .fcos import focal_loss
        return focal_loss(labels, logits, alpha, gamma)

    def smooth_l1_loss(self, xy_true, xy_pred, mask=1.0, delta=1.0):
        from .fcos import smooth_l1_loss
        return smooth_l1_loss(xy_true, xy_pred, mask, delta)

    # ---- inference decode (retinanet_module.py:428-529) -----------------------------------------
    def prediction_to_corners(self, xy_pred, anchor_dim, stride):
        """retinanet_module.py:428-451 -> float64 [S0,S1,4] (y1, x1, y2, x2) (cvl_retina_corners)."""
        _lib.require_cuda()
        xy = torch.as_tensor(np.asarray(xy_pred, f32) if not torch.is_tensor(xy_pred) else xy_pred,
                             dtype=torch.float32).cuda().contiguous()
        H, W, ld = int(xy.shape[0]), int(xy.shape[1]), int(xy.shape[2])
        out = torch.empty((H, W, 4), dtype=torch.float32, device="cuda")
        _lib.call("cvl_retina_corners", _lib.ptr(xy), ld, H, W, float(f32(anchor_dim[0])), float(f32(anchor_dim[1])),
                  int(stride), _lib.ptr(out), _lib.stream())
        return out.cpu().numpy().astype(np.float64)

    def cpu_nms(self, dets, base_thr):
        """retinanet_module.py:453-481 -> int64 indices of the kept rows in selection order
        (cvl_retina_nms; fp32 arithmetic, the dtype image_detections feeds it)."""
        _lib.require_cuda()
        d = torch.as_tensor(np.asarray(dets, f32) if not torch.is_tensor(dets) else dets,
                            dtype=torch.float32).cuda().contiguous().reshape(-1, int(np.shape(dets)[-1]))
        n = int(d.shape[0])
        if n == 0:
            return np.array([])
        if d.shape[1] != 6:
            d6 = torch.zeros((n, 6), dtype=torch.float32, device="cuda")
            d6[:, :5] = d[:, :5]
            d = d6
        cnt = torch.tensor([n], dtype=torch.int32, device="cuda")
        keep, nk = self._nms(d, n, cnt, 1, n, base_thr)
        return keep[0, :int(nk[0])].cpu().numpy().astype(np.int64)

    def _nms(self, dets, rows_per_img, count, B, n_cap, thr):
        keep = torch.empty((B, n_cap), dtype=torch.int32, device="cuda")
        nk = torch.empty(B, dtype=torch.int32, device="cuda")
        ws = torch.empty(max(1, _lib.load().cvl_retina_nms_workspace_size(B, n_cap)), dtype=torch.uint8, device="cuda")
        _lib.call("cvl_retina_nms", _lib.ptr(dets), rows_per_img, _lib.ptr(count), B, n_cap, float(thr),
                  _lib.ptr(keep), _lib.ptr(nk), _lib.ptr(ws), _lib.stream())
        return keep, nk

    def decode_detections(self, reg, cls, shapes, iou_thresh=0.5, cls_thresh=0.05, nms_cap=None):
        """Batched device decode of the fused head outputs (reg [B,P,ld_reg], cls [B,P,ld_cls]
        fp32, level shapes [(h, w)] x 5): cvl_retina_decode (corners, sigmoid max/argmax,
        threshold, ordered compaction) then cvl_retina_nms chained on the device counts.
        Returns a list of B fp32 [k,6] arrays (y1, x1, y2, x2, score, class), as
        image_detections.  nms_cap bounds the rows NMS considers (default: all)."""
        _lib.require_cuda(reg, cls)
        B, ld_reg, ld_cls = int(reg.shape[0]), int(reg.shape[-1]), int(cls.shape[-1])
        A, C = self.n_anchors, self.n_class
        hw_arr = (ctypes.c_int32 * 10)(*[int(v) for hwl in shapes for v in hwl])
        st_arr = (ctypes.c_int32 * 5)(*self.strides)
        hw, st = ctypes.cast(hw_arr, ctypes.c_void_p), ctypes.cast(st_arr, ctypes.c_void_p)
        R = A * sum(h * w for h, w in shapes)
        dets = torch.empty((B, R, 6), dtype=torch.float32, device="cuda")
        cnt = torch.empty(B, dtype=torch.int32, device="cuda")
        wsb = _lib.load().cvl_retina_decode_workspace_size(B, hw, A)
        ws = torch.empty(wsb, dtype=torch.uint8, device="cuda")
        _lib.call("cvl_retina_decode", _lib.ptr(reg), ld_reg, _lib.ptr(cls), ld_cls, B, hw, st,
                  _lib.ptr(self.anchor_dims_device()), A, C, float(f32(cls_thresh)), _lib.ptr(dets), _lib.ptr(cnt),
                  _lib.ptr(ws), wsb, _lib.stream())
        cap = R if nms_cap is None else min(R, int(nms_cap))
        keep, nk = self._nms(dets, R, cnt, B, cap, iou_thresh)
        cnt_h, nk_h, keep_h = cnt.cpu().numpy(), nk.cpu().numpy(), keep.cpu()
        out = []
        for b in range(B):
            n = int(cnt_h[b])
            if n == 0 or int(nk_h[b]) == 0:
                out.append(dets[b, :n].cpu().numpy())
            else:
                out.append(dets[b][keep_h[b, :int(nk_h[b])].long().cuda()].cpu().numpy())
        return out

    def image_detections(self, image, iou_thresh=0.5, cls_thresh=0.05):
        """retinanet_module.py:483-529: inference forward (BN running statistics), decode, NMS ->
        fp32 [k,6] (y1, x1, y2, x2, score, class) for image [1,H,W,3] (or [H,W,3])."""
        net = self.model
        x = torch.as_tensor(image, dtype=torch.float32, device="cuda")
        if x.dim() == 3:
            x = x.unsqueeze(0)
        B, H, W = int(x.shape[0]), int(x.shape[1]), int(x.shape[2])
        shapes, _, _ = net.layout(B, H, W)
        reg, cls = net.forward(x.contiguous(), train=False)
        return self.decode_detections(reg, cls, shapes, iou_thresh, cls_thresh)[0]
