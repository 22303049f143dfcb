"""FCOS ResNet-50-FPN network (FCOS/fcos.py:6-110) on the cvlite kernels, explicit fwd/bwd.

Trunk (backbone, FPN, shared towers): fpn_det.FPNDetector.  The per-level heads
(`logits_output_l`, `reg_output_l`, fcos.py:85-101) are one segmented launch each (per-segment
weights) writing fp32 straight into the loss layout [B, P, ld] (P = sum S^2, level-major cells),
so the concat of fcos.py:104-108 disappears.
"""
import math

import torch

from . import _lib, ops_nn as nn
from .fpn_det import FPN_C, STRIDES, FPNDetector  # noqa: F401
from .layers import Conv

# the towers' final ReLU backward inside the heads' data-gradient epilogue (cvl_conv_igemm_relu_mask)
FUSE_TOP_RELU = not _lib.dispatch("no_top_relu_fuse")


class FCOSNet(FPNDetector):
    def __init__(self, num_classes, backbone_model="resnet50", device="cuda", seed=0, precision=None):
        """precision: "bf16" (production) / "fp32" (parity mode); None = CVL_PRECISION or bf16."""
        self._init_common(num_classes, backbone_model, device, seed, precision)
        self.cls_ld = self.cls_heads[0].cout_pad      # >= C, multiple of 32
        self.reg_ld = 8

    def _build_heads(self, st, num_classes):
        b_focal = math.log(0.01 / 0.99)
        # (packing the forward 64 wide, so that the halo 3x3 kernel takes the heads, measured no
        # faster in round 4: 63 + 70 us vs 2 x 65 us per step -- the halo kernel re-stages the
        # heads' 36 KiB of weights per channel block and tile)
        self.cls_heads = [Conv(st, "logits_output_%d" % (l + 1), 3, FPN_C, num_classes, bias_init=b_focal)
                          for l in range(5)]
        self.reg_heads = [Conv(st, "reg_output_%d" % (l + 1), 3, FPN_C, 5) for l in range(5)]

    def head_convs(self):
        return self.cls_heads + self.reg_heads

    def _heads_forward(self, towers, B, shapes, off, P):
        """Returns reg [B,P,8] fp32 (t,b,l,r,centerness), cls [B,P,ld] fp32."""
        dev = towers[0][0].device
        # the trainer's persistent output pair (FCOSTrainer: allocated zeroed once; the heads write
        # only their n_store columns, so the padding columns stay zero) -- else fresh zeroed buffers
        buf = getattr(self, "head_out", None)
        if buf is not None and tuple(buf[1].shape) == (B, P, self.cls_ld) and buf[1].device == dev:
            reg_out, cls_out = buf
        else:
            cls_out = torch.zeros((B, P, self.cls_ld), dtype=torch.float32, device=dev)
            reg_out = torch.zeros((B, P, self.reg_ld), dtype=torch.float32, device=dev)
        for heads, acts, out, ld in ((self.cls_heads, towers[0], cls_out, self.cls_ld),
                                     (self.reg_heads, towers[1], reg_out, self.reg_ld)):
            segs = [nn.seg(h, w, h, w, heads[l].wf, heads[l].bias_arg(), src_base=B * off[l], src_img=h * w,
                           dst_base=off[l], dst_img=P) for l, (h, w) in enumerate(shapes)]
            d = heads[0].fwd_desc(B, segs, ld_dst=ld, dst_f32=True, n_store=heads[0].cout)
            nn.conv_igemm(d, acts[-1], out)
        return reg_out, cls_out

    def _heads_backward(self, grads, towers, B, shapes, off, P):
        """grads = (d_reg, d_cls): bf16 [B, P, 32] (padding channels zero) from the fused loss."""
        d_reg, d_cls = grads
        dAs = []
        # the two towers' input gradients as the halves of one buffer: the trunk then runs each
        # tower layer's data gradient as one paired launch (FPNDetector.trunk_backward)
        a0 = towers[0][0]
        dA_pair = torch.empty((2,) + tuple(a0.shape), dtype=a0.dtype, device=a0.device)
        # the ten per-level head bias gradients (column sums of the loss gradients): one launch pair
        nn.bias_grad_multi([(dout, int(dout.shape[-1]), 0, heads[l].cout, off[l], P, h * w, B, heads[l].db, 0.0)
                            for heads, dout in ((self.cls_heads, d_cls), (self.reg_heads, d_reg))
                            for l, (h, w) in enumerate(shapes)])
        for heads, acts, dout in ((self.cls_heads, towers[0], d_cls), (self.reg_heads, towers[1], d_reg)):
            ld = int(dout.shape[-1])
            # heads: the five levels' weight gradients as one grouped launch (one group per level,
            # each with its own dw; small-N kernel conv_wgrad_sn), data grad for all levels in one launch
            d = heads[0].fwd_desc(B, [nn.seg(h, w, h, w, heads[l].wf, None, src_base=B * off[l], src_img=h * w,
                                             dst_base=off[l], dst_img=P) for l, (h, w) in enumerate(shapes)],
                                  ld_dst=ld, npad=heads[0].cout_pad)
            nn.conv_wgrad_grouped(d, acts[-1], dout, [heads[l].dw for l in range(len(shapes))])
            dA = dA_pair[len(dAs)]
            segs = [nn.seg(h, w, h, w, heads[l].wd, None, src_base=off[l], src_img=P, dst_base=B * off[l],
                           dst_img=h * w) for l, (h, w) in enumerate(shapes)]
            d = heads[0].dgrad_desc(B, segs, ld_dst=FPN_C)
            fuse = FUSE_TOP_RELU and dA.dtype == torch.bfloat16      # (fp32 parity mode: two launches)
            if fuse:                  # the towers' final ReLU backward in the data gradient's epilogue
                nn.conv_igemm_relu_mask(d, dout, dA, acts[-1])
            else:
                nn.conv_igemm(d, dout, dA)
            dAs.append(dA)
        self._top_relu_done = fuse
        return dAs
