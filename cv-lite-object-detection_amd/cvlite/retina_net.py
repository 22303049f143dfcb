"""RetinaNet ResNet-50-FPN network (RetinaNet/retinanet_module.py:8-159) on the cvlite kernels.

Trunk (backbone, FPN, shared towers): fpn_det.FPNDetector -- the reference's FPN/tower code is the
same as FCOS's.  Heads: the reference builds a separate 3x3 conv per (level, anchor) --
`cls_output_{l}_anchor_{a}` (256 -> C, bias log(0.01/0.99)) and `reg_output_{l}_anchor_{a}`
(256 -> 4), 90 convs (Q28).  The 9 anchor convs of a level read the same tower output, so here
they are ONE conv per level with the anchors' output channels side by side (cls: 9C, reg: 36;
kernel [3,3,256,9C] = the 9 Keras kernels concatenated on the output axis, each initialised as
its own glorot-uniform conv), and the five levels are one segmented launch.  Outputs are written
fp32 into [B, P, ld] (P = sum S^2 level-major cells; anchor a at channels aC.. / 4a..), which
cvl_retina_loss reads directly; `outputs_nested` restores the reference's [5][9] list of
[B,S,S,4+C] maps.
"""
import math

import torch

from . import ops_nn as nn
from .fpn_det import FPN_C, STRIDES, FPNDetector  # noqa: F401
from .layers import Conv


class RetinaNetNet(FPNDetector):
    @staticmethod
    def backbone_kind(name):
        """RetinaNet/retinanet_module.py:30-71: ResNet50 / 101 / 152, ResNeXt50 / 101 (third-party
        classification_models, not built), every other name MobileNetV2."""
        n = name.lower()
        if n in ("resnet50", "resnet101", "resnet152"):
            return n
        if n in ("resnext50", "resnext101"):
            raise NotImplementedError("the ResNeXt backbones come from the third-party classification_models "
                                      "package; cvlite builds the ResNet and MobileNetV2 branches")
        return "mobilenetv2"

    A = 9
    def __init__(self, num_classes, n_anchors=9, backbone_model="resnet50", device="cuda", seed=0, precision=None):
        """precision: "bf16" (production) / "fp32" (parity mode); None = CVL_PRECISION or bf16."""
        self.A = n_anchors
        self._init_common(num_classes, backbone_model, device, seed, precision)
        self.cls_ld = self.cls_heads[0].npad
        self.reg_ld = self.reg_heads[0].npad

    def _build_heads(self, st, num_classes):
        A = self.A
        b_focal = math.log(0.01 / 0.99)
        cls_np = (A * num_classes + 127) // 128 * 128       # N tiles of the large conv kernels
        self.cls_heads = [Conv(st, "cls_output_%d" % (l + 1), 3, FPN_C, A * num_classes, bias_init=b_focal,
                               npad=cls_np, init_fan_out=9 * num_classes) for l in range(5)]
        self.reg_heads = [Conv(st, "reg_output_%d" % (l + 1), 3, FPN_C, A * 4, npad=64, init_fan_out=9 * 4)
                          for l in range(5)]

    def head_convs(self):
        return self.cls_heads + self.reg_heads

    def keras_names(self):
        """(Keras per-anchor name, store name, output-channel slice) for checkpoint interchange."""
        out = []
        for kind, heads, k in (("cls", self.cls_heads, self.C), ("reg", self.reg_heads, 4)):
            for l, hd in enumerate(heads):
                for a in range(self.A):
                    nm = "%s_output_%d_anchor_%d" % (kind, l + 1, a + 1)
                    out.append((nm + "/kernel", hd.wname, slice(a * k, (a + 1) * k)))
                    out.append((nm + "/bias", hd.bname, slice(a * k, (a + 1) * k)))
        return out

    def _heads_forward(self, towers, B, shapes, off, P):
        """Returns reg [B,P,reg_ld] fp32 (anchor a: t_y, t_x, t_h, t_w at 4a..), cls [B,P,cls_ld] fp32."""
        dev = towers[0][0].device
        cls_out = torch.empty((B, P, self.cls_ld), dtype=torch.float32, device=dev)
        reg_out = torch.empty((B, P, self.reg_ld), dtype=torch.float32, device=dev)
        for heads, acts, out, ld in ((self.cls_heads, towers[0], cls_out, self.cls_ld),
                                     (self.reg_heads, towers[1], reg_out, self.reg_ld)):
            segs = [nn.seg(h, w, h, w, heads[l].wf, heads[l].bias_arg(), src_base=B * off[l], src_img=h * w,
                           dst_base=off[l], dst_img=P) for l, (h, w) in enumerate(shapes)]
            d = heads[0].fwd_desc(B, segs, ld_dst=ld, dst_f32=True, n_store=heads[0].cout)
            nn.conv_igemm(d, acts[-1], out)
        return reg_out, cls_out

    def _heads_backward(self, grads, towers, B, shapes, off, P):
        """grads = (d_reg [B,P,reg_ld], d_cls [B,P,cls_ld]) bf16, padding channels zero."""
        d_reg, d_cls = grads
        dAs = []
        # the two towers' input gradients as the halves of one buffer: the trunk then runs each
        # tower layer's data gradient as one paired launch (FPNDetector.trunk_backward)
        a0 = towers[0][0]
        dA_pair = torch.empty((2,) + tuple(a0.shape), dtype=a0.dtype, device=a0.device)
        nn.bias_grad_multi([(dout, int(dout.shape[-1]), 0, heads[l].cout, off[l], P, h * w, B, heads[l].db, 0.0)
                            for heads, dout in ((self.cls_heads, d_cls), (self.reg_heads, d_reg))
                            for l, (h, w) in enumerate(shapes)])
        for heads, acts, dout in ((self.cls_heads, towers[0], d_cls), (self.reg_heads, towers[1], d_reg)):
            ld = int(dout.shape[-1])
            for l, (h, w) in enumerate(shapes):
                hd = heads[l]
                d = hd.fwd_desc(B, [nn.seg(h, w, h, w, hd.wf, None, src_base=B * off[l], src_img=h * w,
                                           dst_base=off[l], dst_img=P)], ld_dst=ld)
                nn.conv_wgrad(d, acts[-1], dout, hd.dw)
            dA = dA_pair[len(dAs)]
            segs = [nn.seg(h, w, h, w, heads[l].wd, None, src_base=off[l], src_img=P, dst_base=B * off[l],
                           dst_img=h * w) for l, (h, w) in enumerate(shapes)]
            d = heads[0].dgrad_desc(B, segs, ld_dst=FPN_C)
            nn.conv_igemm(d, dout, dA)
            dAs.append(dA)
        return dAs

    def outputs_nested(self, reg_out, cls_out, H, W):
        """The reference's model output: [5][A] list of [B, S, S, 4+C] (concat [reg4, clsC])."""
        B = reg_out.shape[0]
        shapes, off, P = self.layout(B, H, W)
        out = []
        for l, (h, w) in enumerate(shapes):
            lev = []
            for a in range(self.A):
                r = reg_out[:, off[l]:off[l] + h * w, 4 * a:4 * a + 4]
                c = cls_out[:, off[l]:off[l] + h * w, a * self.C:(a + 1) * self.C]
                lev.append(torch.cat([r, c], -1).reshape(B, h, w, 4 + self.C))
            out.append(lev)
        return out
