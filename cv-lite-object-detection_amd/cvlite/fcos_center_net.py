"""The centre-variant FCOS network of FCOS/fcos_center.py:6-122 and FCOS/fcos_center_v1.py:6-122
(one build_model each, identical but for the sigmoid on the v1 regression head) on the cvlite
kernels, explicit fwd/bwd.

It differs from fcos.py's network only in the heads (fcos_center.py:85-116): the centerness
logit is a 1-channel conv `cen_output_l` on the CLS tower (bias initialised to the focal prior,
like `logits_output_l`), and `reg_output_l` has 4 channels.  MI355X layout (same buffers as
FCOSNet, so the fused loss streams them once):
  * cls_out [B, P, ld] fp32: classes in columns 0..C-1, the centerness logit in column
    cc = round_up(C, 8) (8-aligned, so the centerness weight gradient reads its dY column with the
    16-byte kernels); reg_out [B, P, 8] fp32 columns 0..3;
  * per head type ONE 5-segment launch forward; the cls tower's top gradient (class head +
    centerness head) is ONE 5-segment data-gradient launch over the d_cls rows with a combined
    per-level kernel [3][3][256][ld] (class columns + the centerness column, zeros elsewhere)
    assembled from the two heads' fp32 weights and packed with the other convs after each update;
  * v1's sigmoid on the regression head is applied inside the fused loss (ops_targets.fcos_loss
    reg_sigmoid) and by `outputs_nested` for inference, so the conv writes raw logits.
Keras names kept: `logits_output_l`, `cen_output_l`, `reg_output_l` (l = 1..5).
"""
import math

import torch

from . import ops_nn as nn
from .fcos_net import FCOSNet
from .fpn_det import FPN_C
from .layers import Conv


class FCOSCenterNet(FCOSNet):
    @staticmethod
    def backbone_kind(name):
        """FCOS/fcos_center.py:30-48 (and fcos_center_v1.py:30-48): "resnet50" -> ResNet50,
        "resnet101" -> ResNet101 (taps conv3_block4_out / conv4_block23_out / conv5_block3_out),
        every other name -> MobileNetV2.  (Plain fcos.py:29-41 has no ResNet101 branch.)"""
        n = name.lower()
        return n if n in ("resnet50", "resnet101") else "mobilenetv2"

    def __init__(self, num_classes, backbone_model="resnet50", device="cuda", seed=0, v1=False):
        self.v1 = v1
        # the combined class + centerness data-gradient kernels are packed bf16: production precision
        self._init_common(num_classes, backbone_model, device, seed, precision="bf16")
        self.cen_col, self.cls_ld = self._comb_cc, self._comb_ld
        self.reg_ld = 8

    def _build_heads(self, st, num_classes):
        b_focal = math.log(0.01 / 0.99)
        self.cls_heads, self.cen_heads = [], []
        for l in range(5):       # the data gradient runs on the combined kernel (pack): no own dgrad pack
            self.cen_heads.append(Conv(st, "cen_output_%d" % (l + 1), 3, FPN_C, 1, bias_init=b_focal, dgrad=False))
            self.cls_heads.append(Conv(st, "logits_output_%d" % (l + 1), 3, FPN_C, num_classes, bias_init=b_focal,
                                       dgrad=False))
        self.reg_heads = [Conv(st, "reg_output_%d" % (l + 1), 3, FPN_C, 4) for l in range(5)]

    def head_convs(self):
        return self.cls_heads + self.cen_heads + self.reg_heads

    def pack(self):
        """Assemble the combined class + centerness data-gradient kernels from the fp32 masters, then
        the batched re-pack of every conv (FPNDetector.pack) including them."""
        if getattr(self, "_comb", None) is None:
            cc = (self.C + 7) // 8 * 8
            ld = (cc + 32 + 31) // 32 * 32      # the centerness wgrad reads 32 dY columns from cc
            dev = self.store.flat.device
            self._comb = [torch.zeros((3, 3, FPN_C, ld), dtype=torch.float32, device=dev) for _ in range(5)]
            self._comb_wd = [torch.empty((FPN_C, 9 * ld), dtype=torch.bfloat16, device=dev) for _ in range(5)]
            self._comb_cc, self._comb_ld = cc, ld
        cc = self._comb_cc
        for l in range(5):
            self._comb[l][..., :self.C].copy_(self.cls_heads[l].w)
            self._comb[l][..., cc:cc + 1].copy_(self.cen_heads[l].w)
        if self._pack_plan is None:
            bb = set(id(c) for c in self.backbone.convs())
            entries = self.backbone.pack_entries()
            for c in self.all_convs():
                if id(c) not in bb:
                    entries += c.pack_entries()
            ld = self._comb_ld
            entries += [(self._comb[l], 9, FPN_C, ld, FPN_C, ld, None, FPN_C, ld, self._comb_wd[l]) for l in range(5)]
            self._pack_plan = nn.PackPlan(entries, self.device)
        self._pack_plan.run()

    def _head_launch(self, heads, acts, out, ld, coff, B, shapes, off, P):
        segs = [nn.seg(h, w, h, w, heads[l].wf, heads[l].bias_arg(), src_base=B * off[l], src_img=h * w,
                       dst_base=off[l], dst_img=P) for l, (h, w) in enumerate(shapes)]
        d = heads[0].fwd_desc(B, segs, ld_dst=ld, dst_coff=coff, dst_f32=True, n_store=heads[0].cout)
        nn.conv_igemm(d, acts, out)

    def _heads_forward(self, towers, B, shapes, off, P):
        """Returns reg [B,P,8] fp32 (raw t,b,l,r logits), cls [B,P,ld] fp32 (classes, centerness at
        column cen_col)."""
        dev = towers[0][0].device
        cls_out = torch.zeros((B, P, self.cls_ld), dtype=torch.float32, device=dev)
        reg_out = torch.zeros((B, P, self.reg_ld), dtype=torch.float32, device=dev)
        self._head_launch(self.cls_heads, towers[0][-1], cls_out, self.cls_ld, 0, B, shapes, off, P)
        self._head_launch(self.cen_heads, towers[0][-1], cls_out, self.cls_ld, self.cen_col, B, shapes, off, P)
        self._head_launch(self.reg_heads, towers[1][-1], reg_out, self.reg_ld, 0, B, shapes, off, P)
        return reg_out, cls_out

    def _heads_backward(self, grads, towers, B, shapes, off, P):
        """grads = (d_reg [B,P,32], d_cls [B,P,ld]) bf16 from the fused loss (centre flags)."""
        d_reg, d_cls = grads
        a0 = towers[0][0]
        dA_pair = torch.empty((2,) + tuple(a0.shape), dtype=a0.dtype, device=a0.device)
        items = []
        for heads, dout, coff in ((self.cls_heads, d_cls, 0), (self.cen_heads, d_cls, self.cen_col),
                                  (self.reg_heads, d_reg, 0)):
            items += [(dout, int(dout.shape[-1]), coff, heads[l].cout, off[l], P, h * w, B, heads[l].db, 0.0)
                      for l, (h, w) in enumerate(shapes)]
        nn.bias_grad_multi(items)
        for heads, acts, dout, coff in ((self.cls_heads, towers[0], d_cls, 0),
                                        (self.cen_heads, towers[0], d_cls, self.cen_col),
                                        (self.reg_heads, towers[1], d_reg, 0)):
            ld = int(dout.shape[-1])
            d = heads[0].fwd_desc(B, [nn.seg(h, w, h, w, heads[l].wf, None, src_base=B * off[l], src_img=h * w,
                                             dst_base=off[l], dst_img=P) for l, (h, w) in enumerate(shapes)],
                                  ld_dst=ld, dst_coff=coff)
            nn.conv_wgrad_grouped(d, acts[-1], dout, [heads[l].dw for l in range(len(shapes))])
        # data gradients: cls tower from the combined class + centerness kernels over all d_cls
        # columns (pitch ld = the combined kernel's K channels); reg tower from the reg head
        ld = self._comb_ld
        assert int(d_cls.shape[-1]) == ld
        _, _, pt, pl = self.cls_heads[0].out_hw(shapes[0][0], shapes[0][1])
        segs = [nn.seg(h, w, h, w, self._comb_wd[l], None, src_base=off[l], src_img=P, dst_base=B * off[l],
                       dst_img=h * w) for l, (h, w) in enumerate(shapes)]
        d = nn.make_desc(nn.DGRAD, B, ld, 3, 3, 1, pt, pl, FPN_C, FPN_C, FPN_C, segs)
        nn.conv_igemm(d, d_cls, dA_pair[0])
        segs = [nn.seg(h, w, h, w, self.reg_heads[l].wd, None, src_base=off[l], src_img=P, dst_base=B * off[l],
                       dst_img=h * w) for l, (h, w) in enumerate(shapes)]
        nn.conv_igemm(self.reg_heads[0].dgrad_desc(B, segs, ld_dst=FPN_C), d_reg, dA_pair[1])
        return [dA_pair[0], dA_pair[1]]

    def outputs_nested(self, reg_out, cls_out, H, W):
        """The reference model output: [5] list of [B, S, S, 5+C] = concat[reg(4), cen(1), cls(C)]
        (v1: sigmoid on the reg channels)."""
        B = reg_out.shape[0]
        shapes, off, P = self.layout(B, H, W)
        out = []
        for l, (h, w) in enumerate(shapes):
            r = reg_out[:, off[l]:off[l] + h * w, :4]
            if self.v1:
                r = torch.sigmoid(r)
            c = cls_out[:, off[l]:off[l] + h * w, self.cen_col:self.cen_col + 1]
            k = cls_out[:, off[l]:off[l] + h * w, :self.C]
            out.append(torch.cat([r, c, k], -1).reshape(B, h, w, 5 + self.C))
        return out
