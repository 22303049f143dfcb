"""CenterNet ResNet stride-8 multi-scale detector (CenterNet/tf_centernet_resnet_s8.py build_model
:87-208, as train_centernet_crowdhuman.py builds it: backbone_model="resnet101", n_scales = 5) as an
explicit forward / backward graph on the cvlite kernels.

Graph: Keras ResNet C3 / C4 / C5 (per-image BatchNorm: the trainer's sub_batch_sz is 1), 1x1
laterals `c3_1x1`..`c5_1x1`, P6 = ReLU(conv3x3/2(P5_1x1)) (`c6_3x3`), P7 = conv3x3/2(P6)
(`c7_3x3`), nearest x2 top-down residuals P6 + up(P7) -> P5_1x1 + up(.) -> P4 -> P3, the 3x3
`cnn_feature_map` on P3 (stride 8), the shared 4-layer towers (`cls_layer_k` / `reg_layer_k`: no
bias, no activation between layers, one ReLU), per-scale 3x3 heads `cnn_cls_output_<s>` (C,
b_focal bias init) and `cnn_reg_output_<s>` (4, sigmoid inside the fused loss).

MI355X mapping: every scale calls the SAME tower layers on the SAME input (:171-190), so the towers
run once; the n_scales heads of a kind share their input, so they run as ONE conv whose output
channels are the scales' heads side by side (`cls_comb` / `reg_comb`, assembled from the heads'
fp32 weights before each re-pack; their weight / bias gradients are scattered back to the heads).
The towers' weight gradient therefore sums over the scales exactly as the reference's repeated
layer calls do.  Reference quirk kept visible: build_model's `if resnet50 / if resnet101 / else
MobileNetV2` sends backbone_model="resnet50" to the MobileNetV2 branch (Q-s8); only "resnet101"
builds a ResNet (cvlite.mobilenet_v2 serves the other names).
"""
import math

import torch

from . import ops_nn as nn
from .layers import BF16, Conv, ParamStore, constant
from .mobilenet_v2 import MobileNetV2
from .resnet import ResNet50

FPN_C = 256


class CenterNetS8Net(object):
    def __init__(self, num_classes, n_scales=5, backbone_model="resnet101", device="cuda", seed=0):
        # :117-131: `if resnet50: ...` is followed by `if resnet101: ... else: MobileNetV2`, so only
        # "resnet101" keeps a ResNet; every other name (including "resnet50") ends on MobileNetV2
        self.backbone_model = "resnet101" if backbone_model.lower() == "resnet101" else "mobilenetv2"
        self.C, self.ns = num_classes, n_scales
        self.device = torch.device(device)
        st, eff = ParamStore(), ParamStore()
        self._build(st, eff, num_classes, n_scales)
        st.finalize(self.device, seed)
        eff.finalize(self.device, seed + 1)
        self.store, self.eff = st, eff
        for bn in self.backbone.bns():
            bn.init_buffers(self.device)
        self.cls_ld, self.reg_ld = self.cls_comb.npad, self.reg_comb.npad
        self._plan = None
        self._saved = None
        self.pack()

    def _build(self, st, eff, C, ns):
        # creation order follows build_model: towers, backbone, FPN, feature map, heads
        self.cls_tower = [Conv(st, "cls_layer_%d" % (i + 1), 3, FPN_C, FPN_C, bias=False) for i in range(4)]
        self.reg_tower = [Conv(st, "reg_layer_%d" % (i + 1), 3, FPN_C, FPN_C, bias=False) for i in range(4)]
        kind = getattr(self, "backbone_model", "resnet101")
        self.backbone = ResNet50(st, "resnet101") if kind == "resnet101" else MobileNetV2(st)
        t3, t4, t5 = self.backbone.tap_channels
        self.c3_1x1 = Conv(st, "c3_1x1", 1, t3, FPN_C)
        self.c4_1x1 = Conv(st, "c4_1x1", 1, t4, FPN_C)
        self.c5_1x1 = Conv(st, "c5_1x1", 1, t5, FPN_C)
        self.c6_3x3 = Conv(st, "c6_3x3", 3, FPN_C, FPN_C, stride=2)
        self.c7_3x3 = Conv(st, "c7_3x3", 3, FPN_C, FPN_C, stride=2)
        self.feat = Conv(st, "cnn_feature_map", 3, FPN_C, FPN_C)
        b_focal = math.log(0.01 / 0.99)
        self.cls_heads = [Conv(st, "cnn_cls_output_%d" % (s + 1), 3, FPN_C, C, bias_init=b_focal, dgrad=False)
                          for s in range(ns)]
        self.reg_heads = [Conv(st, "cnn_reg_output_%d" % (s + 1), 3, FPN_C, 4, dgrad=False) for s in range(ns)]
        self.cls_comb = Conv(eff, "cls_comb", 3, FPN_C, ns * C)
        self.reg_comb = Conv(eff, "reg_comb", 3, FPN_C, ns * 4)

    # ---- parameters ---------------------------------------------------------------------------
    def convs(self):
        return (self.cls_tower + self.reg_tower + [self.c3_1x1, self.c4_1x1, self.c5_1x1, self.c6_3x3,
                                                   self.c7_3x3, self.feat, self.cls_comb, self.reg_comb])

    def bns(self):
        return self.backbone.bns()

    def grad_groups(self):
        return [("all", list(self.store.offsets))]

    def _assemble(self):
        for comb, heads, w in ((self.cls_comb, self.cls_heads, self.C), (self.reg_comb, self.reg_heads, 4)):
            for s, h in enumerate(heads):
                comb.w[..., s * w:(s + 1) * w].copy_(h.w)
                comb.b[s * w:(s + 1) * w].copy_(h.b)

    def _scatter_grads(self):
        for comb, heads, w in ((self.cls_comb, self.cls_heads, self.C), (self.reg_comb, self.reg_heads, 4)):
            for s, h in enumerate(heads):
                h.dw.copy_(comb.dw[..., s * w:(s + 1) * w])
                h.db.copy_(comb.db[s * w:(s + 1) * w])

    def pack(self):
        """Assemble the combined heads, then one batched bf16 re-pack of every conv."""
        self._assemble()
        if self._plan is None:
            entries = self.backbone.pack_entries()
            for c in self.convs():
                entries += c.pack_entries()
            self._plan = nn.PackPlan(entries, self.device)
        self._plan.run()

    @staticmethod
    def out_hw(H, W):
        return H // 8, W // 8

    # ---- forward / backward -----------------------------------------------------------------
    def forward(self, x, train=True):
        """x [B,H,W,3] fp32 (H, W multiples of 128) -> (reg [B,P,ns*4], cls [B,P,ns*C]) fp32 raw
        logits, P = (H/8)*(W/8), cell-major then scale."""
        B, H, W, _ = x.shape
        assert H % 128 == 0 and W % 128 == 0, "the P7 -> P3 residual chain needs H, W multiples of 128"
        dev = x.device
        (C3, C4, C5), bsv = self.backbone.forward(x, train)
        (c3, H3, W3), (c4, H4, W4), (c5, H5, W5) = C3, C4, C5
        l3, _, _ = self.c3_1x1.fwd(c3, B, H3, W3)
        l4, _, _ = self.c4_1x1.fwd(c4, B, H4, W4)
        l5, _, _ = self.c5_1x1.fwd(c5, B, H5, W5)
        p6r, H6, W6 = self.c6_3x3.fwd(l5, B, H5, W5, relu_out=True)
        p7, H7, W7 = self.c7_3x3.fwd(p6r, B, H6, W6)
        r6 = torch.empty_like(p6r)
        nn.upsample2x_add(p6r, p7, r6, B, H6, W6, FPN_C)
        r5 = torch.empty_like(l5)
        nn.upsample2x_add(l5, r6, r5, B, H5, W5, FPN_C)
        r4 = torch.empty_like(l4)
        nn.upsample2x_add(l4, r5, r4, B, H4, W4, FPN_C)
        r3 = torch.empty_like(l3)
        nn.upsample2x_add(l3, r4, r3, B, H3, W3, FPN_C)
        f, _, _ = self.feat.fwd(r3, B, H3, W3)
        towers = []
        for tw in (self.cls_tower, self.reg_tower):
            acts = [f]
            for i, c in enumerate(tw):
                y, _, _ = c.fwd(acts[-1], B, H3, W3, relu_out=(i == 3))
                acts.append(y)
            towers.append(acts)
        P = H3 * W3
        outs = []
        for comb, acts in ((self.reg_comb, towers[1]), (self.cls_comb, towers[0])):
            o = torch.empty((B, P, comb.cout), dtype=torch.float32, device=dev)
            d = comb.fwd_desc(B, [nn.seg(H3, W3, H3, W3, comb.wf, comb.b)], ld_dst=comb.cout, dst_f32=True)
            nn.conv_igemm(d, acts[-1], o)
            outs.append(o)
        self._saved = dict(bsv=bsv, C=(C3, C4, C5), l=(l3, l4, l5), p6r=p6r, r=(r3, r4, r5, r6), towers=towers,
                           B=B, hw=((H3, W3), (H4, W4), (H5, W5), (H6, W6), (H7, W7)))
        return outs[0], outs[1]

    def backward(self, d_reg, d_cls, hook=None):
        """d_reg bf16 [B,P,reg_ld], d_cls bf16 [B,P,cls_ld] (cvl_centernet_s8_loss)."""
        s = self._saved
        B = s["B"]
        (H3, W3), (H4, W4), (H5, W5), (H6, W6), (H7, W7) = s["hw"]
        towers = s["towers"]
        dts = []
        for comb, acts, dy in ((self.cls_comb, towers[0], d_cls), (self.reg_comb, towers[1], d_reg)):
            comb.wgrad(acts[-1], dy, B, H3, W3)                      # weight + bias (all scales)
            dt = comb.dgrad(dy, B, H3, W3)
            nn.relu_backward(dt, acts[-1], dt)                       # the towers' final ReLU
            dts.append(dt)
        self._scatter_grads()
        df = torch.empty_like(towers[0][0])
        for t, tw in enumerate((self.cls_tower, self.reg_tower)):
            g = dts[t]
            for i in range(3, -1, -1):
                c = tw[i]
                c.wgrad(towers[t][i], g, B, H3, W3)
                if i > 0:
                    g = c.dgrad(g, B, H3, W3)
                else:
                    c.dgrad(g, B, H3, W3, out=df, beta=(1.0 if t == 1 else 0.0))
        r3, r4, r5, r6 = s["r"]
        self.feat.wgrad(r3, df, B, H3, W3)
        dr3 = self.feat.dgrad(df, B, H3, W3)
        # r3 = l3 + up(r4), r4 = l4 + up(r5), r5 = l5 + up(r6), r6 = p6r + up(p7)
        dr4 = torch.empty_like(r4)
        nn.upsample2x_backward(dr3, dr4, B, H3, W3, FPN_C)
        dr5 = torch.empty_like(r5)
        nn.upsample2x_backward(dr4, dr5, B, H4, W4, FPN_C)
        dr6 = torch.empty_like(r6)
        nn.upsample2x_backward(dr5, dr6, B, H5, W5, FPN_C)
        dp7 = torch.empty((B, H7, W7, FPN_C), dtype=BF16, device=df.device)
        nn.upsample2x_backward(dr6, dp7, B, H6, W6, FPN_C)
        p6r = s["p6r"]
        l3, l4, l5 = s["l"]
        self.c7_3x3.wgrad(p6r, dp7, B, H6, W6)
        self.c7_3x3.dgrad(dp7, B, H6, W6, out=dr6, beta=1.0)          # d relu(P6)
        nn.relu_backward(dr6, p6r, dr6)
        self.c6_3x3.wgrad(l5, dr6, B, H5, W5)
        self.c6_3x3.dgrad(dr6, B, H5, W5, out=dr5, beta=1.0)          # d P5_1x1
        (C3, C4, C5) = s["C"]
        dC = []
        for conv, (src, h, w), dl in ((self.c3_1x1, C3, dr3), (self.c4_1x1, C4, dr4), (self.c5_1x1, C5, dr5)):
            conv.wgrad(src, dl, B, h, w)
            dC.append(conv.dgrad(dl, B, h, w))
        self.backbone.backward(dC, s["bsv"], hook=None)
        self._saved = None
        if hook is not None:
            hook("all")

    def outputs(self, reg, cls, H, W):
        """The Keras model output [B,S,S,ns,4+C]: sigmoid boxes, class logits."""
        B = reg.shape[0]
        S0, S1 = H // 8, W // 8
        r = torch.sigmoid(reg.view(B, S0, S1, self.ns, 4))
        return torch.cat([r, cls.view(B, S0, S1, self.ns, self.C)], -1)

    @staticmethod
    def param_dict(num_classes, n_scales=5, seed=0, backbone_model="resnet101"):
        """Initial parameters (Keras names -> CPU fp32) without a GPU (oracle / checkpoints)."""
        obj = CenterNetS8Net.__new__(CenterNetS8Net)
        obj.backbone_model = "resnet101" if backbone_model.lower() == "resnet101" else "mobilenetv2"
        st, eff = ParamStore(), ParamStore()
        obj._build(st, eff, num_classes, n_scales)
        st.finalize("cpu", seed)
        return st.state_dict()
