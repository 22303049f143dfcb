"""Shared trunk of the FPN detectors (FCOS/fcos.py:6-110, RetinaNet/retinanet_module.py:8-159):
Keras ResNet-50 v1 backbone, the FPN of both modules (identical code in the reference, incl. the
P3 += up2(P4_1x1) and P6-from-C5 quirks) and the two shared 4-layer towers (3x3
256->256, no bias, no activation between layers, one final ReLU, Q14), explicit fwd/bwd.

MI355X layout decisions:
* P3..P7 live in ONE packed, level-major bf16 buffer [sum_l B*S_l^2, 256]; each shared tower
  layer (`cls_layer_k` / `reg_layer_k`) is one segmented MFMA launch over all five levels (shared
  weights), forward, data-gradient and weight-gradient (the weight gradient reduces over all
  levels and images at once -- the reference loops levels in Python).
* c7_3x3 reads relu(P6) through the conv's relu-on-load flag (fcos.py:70-72).
* Subclasses add the per-level output heads (`_build_heads`, `_heads_forward`, `_heads_backward`).
"""
import os

import torch

from . import ops_nn as nn
from .layers import BF16, Conv, ParamStore, act_dtype, wgrad_batch
from .layers import conv_wgrad as wgrad_collect
from .mobilenet_v2 import MobileNetV2
from .resnet import ResNet50
from . import _lib

FPN_C = 256
STRIDES = (8, 16, 32, 64, 128)


# CVL_DISPATCH=no_tower_pair runs the two towers as separate launches (A/B only; the paired
# 10-segment launches are the default)
PAIR_TOWERS = not _lib.dispatch("no_tower_pair")


def pair_tower0_dgrad():
    """Tower layer 0 reads the shared F: its two data gradients as ONE paired launch into a
    temporary + one add (default), or (CVL_DISPATCH=no_tower0_pair) two launches, the second
    accumulating into dF.  Read per backward, so both forms are testable in one process."""
    return not _lib.dispatch("no_tower0_pair")

# CVL_DISPATCH=no_fpn_fuse runs P3..P5's 3x3 output convs as separate launches (A/B only)
FUSE_FPN = not _lib.dispatch("no_fpn_fuse")
# weight-gradient split reductions batched per gradient group (ops_nn.deferred_wgrad;
# CVL_DISPATCH=no_wgrad_defer: one reduction launch per weight gradient)
DEFER_WGRAD = not _lib.dispatch("no_wgrad_defer")

class FPNDetector(object):
    @staticmethod
    def backbone_kind(name):
        """FCOS/fcos.py:29-41: "resnet50" builds ResNet50, EVERY other name builds MobileNetV2
        (fcos_center*.py add a ResNet101 branch: FCOSCenterNet.backbone_kind)."""
        return "resnet50" if name.lower() == "resnet50" else "mobilenetv2"

    def _init_common(self, num_classes, backbone_model, device, seed, precision=None):
        self.backbone_model = self.backbone_kind(backbone_model)
        self.C = num_classes
        self.store = st = ParamStore()
        st.act = act_dtype(precision)      # bf16 (production) or fp32 (parity mode)
        if st.act != BF16 and self.backbone_model != "resnet50" and self.backbone_model != "resnet101":
            raise NotImplementedError("the fp32 parity mode covers the ResNet backbones")
        self._build_layers(st, num_classes)
        st.finalize(device, seed)
        for bn in self.backbone.bns():
            bn.init_buffers(device)
        self.device = device
        self._pack_plan = None
        self.pack()

    def _build_layers(self, st, num_classes):
        # creation order follows build_model: towers, backbone, FPN, heads
        self.cls_tower = [Conv(st, "cls_layer_%d" % (i + 1), 3, FPN_C, FPN_C, bias=False) for i in range(4)]
        self.reg_tower = [Conv(st, "reg_layer_%d" % (i + 1), 3, FPN_C, FPN_C, bias=False) for i in range(4)]
        kind = getattr(self, "backbone_model", "resnet50")
        self.backbone = MobileNetV2(st) if kind == "mobilenetv2" else ResNet50(st, kind)
        t3, t4, t5 = self.backbone.tap_channels
        self.c3_1x1 = Conv(st, "c3_1x1", 1, t3, FPN_C)
        self.c4_1x1 = Conv(st, "c4_1x1", 1, t4, FPN_C)
        self.c5_1x1 = Conv(st, "c5_1x1", 1, t5, FPN_C)
        self.c3_3x3 = Conv(st, "c3_3x3", 3, FPN_C, FPN_C)
        self.c4_3x3 = Conv(st, "c4_3x3", 3, FPN_C, FPN_C)
        self.c5_3x3 = Conv(st, "c5_3x3", 3, FPN_C, FPN_C)
        self.c6_3x3 = Conv(st, "c6_3x3", 3, t5, FPN_C, stride=2)
        self.c7_3x3 = Conv(st, "c7_3x3", 3, FPN_C, FPN_C, stride=2)
        self._build_heads(st, num_classes)

    @classmethod
    def param_dict(cls, num_classes, seed=0, backbone_model="resnet50"):
        """The initial parameters (Keras names -> CPU fp32) without touching a GPU."""
        obj = cls.__new__(cls)
        obj.backbone_model = cls.backbone_kind(backbone_model)
        st = ParamStore()
        obj._build_layers(st, num_classes)
        st.finalize("cpu", seed)
        return st.state_dict()

    # ---- parameters ------------------------------------------------------------------------------
    def head_convs(self):
        raise NotImplementedError

    def all_convs(self):
        return (self.cls_tower + self.reg_tower + self.backbone.convs()[1:] +
                [self.c3_1x1, self.c4_1x1, self.c5_1x1, self.c3_3x3, self.c4_3x3, self.c5_3x3,
                 self.c6_3x3, self.c7_3x3] + self.head_convs())

    def pack(self):
        """Refresh the bf16 packed weights from the fp32 masters (after every update): one
        batched launch over every conv (ops_nn.PackPlan)."""
        if self._pack_plan is None:
            bb = set(id(c) for c in self.backbone.convs())
            entries = self.backbone.pack_entries()
            for c in self.all_convs():
                if id(c) not in bb:
                    entries += c.pack_entries()
            self._pack_plan = nn.PackPlan(entries, self.device)
        self._pack_plan.run()

    # ---- geometry ---------------------------------------------------------------------------------
    @staticmethod
    def level_shapes(H, W):
        return [(-(-H // s), -(-W // s)) for s in STRIDES]

    def layout(self, B, H, W):
        shapes = self.level_shapes(H, W)
        off, o = [], 0
        for (h, w) in shapes:
            off.append(o)
            o += h * w
        return shapes, off, o     # per-image cell offsets, P

    def _tower_segs(self, conv, B, shapes, off, wf=True):
        return [nn.seg(h, w, h, w, conv.wf if wf else conv.wd, None, src_base=B * off[l], src_img=h * w,
                       dst_base=B * off[l], dst_img=h * w) for l, (h, w) in enumerate(shapes)]

    def _pair_segs(self, i, B, shapes, off, P, fwd=True):
        """Segments of tower layer i for BOTH towers (cls rows [0, B*P), reg rows [B*P, 2*B*P) of
        the source and destination buffers).  Forward layer 0 reads the shared FPN buffer F
        (both towers at offset 0); dgrad layers read/write the paired gradient buffers."""
        segs = []
        for t, tw in enumerate((self.cls_tower, self.reg_tower)):
            conv = tw[i]
            s_off = 0 if (fwd and i == 0) else t * B * P
            segs += [nn.seg(h, w, h, w, conv.wf if fwd else conv.wd, None, src_base=s_off + B * off[l],
                            src_img=h * w, dst_base=t * B * P + B * off[l], dst_img=h * w)
                     for l, (h, w) in enumerate(shapes)]
        return segs

    # ---- forward -------------------------------------------------------------------------------------
    def trunk_forward(self, x, train=True):
        """Backbone + FPN + both towers.  Returns the two towers' activation lists (each [F, a1..a4],
        a4 = ReLU output) over the packed level-major buffer."""
        B, H, W, _ = x.shape
        dev = x.device
        (C3, C4, C5), bsv = self.backbone.forward(x, train)
        (c3, H3, W3), (c4, H4, W4), (c5, H5, W5) = C3, C4, C5
        # the three 3x3 output convs' sources (P3r, P4r, P5 = l5) share one buffer, so the convs run
        # as ONE 3-segment launch (fcos.py:62-66: same geometry, own weights and biases)
        n3, n4, n5 = B * H3 * W3, B * H4 * W4, B * H5 * W5
        PR = torch.empty((n3 + n4 + n5, FPN_C), dtype=self.store.act, device=dev)
        p3r = PR[:n3].view(B, H3, W3, FPN_C)
        p4r = PR[n3:n3 + n4].view(B, H4, W4, FPN_C)
        l3, _, _ = self.c3_1x1.fwd(c3, B, H3, W3)
        l4, _, _ = self.c4_1x1.fwd(c4, B, H4, W4)
        l5, _, _ = self.c5_1x1.fwd(c5, B, H5, W5, out=PR[n3 + n4:].view(B, H5, W5, FPN_C))
        nn.upsample2x_add(l4, l5, p4r, B, H4, W4, FPN_C)          # fcos.py:57-58
        nn.upsample2x_add(l3, l4, p3r, B, H3, W3, FPN_C)          # fcos.py:59-60 (up2 of P4_1x1, Q13)
        shapes, off, P = self.layout(B, H, W)
        F = torch.empty((B * P, FPN_C), dtype=self.store.act, device=dev)
        pr_base = (0, n3, n3 + n4)
        if FUSE_FPN:
            segs = [nn.seg(shapes[l][0], shapes[l][1], h, w, conv.wf, conv.bias_arg(), src_base=pr_base[l],
                           dst_base=B * off[l])
                    for l, (conv, h, w) in enumerate(((self.c3_3x3, H3, W3), (self.c4_3x3, H4, W4),
                                                      (self.c5_3x3, H5, W5)))]
            nn.conv_igemm(self.c3_3x3.fwd_desc(B, segs, ld_dst=FPN_C), PR, F)
            srcs = [None, None, None, (self.c6_3x3, c5, H5, W5)]
        else:
            srcs = [(self.c3_3x3, p3r, H3, W3), (self.c4_3x3, p4r, H4, W4), (self.c5_3x3, l5, H5, W5),
                    (self.c6_3x3, c5, H5, W5)]
        for l, sc in enumerate(srcs):
            if sc is None:
                continue
            conv, src, h, w = sc
            Ho, Wo = shapes[l]
            d = conv.fwd_desc(B, [nn.seg(Ho, Wo, h, w, conv.wf, conv.bias_arg(), dst_base=B * off[l])],
                              ld_dst=FPN_C)
            nn.conv_igemm(d, src, F)
        h6, w6 = shapes[3]
        d = self.c7_3x3.fwd_desc(B, [nn.seg(shapes[4][0], shapes[4][1], h6, w6, self.c7_3x3.wf,
                                            self.c7_3x3.bias_arg(), src_base=B * off[3], dst_base=B * off[4])],
                                 ld_dst=FPN_C, relu_in=True)
        nn.conv_igemm(d, F, F)                                      # P7 = conv(relu(P6))
        # fcos.py:76-101: the cls and reg towers share geometry, so each tower layer is ONE launch
        # of 10 segments (2 towers x 5 levels, each with its own weights) writing a [2*B*P, 256]
        # buffer whose halves are the two towers' activations
        towers = [[F], [F]]
        bufs = []
        src = F
        for i in range(4):
            out = torch.empty((2 * B * P, FPN_C), dtype=self.store.act, device=dev)
            if PAIR_TOWERS:
                d = self.cls_tower[i].fwd_desc(B, self._pair_segs(i, B, shapes, off, P, fwd=True), ld_dst=FPN_C,
                                               relu_out=(i == 3))
                probe = getattr(self, "tower_probe", None)      # bench.py: in-step launch timing
                if probe is not None:
                    nn.probe_arm(probe)
                nn.conv_igemm(d, src, out)
            else:                                   # A/B reference: one launch per tower
                for t, tw in enumerate((self.cls_tower, self.reg_tower)):
                    d = tw[i].fwd_desc(B, self._tower_segs(tw[i], B, shapes, off), ld_dst=FPN_C, relu_out=(i == 3))
                    nn.conv_igemm(d, towers[t][-1], out[t * B * P:(t + 1) * B * P])
            towers[0].append(out[:B * P])
            towers[1].append(out[B * P:])
            bufs.append(out)
            src = out
        self._saved = dict(bsv=bsv, C=(C3, C4, C5), l=(l3, l4, l5), p=(p3r, p4r), PR=PR, F=F, towers=towers,
                           tower_bufs=bufs, B=B, H=H, W=W, shapes=shapes, off=off, P=P)
        return towers

    def forward(self, x, train=True):
        towers = self.trunk_forward(x, train)
        s = self._saved
        return self._heads_forward(towers, s["B"], s["shapes"], s["off"], s["P"])

    # ---- gradient groups (data-parallel overlap, dist.GradSync) ---------------------------------------
    def grad_groups(self):
        """[(name, param names)] in the order backward() finalises them; backward(hook=) calls
        hook(name) at each of these points."""
        def names(convs):
            return [n for c in convs for n in (c.wname, c.bname) if n]

        def units(us):
            return [n for u in us for n in (u.conv.wname, u.conv.bname, u.bn.gname, u.bn.bname)]
        bb = self.backbone
        g = [("heads_towers", names(self.head_convs() + self.cls_tower + self.reg_tower)),
             ("fpn", names([self.c3_1x1, self.c4_1x1, self.c5_1x1, self.c3_3x3, self.c4_3x3, self.c5_3x3,
                            self.c6_3x3, self.c7_3x3]))]
        if isinstance(bb, MobileNetV2):
            return g + [("backbone", bb.param_names())]
        for si in (3, 2, 1):
            g.append(("conv%d" % (si + 2), units([u for b in bb.stages[si] for u in b.units()])))
        stem = [bb.stem.conv.wname, bb.stem.conv.bname, bb.stem.bn.gname, bb.stem.bn.bname]
        g.append(("conv2_stem", units([u for b in bb.stages[0] for u in b.units()]) + stem))
        return g

    # ---- backward ------------------------------------------------------------------------------------
    def backward(self, *head_grads, hook=None):
        """The split weight-gradient reductions run deferred: one batched launch before each gradient
        group is reported final (hook) and one at the end (DEFER_WGRAD; CVL_DISPATCH=no_wgrad_defer: off)."""
        s = self._saved
        if not DEFER_WGRAD:
            dA = self._heads_backward(head_grads, s["towers"], s["B"], s["shapes"], s["off"], s["P"])
            self.trunk_backward(dA, hook=hook)
            return

        def flush_then(name):
            nn.wgrad_flush()
            if hook is not None:
                hook(name)
        with nn.deferred_wgrad():
            dA = self._heads_backward(head_grads, s["towers"], s["B"], s["shapes"], s["off"], s["P"])
            self.trunk_backward(dA, hook=flush_then)

    def trunk_backward(self, dA_top, hook=None):
        """dA_top: per tower, the gradient w.r.t. its ReLU output (buffer reused in place).
        hook(name) fires as each grad_groups() group becomes final."""
        hook = hook or (lambda name: None)
        s = self._saved
        B, shapes, off, P = s["B"], s["shapes"], s["off"], s["P"]
        dev = s["F"].device
        F, towers = s["F"], s["towers"]
        dF = torch.empty_like(F)
        dAs = list(dA_top)
        BP = B * P
        # the two towers' gradients are the halves of one [2*B*P, 256] buffer (the heads' backward
        # allocates them so): then each tower layer's data gradient is ONE 10-segment launch
        paired = PAIR_TOWERS and (dAs[1].data_ptr() - dAs[0].data_ptr() == BP * FPN_C * dAs[0].element_size()
                  and dAs[0].is_contiguous() and dAs[1].is_contiguous())
        pair0 = pair_tower0_dgrad()
        # the towers' final ReLU: one launch over both halves when they are one buffer (skipped when
        # the heads' data gradients applied it in their epilogues: FCOSNet._heads_backward)
        y_top = s["tower_bufs"][-1]
        if self.__dict__.pop("_top_relu_done", False):
            pass
        elif paired and towers[1][-1].data_ptr() - towers[0][-1].data_ptr() == BP * FPN_C * y_top.element_size():
            dA_all = torch.as_strided(dAs[0], (2 * BP, FPN_C), (FPN_C, 1))
            nn.relu_backward(dA_all, y_top, dA_all)
        else:
            for t in range(2):
                nn.relu_backward(dAs[t], towers[t][-1], dAs[t])
        for i in range(3, -1, -1):
            if paired:      # both towers' weight gradients: ONE launch, 2 groups x 5 levels
                d = self.cls_tower[i].fwd_desc(B, self._pair_segs(i, B, shapes, off, P, fwd=True), ld_dst=FPN_C)
                x_all = F if i == 0 else s["tower_bufs"][i - 1]
                dy_all = torch.as_strided(dAs[0], (2 * BP, FPN_C), (FPN_C, 1))
                nn.conv_wgrad_grouped(d, x_all, dy_all, [self.cls_tower[i].dw, self.reg_tower[i].dw])
            else:
                for t, tw in enumerate((self.cls_tower, self.reg_tower)):
                    conv = tw[i]
                    d = conv.fwd_desc(B, self._tower_segs(conv, B, shapes, off), ld_dst=FPN_C)
                    nn.conv_wgrad(d, towers[t][i], dAs[t], conv.dw)
            if paired and (i > 0 or pair0):
                dd = self.cls_tower[i].dgrad_desc(B, self._pair_segs(i, B, shapes, off, P, fwd=False), ld_dst=FPN_C)
                dst = torch.empty((2 * BP, FPN_C), dtype=self.store.act, device=dev)
                src_all = torch.as_strided(dAs[0], (2 * BP, FPN_C), (FPN_C, 1))
                nn.conv_igemm(dd, src_all, dst)
                if i == 0:          # both towers read F: dF = the two halves' sum (one 682-tile launch)
                    nn.add(dst[:BP], dst[BP:], dF)
                    dAs = [dF, dF]
                else:
                    dAs = [dst[:BP], dst[BP:]]
                continue
            nxt = []
            for t, tw in enumerate((self.cls_tower, self.reg_tower)):
                conv = tw[i]
                dd = conv.dgrad_desc(B, self._tower_segs(conv, B, shapes, off, wf=False), ld_dst=FPN_C,
                                     beta=(1.0 if (i == 0 and t == 1) else 0.0))
                dst = dF if i == 0 else torch.empty_like(F)
                nn.conv_igemm(dd, dAs[t], dst)
                nxt.append(dst)
            dAs = nxt
        hook("heads_towers")
        # ---- FPN backward (fcos.py:49-72) ----
        (C3, C4, C5) = s["C"]
        (c3, H3, W3), (c4, H4, W4), (c5, H5, W5) = C3, C4, C5
        l3, l4, l5 = s["l"]
        p3r, p4r = s["p"]
        h6, w6 = shapes[3]
        h7, w7 = shapes[4]
        # the FPN's weight gradients (3x3 outputs, 1x1 laterals): one batched call before the "fpn" hook
        # (layers.wgrad_batch: the laterals share a 256-wide launch, the stride-1 3x3 outputs a halo one)
        with wgrad_batch():
            # P7 = c7(relu(P6)): weights (relu on load), then d relu(P6) -> dP6 (masked, accumulated)
            d = self.c7_3x3.fwd_desc(B, [nn.seg(h7, w7, h6, w6, self.c7_3x3.wf, None, src_base=B * off[3],
                                                dst_base=B * off[4])], ld_dst=FPN_C, relu_in=True)
            wgrad_collect(d, F, dF, self.c7_3x3.dw)
            # bias gradients of the eight FPN convs: collected, then one batched launch pair
            bias_items = [(dF, FPN_C, 0, FPN_C, B * off[4], h7 * w7, h7 * w7, B, self.c7_3x3.db, 0.0)]
            dr6 = torch.empty((B, h6, w6, FPN_C), dtype=self.store.act, device=dev)
            dd = self.c7_3x3.dgrad_desc(B, [nn.seg(h6, w6, h7, w7, self.c7_3x3.wd, None, src_base=B * off[4])],
                                        ld_dst=FPN_C)
            nn.conv_igemm(dd, dF, dr6)
            dP6 = dF[B * off[3]:B * off[4]]
            P6 = F[B * off[3]:B * off[4]]
            nn.relu_backward(dr6, P6, dP6, beta=1.0)
            # c6 (stride 2 on C5), c5_3x3, c4_3x3, c3_3x3: weight/bias grads and data grads
            dC5 = torch.empty_like(c5)
            n3, n4 = p3r.numel() // FPN_C, p4r.numel() // FPN_C
            dPR = torch.empty_like(s["PR"])
            dp3r = dPR[:n3].view(p3r.shape)
            dp4r = dPR[n3:n3 + n4].view(p4r.shape)
            dl5 = dPR[n3 + n4:].view(l5.shape)
            pr_base = (0, n3, n3 + n4)
            trio = []
            for l, (conv, src, h, w, dsrc) in enumerate(((self.c3_3x3, p3r, H3, W3, dp3r),
                                                         (self.c4_3x3, p4r, H4, W4, dp4r),
                                                         (self.c5_3x3, l5, H5, W5, dl5),
                                                         (self.c6_3x3, c5, H5, W5, dC5))):
                Ho, Wo = shapes[l]
                d = conv.fwd_desc(B, [nn.seg(Ho, Wo, h, w, conv.wf, None, dst_base=B * off[l])], ld_dst=FPN_C)
                wgrad_collect(d, src, dF, conv.dw)
                bias_items.append((dF, FPN_C, 0, FPN_C, B * off[l], Ho * Wo, Ho * Wo, B, conv.db, 0.0))
                if FUSE_FPN and l < 3:            # P3..P5 data gradients: one 3-segment launch below
                    trio.append(nn.seg(h, w, Ho, Wo, conv.wd, None, src_base=B * off[l], dst_base=pr_base[l]))
                    continue
                dd = conv.dgrad_desc(B, [nn.seg(h, w, Ho, Wo, conv.wd, None, src_base=B * off[l])],
                                     ld_dst=conv.cin)
                nn.conv_igemm(dd, dF, dsrc)
            if trio:
                nn.conv_igemm(self.c3_3x3.dgrad_desc(B, trio, ld_dst=FPN_C), dF, dPR)
            # top-down adds: p4r = l4 + up(l5); p3r = l3 + up(l4)
            nn.upsample2x_backward(dp4r, dl5, B, H4, W4, FPN_C, beta=1.0)   # dl5 += up^T(dp4r)
            dl4 = dp4r
            nn.upsample2x_backward(dp3r, dl4, B, H3, W3, FPN_C, beta=1.0)   # dl4 += up^T(dp3r)
            dl3 = dp3r
            dC3 = torch.empty_like(c3)
            dC4 = torch.empty_like(c4)
            for conv, src, h, w, dl, dC, beta in ((self.c3_1x1, c3, H3, W3, dl3, dC3, 0.0),
                                                  (self.c4_1x1, c4, H4, W4, dl4, dC4, 0.0),
                                                  (self.c5_1x1, c5, H5, W5, dl5, dC5, 1.0)):
                conv.wgrad(src, dl, B, h, w, bias=False)
                bias_items.append((dl, FPN_C, 0, FPN_C, 0, h * w, h * w, B, conv.db, 0.0))
                conv.dgrad(dl, B, h, w, out=dC, beta=beta)
        nn.bias_grad_multi(bias_items)
        hook("fpn")
        self.backbone.backward([dC3, dC4, dC5], s["bsv"], hook=hook)
        self._saved = None
