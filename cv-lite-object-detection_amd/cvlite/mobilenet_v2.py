"""Keras MobileNetV2 (alpha 1.0, tf.keras.applications.MobileNetV2(include_top=False)) as the
detectors use it (FCOS/fcos.py:36-41 — every backbone_model other than "resnet50" —,
RetinaNet/retinanet_module.py:67-71, CenterNet/tf_centernet.py:72-76, tf_centernet_resnet_s8.py:125-
129): the feature taps are the raw conv outputs `block_6_expand` (stride 8, 192 ch),
`block_13_expand` (stride 16, 576 ch) and `Conv_1` (stride 32, 1280 ch).  The layers after Conv_1
(Conv_1_bn, out_relu) feed no detector output, so they are not part of the trained model.

Graph: Conv1 (3x3/2 "same", 32) + BN + ReLU6; block 0 (depthwise 3x3 + BN + ReLU6, project 1x1 16
+ BN); blocks 1..16 (expand 1x1 x6 + BN + ReLU6, depthwise 3x3 stride s — ZeroPadding2D
(correct_pad) = pads (0, 1) + "valid" for s = 2 — + BN + ReLU6, project 1x1 + BN, residual add
when s = 1 and cin = cout); Conv_1 1x1 1280.  Convs have no bias; BN eps 1e-3, momentum 0.999,
training-mode statistics per image (the FCOS trainer forwards one image per BN group).

MI355X mapping: 1x1 convs on the MFMA implicit-GEMM kernels with the BN statistics fused into their
epilogue; depthwise convs on cvl_depthwise_* (HBM-bound 16-byte streams, deterministic weight
gradient); the stem as im2col (K = 27 -> 32) + one GEMM.  Maps whose channel count is not a
multiple of 32 (16, 24, 144) live with a zero-padded channel pitch cp(c); the parameters of those
layers are stored zero-padded to that pitch (kernels [.., cp(cin), cp(cout)], BN [cp(c)]): the
pads start at zero and receive exactly zero gradient, so they stay zero (Keras shapes = the
leading [cin, cout] block, `keras_view`).
"""
import math

import torch

from . import ops_nn as nn
from .layers import BF16, BatchNorm, Conv, StatsArena

BN_EPS, BN_MOM = 1e-3, 0.999
STEM_KP = 32
# (expansion t, output channels, stride) of blocks 0..16 (Keras MobileNetV2, alpha 1)
CFG = ((1, 16, 1), (6, 24, 2), (6, 24, 1), (6, 32, 2), (6, 32, 1), (6, 32, 1), (6, 64, 2), (6, 64, 1), (6, 64, 1),
       (6, 64, 1), (6, 96, 1), (6, 96, 1), (6, 96, 1), (6, 160, 2), (6, 160, 1), (6, 160, 1), (6, 320, 1))
TAP_CHANNELS = (192, 576, 1280)


def cp(c):
    return (c + 31) // 32 * 32


def padded_glorot(real_shape, fan_in, fan_out):
    """glorot_uniform over the real (Keras) block, zero in the channel pads."""
    lim = math.sqrt(6.0 / (fan_in + fan_out))

    def init(gen, shape):
        t = torch.zeros(shape, dtype=torch.float32)
        r = (torch.rand(real_shape, generator=gen, dtype=torch.float64) * 2 - 1).mul_(lim).float()
        t[tuple(slice(0, n) for n in real_shape)] = r
        return t
    return init


def _set_init(store, name, init):
    i = store.index[name]
    n, shape, _ = store.specs[i]
    store.specs[i] = (n, shape, init)


class PWUnit(object):
    """1x1 conv (no bias) -> BN [-> ReLU6] on channel-padded maps."""

    def __init__(self, store, name, bn_name, cin, cout, relu6, with_bn=True):
        self.cin, self.cout, self.relu6 = cin, cout, relu6
        self.ci, self.co = cp(cin), cp(cout)
        self.conv = Conv(store, name, 1, self.ci, self.co, bias=False)
        _set_init(store, self.conv.wname, padded_glorot((1, 1, cin, cout), cin, cout))
        self.bn = BatchNorm(store, bn_name, self.co, eps=BN_EPS, momentum=BN_MOM) if with_bn else None

    def desc(self, B, H, W):
        c = self.conv
        return c.fwd_desc(B, [nn.seg(H, W, H, W, c.wf, None)], ld_dst=self.co, n_store=self.co)

    def forward(self, x, B, H, W, train, arena, residual=None):
        stats = arena.take(B, self.co) if (train and self.bn is not None) else None
        z = torch.empty((B, H, W, self.co), dtype=BF16, device=x.device)
        nn.conv_igemm(self.desc(B, H, W), x, z, stats)
        if self.bn is None:
            return z, z, (x, z, None, None, B, H, W)
        y, mr = self.bn.normalize(z, stats, B, H * W, 2 if self.relu6 else 0, residual=residual, train=train)
        return z, y, (x, z, y, mr, B, H, W)

    def backward(self, dy, saved, dx_out=None, dx_beta=0.0, d_tap=None):
        """dy: grad of the unit output (BN output / ReLU6 output); d_tap: extra gradient of the raw
        conv output z (a feature tap).  Returns dx (written / accumulated into dx_out)."""
        x, z, y, mr, B, H, W = saved
        st = self.conv.store
        if self.bn is not None:
            dz = torch.empty_like(z)
            if self.relu6:
                nn.bn_backward_relu6(dy, z, mr, self.bn.gamma, self.bn.beta, dz, st.g(self.bn.gname),
                                     st.g(self.bn.bname), B, H * W, self.co)
            else:
                nn.bn_backward(dy, None, z, mr, self.bn.gamma, dz, None, st.g(self.bn.gname), st.g(self.bn.bname),
                               B, H * W, self.co)
            if d_tap is not None:
                nn.add(dz, d_tap, dz)
        else:
            dz = d_tap if d_tap is not None else dy
        c = self.conv
        nn.conv_wgrad(self.desc(B, H, W), x, dz, c.dw)
        if dx_out is None:
            dx_out = torch.empty((B, H, W, self.ci), dtype=BF16, device=dz.device)
            dx_beta = 0.0
        d = nn.make_desc(nn.DGRAD, B, self.co, 1, 1, 1, 0, 0, self.ci, self.ci, self.ci,
                         [nn.seg(H, W, H, W, c.wd, None)], beta=dx_beta)
        nn.conv_igemm(d, dz, dx_out)
        return dx_out


class DWUnit(object):
    """DepthwiseConv2D(3, stride, use_bias=False) -> BN -> ReLU6 (channel-padded)."""

    def __init__(self, store, name, c, stride):
        self.c, self.stride = c, stride
        self.cc = cp(c)
        self.wname = store.add(name + "/depthwise_kernel", (3, 3, self.cc, 1), padded_glorot((3, 3, c, 1), 9 * c, 9))
        self.bn = BatchNorm(store, name + "_BN", self.cc, eps=BN_EPS, momentum=BN_MOM)
        self.store = store

    def geo(self, H, W):
        if self.stride == 1:
            return H, W, 1, 1
        return (H - 2) // 2 + 1, (W - 2) // 2 + 1, 0, 0         # ZeroPadding2D((0, 1), (0, 1)) + "valid"

    def forward(self, x, B, H, W, train, arena):
        Ho, Wo, pt, pl = self.geo(H, W)
        z = torch.empty((B, Ho, Wo, self.cc), dtype=BF16, device=x.device)
        nn.depthwise_fwd(x, self.store.p(self.wname), z, 3, self.stride, pt, pl)
        if train:
            stats = arena.take(B, self.cc)
            nn.bn_stats(z, B, Ho * Wo, self.cc, stats)
        else:
            stats = None
        y, mr = self.bn.normalize(z, stats, B, Ho * Wo, 2, train=train)
        return y, Ho, Wo, (x, z, y, mr, B, H, W, Ho, Wo)

    def backward(self, dy, saved):
        x, z, y, mr, B, H, W, Ho, Wo = saved
        st = self.store
        dz = torch.empty_like(z)
        nn.bn_backward_relu6(dy, z, mr, self.bn.gamma, self.bn.beta, dz, st.g(self.bn.gname), st.g(self.bn.bname), B,
                             Ho * Wo, self.cc)
        _, _, pt, pl = self.geo(H, W)
        nn.depthwise_wgrad(x, dz, st.g(self.wname), 3, self.stride, pt, pl)
        dx = torch.empty_like(x)
        nn.depthwise_dgrad(dz, st.p(self.wname), dx, 3, self.stride, pt, pl)
        return dx


class InvertedResidual(object):
    def __init__(self, store, bid, cin, t, cout, stride):
        pre = "expanded_conv_" if bid == 0 else "block_%d_" % bid
        mid = cin * t
        self.expand = PWUnit(store, pre + "expand", pre + "expand_BN", cin, mid, True) if t != 1 else None
        self.dw = DWUnit(store, pre + "depthwise", mid, stride)
        self.project = PWUnit(store, pre + "project", pre + "project_BN", mid, cout, False)
        self.residual = stride == 1 and cin == cout
        self.cin, self.cout = cin, cout

    def units(self):
        return [u for u in (self.expand, self.project) if u is not None]

    def bns(self):
        return [u.bn for u in self.units()] + [self.dw.bn]

    def forward(self, x, B, H, W, train, arena):
        sv = {}
        h = x
        tap = None
        if self.expand is not None:
            tap, h, sv["e"] = self.expand.forward(x, B, H, W, train, arena)
        h, Ho, Wo, sv["d"] = self.dw.forward(h, B, H, W, train, arena)
        _, y, sv["p"] = self.project.forward(h, B, Ho, Wo, train, arena, residual=x if self.residual else None)
        return y, Ho, Wo, tap, sv

    def backward(self, dy, sv, d_tap=None):
        dh = self.project.backward(dy, sv["p"])
        dh = self.dw.backward(dh, sv["d"])
        if self.expand is not None:
            if self.residual:
                return self.expand.backward(dh, sv["e"], dx_out=dy, dx_beta=1.0, d_tap=d_tap)   # + skip
            return self.expand.backward(dh, sv["e"], d_tap=d_tap)
        return dh


class MobileNetV2(object):
    """Backbone up to the Conv_1 tap.  forward(x) -> ([(C3, H3, W3), (C4, ..), (C5, ..)], saved)
    with C3 = block_6_expand, C4 = block_13_expand, C5 = Conv_1 raw conv outputs (bf16 NHWC)."""
    tap_channels = TAP_CHANNELS

    def __init__(self, store):
        self.store = store
        self.stem_wname = store.add("Conv1/kernel", (3, 3, 3, 32), padded_glorot((3, 3, 3, 32), 27, 9 * 32))
        self.stem_bn = BatchNorm(store, "bn_Conv1", 32, eps=BN_EPS, momentum=BN_MOM)
        self.blocks = []
        cin = 32
        for bid, (t, c, s) in enumerate(CFG):
            self.blocks.append(InvertedResidual(store, bid, cin, t, c, s))
            cin = c
        self.head = PWUnit(store, "Conv_1", None, 320, 1280, None, with_bn=False)
        self.stem_wf = None

    # ---- parameters -----------------------------------------------------------------------------
    def convs(self):
        return [None] + [u.conv for b in self.blocks for u in b.units()] + [self.head.conv]

    def bns(self):
        return [self.stem_bn] + [bn for b in self.blocks for bn in b.bns()]

    def pack_entries(self):
        if self.stem_wf is None:
            self.stem_wf = torch.empty((32, STEM_KP), dtype=BF16, device=self.store.flat.device)
        w = self.store.p(self.stem_wname)
        out = [(w, 1, 27, 32, STEM_KP, 32, self.stem_wf, 0, 0, None)]
        for c in self.convs()[1:]:
            out.append(c.pack_entry())
        return out

    def param_names(self):
        return list(n for n in self.store.offsets if self._mine(n))

    def _mine(self, n):
        return n.startswith(("Conv1/", "bn_Conv1/", "expanded_conv_", "block_", "Conv_1/"))

    # ---- forward / backward -----------------------------------------------------------------------
    def _stem_desc(self, B, Ho, Wo):
        return nn.make_desc(nn.FWD, B, STEM_KP, 1, 1, 1, 0, 0, 32, 32, 32, [nn.seg(Ho, Wo, Ho, Wo, self.stem_wf, None)])

    def forward(self, x, train=True):
        B, H, W, _ = x.shape
        arena = StatsArena(2 * B * sum(bn.c for bn in self.bns()), x.device) if train else None
        Ho, Wo = -(-H // 2), -(-W // 2)
        pt = max((Ho - 1) * 2 + 3 - H, 0) // 2
        pl = max((Wo - 1) * 2 + 3 - W, 0) // 2
        A = torch.empty((B * Ho * Wo, STEM_KP), dtype=BF16, device=x.device)
        nn.im2col(x, 3, 3, 2, pt, pl, Ho, Wo, STEM_KP, A)
        stats = arena.take(B, 32) if train else None
        z = torch.empty((B, Ho, Wo, 32), dtype=BF16, device=x.device)
        nn.conv_igemm(self._stem_desc(B, Ho, Wo), A, z, stats)
        h, mr = self.stem_bn.normalize(z, stats, B, Ho * Wo, 2, train=train)
        sv_stem = (A, z, h, mr, B, Ho, Wo)
        H, W = Ho, Wo
        taps, saved = [], []
        for bid, blk in enumerate(self.blocks):
            h, H2, W2, tap, sv = blk.forward(h, B, H, W, train, arena)
            saved.append(sv)
            if bid in (6, 13):
                taps.append((tap, H, W))                 # block_6_expand / block_13_expand (input size)
            H, W = H2, W2
        c5, _, svh = self.head.forward(h, B, H, W, train, arena)
        taps.append((c5, H, W))
        return taps, (sv_stem, saved, svh)

    def backward(self, d_taps, saved, hook=None):
        """d_taps: gradients of the three raw tap outputs."""
        sv_stem, saved, svh = saved
        dh = self.head.backward(None, svh, d_tap=d_taps[2])
        for bid in range(len(self.blocks) - 1, -1, -1):
            dt = {6: d_taps[0], 13: d_taps[1]}.get(bid)
            dh = self.blocks[bid].backward(dh, saved[bid], d_tap=dt)
        A, z, h, mr, B, Ho, Wo = sv_stem
        st = self.store
        dz = torch.empty_like(z)
        nn.bn_backward_relu6(dh, z, mr, self.stem_bn.gamma, self.stem_bn.beta, dz, st.g(self.stem_bn.gname),
                             st.g(self.stem_bn.bname), B, Ho * Wo, 32)
        dw = torch.empty((STEM_KP, 32), dtype=torch.float32, device=dz.device)
        nn.conv_wgrad(self._stem_desc(B, Ho, Wo), A, dz, dw)
        nn.wgrad_flush()                             # dw is read right away (deferred reductions)
        st.g(self.stem_wname).view(27, 32).copy_(dw[:27])
        if hook is not None:
            hook("backbone")
