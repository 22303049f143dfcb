"""ResNet-50 v1 backbone (the Keras `tf.keras.applications.ResNet50` graph tapped by
FCOS/fcos.py:30-46 and RetinaNet/retinanet_module.py:32-38), explicit forward/backward on the
cvlite kernels.  Keras layer names are kept (`conv1_conv`, `conv2_block1_0_conv`, ...).

Keras ResNet50 v1 structure (third-party, restated): ZeroPadding2D(3) -> conv1 7x7/2 (+bias)
-> BN -> ReLU -> ZeroPadding2D(1) -> MaxPool 3x3/2 -> stacks of bottleneck blocks
(filters 64/128/256/512, blocks 3/4/6/3, stride on the first 1x1 and on the projection
shortcut of each stack's first block, BN eps 1.001e-5) -> C3 = conv3_block4_out,
C4 = conv4_block6_out, C5 = conv5_block3_out.
"""
import os

import torch

from . import ops_nn as nn
from .layers import BF16, FUSE_SC_BNSUM, BatchNorm, Conv, ConvBN, StatsArena, wgrad_batch
from . import _lib

STEM_K = 7
# the stem's BN -> ReLU -> max-pool as one pass from z (CVL_DISPATCH=no_stem_pool_fuse: BN apply + pool)
FUSE_POOL = not _lib.dispatch("no_stem_pool_fuse")
# backward: the BN -> ReLU first pass inside the max-pool backward kernel (cvl_maxpool3x3s2_backward_bn_relu)
FUSE_POOL_BWD = not _lib.dispatch("no_stem_pool_bwd_fuse")
# projection shortcut's BN applied inside conv3's BN launch (CVL_DISPATCH=no_sc_bn_fuse: stored and re-read)
FUSE_SC_BN = not _lib.dispatch("no_sc_bn_fuse")
# a stage's last conv3 BN first pass formed by the next stage's strided conv1 data gradient: opt-in
# (CVL_DISPATCH=bnsum_res_s2) -- measured neutral to -0.1 % (the fused launch's 64-wide N tiles and
# three prefetched operands cost what the removed pass saved)
FUSE_BNSUM_RES_S2 = _lib.dispatch("bnsum_res_s2")
STEM_KP = 168            # the stem kernels' K: 7 kernel rows x (7 x 3 values padded to 24)


class Stem(object):
    """conv1_conv (7x7/2 after ZeroPadding2D(3)) straight from the image (cvl_stem_conv7x7s2 /
    cvl_stem_wgrad; round 4: 1.3 % faster per FCOS step than the im2col + GEMM form it replaced, whose
    403 MB patch matrix was written once and read twice), conv1_bn, ReLU, pool1."""

    def __init__(self, store):
        self.conv = Conv(store, "conv1_conv", STEM_K, 3, 64, stride=2, pad=3, bias=True, dgrad=False,
                         cin_k=STEM_KP)
        self.bn = BatchNorm(store, "conv1_bn", 64)

    def pack_entry(self):
        # HWIO [7][7][3][64] == [7][1][21][64]: packed as 7 "taps" (kernel rows) of 21 channels
        # (kx, c) padded to 24 -- the stem kernel's K order; fp32 parity mode: a direct 7x7/2 conv
        # over the 3 image channels
        c = self.conv
        if c.store.act != BF16:
            if c.wf is None:
                c.wf = torch.empty((64, 147), dtype=c.store.act, device=c.store.flat.device)
            return (c.w, 49, 3, 64, 3, 64, c.wf, 0, 0, None)
        if c.wf is None:
            c.wf = torch.empty((64, STEM_KP), dtype=BF16, device=c.store.flat.device)
        return (c.w, 7, 21, 64, 24, 64, c.wf, 0, 0, None)

    def _desc7(self, B, H, W, Ho, Wo):
        """fp32 parity mode: conv1 as a direct 7x7/2 conv (ZeroPadding2D(3) = explicit pad 3)."""
        return nn.make_desc(nn.FWD, B, 3, STEM_K, STEM_K, 2, 3, 3, 64, 64, 64,
                            [nn.seg(Ho, Wo, H, W, self.conv.wf, self.conv.b)])

    def pack(self):
        c = self.conv
        self.pack_entry()
        if c.store.act != BF16:
            nn.pack_conv_weights(c.w, 7, 7, 3, 64, 3, 64, c.wf)
        else:
            nn.pack_conv_weights(c.w, 7, 1, 21, 64, 24, 64, c.wf)

    def forward(self, x, train=True, arena=None):
        B, H, W, _ = x.shape
        Ho, Wo, pt, pl = self.conv.out_hw(H, W)
        act = self.conv.store.act
        stats = None
        if train:
            stats = arena.take(B, 64) if arena is not None else nn.bn_acc(B, 64, x.device)
        z = torch.empty((B, Ho, Wo, 64), dtype=act, device=x.device)
        A = x                                       # the fp32 image (the weight gradient reads it)
        if act == BF16:
            nn.stem_conv7x7s2(x, self.conv.wf, self.conv.b, z, stats)
        else:
            nn.conv_igemm(self._desc7(B, H, W, Ho, Wo), x, z, stats)
        Hp, Wp = (Ho + 2 - 3) // 2 + 1, (Wo + 2 - 3) // 2 + 1
        p = torch.empty((B, Hp, Wp, 64), dtype=act, device=x.device)
        arg = torch.empty((B, Hp, Wp, 64), dtype=torch.uint8, device=x.device)
        if act == BF16 and FUSE_POOL:
            # conv1_bn -> relu -> pool1 in one pass from z: the 256x256x64 BN output is never stored
            # (the backward rebuilds the ReLU mask from z and routes through argmax)
            if train:
                mr = torch.empty((B, 64, 2), dtype=torch.float32, device=x.device)
                nn.bn_finalize(stats, mr, self.bn.run_mean, self.bn.run_var, B, 64, Ho * Wo, self.bn.eps,
                               self.bn.momentum)
            else:
                mr = self.bn.moving_mean_rstd(B)
            nn.bn_relu_maxpool3x3s2(z, mr, self.bn.gamma, self.bn.beta, p, arg)
            return p, (A, z, None, mr, arg, B, Ho, Wo)
        y, mr = self.bn.normalize(z, stats, B, Ho * Wo, True, train=train)
        nn.maxpool3x3s2(y, p, arg)
        return p, (A, z, y, mr, arg, B, Ho, Wo)

    def backward(self, dp, saved):
        A, z, y, mr, arg, B, Ho, Wo = saved
        dz = torch.empty_like(z)
        st = self.bn.store
        dy = torch.empty_like(z)
        if z.dtype == BF16 and FUSE_POOL_BWD:
            nn.maxpool3x3s2_backward_bn_relu(dp, arg, z, mr, self.bn.gamma, self.bn.beta, dy, dz, st.g(self.bn.gname),
                                             st.g(self.bn.bname), conv_dbias=self.conv.db)
        else:
            nn.maxpool3x3s2_backward(dp, arg, dy)
            nn.bn_backward_relu(dy, z, mr, self.bn.gamma, self.bn.beta, dz, st.g(self.bn.gname),
                                st.g(self.bn.bname), B, Ho * Wo, 64, conv_dbias=self.conv.db)
        if z.dtype != BF16:                         # fp32 parity mode: 7x7 weight gradient in place
            nn.conv_wgrad(self._desc7(B, A.shape[1], A.shape[2], Ho, Wo), A, dz, self.conv.dw)
            return
        dw = torch.empty((192, 64), dtype=torch.float32, device=dp.device)    # rows ky*24 + kx*3 + c
        nn.stem_wgrad(A, dz, dw)
        nn.wgrad_flush()                             # dw is read right away (deferred reductions)
        self.conv.dw.view(7, 21, 64).copy_(dw.view(8, 24, 64)[:7, :21])


class Bottleneck(object):
    """Keras `block1` (resnet.py): [1x1/s -> BN -> ReLU] [3x3 -> BN -> ReLU] [1x1 -> BN] + shortcut -> ReLU."""

    def __init__(self, store, name, cin, filters, stride, conv_shortcut):
        self.sc = ConvBN(store, name + "_0", 1, cin, 4 * filters, stride) if conv_shortcut else None
        self.c1 = ConvBN(store, name + "_1", 1, cin, filters, stride)
        self.c2 = ConvBN(store, name + "_2", 3, filters, filters, 1)
        self.c3 = ConvBN(store, name + "_3", 1, filters, 4 * filters, 1)
        self.cout = 4 * filters

    def units(self):
        return [u for u in (self.sc, self.c1, self.c2, self.c3) if u is not None]

    def forward(self, x, B, H, W, train=True, arena=None):
        sv_s = s_bn = None
        s = x
        if self.sc is not None:
            # training, bf16: the shortcut's BN output is formed inside conv3's BN launch
            # (cvl_bn_finalize_apply_bnres) instead of being stored and re-read
            defer = train and FUSE_SC_BN and x.dtype == torch.bfloat16
            s, sv_s = self.sc.forward(x, B, H, W, relu=False, train=train, arena=arena, defer=defer)
            if defer:
                s_bn, s = s, None
        y1, sv1 = self.c1.forward(x, B, H, W, relu=True, train=train, arena=arena)
        H1, W1 = sv1[7], sv1[8]
        y2, sv2 = self.c2.forward(y1, B, H1, W1, relu=True, train=train, arena=arena)
        y3, sv3 = self.c3.forward(y2, B, H1, W1, relu=True, residual=s, train=train, arena=arena, residual_bn=s_bn)
        return y3, H1, W1, (sv_s, sv1, sv2, sv3)

    def backward(self, dy, saved, dx_out=None, dx_beta=0.0, arena=None, sums3=None, prev_ctx=None):
        """Returns (dx, sums of the previous block's conv3 BN or None).  sums3: this block's conv3 BN
        first pass, formed by the next block's conv1 data gradient (skipped here); prev_ctx: the
        previous block's conv3 bn_res_ctx -- this block's conv1 data gradient completes that unit's
        dy (the block-input gradient) and forms its first pass."""
        sv_s, sv1, sv2, sv3 = saved
        x = sv1[0]
        if dx_out is None:
            dx_out = torch.empty_like(x)
        if self.sc is None:
            assert dx_beta == 0.0, "identity blocks own their input gradient buffer"
            g = dx_out                     # residual gradient lands directly in dx
        else:
            g = torch.empty_like(dy)
        # conv1 / conv2 units (BN -> ReLU, one producer of their dy): the producing data gradient
        # also forms their BN backward's first pass (sums), so that pass is skipped
        ctx2, ctx1 = self.c2.bn_next_ctx(sv2, arena), self.c1.bn_next_ctx(sv1, arena)
        s2 = s1 = None
        # projection blocks: the shortcut BN's first pass rides on conv3's fused second pass
        sc_fuse = None
        if self.sc is not None and FUSE_SC_BNSUM and dy.dtype == torch.bfloat16:
            zs, mrs = sv_s[1], sv_s[3]
            sc_fuse = (zs, mrs, torch.empty((zs.shape[0], self.sc.bn.c, 2), dtype=torch.float64, device=zs.device))
        if ctx2 is not None:
            dy2, s2 = self.c3.backward(dy, sv3, g_out=g, bn_next=ctx2, sums=sums3, sc_fuse=sc_fuse)
        else:
            dy2 = self.c3.backward(dy, sv3, g_out=g, sums=sums3, sc_fuse=sc_fuse)
        sc_sums = sc_fuse[2] if (sc_fuse is not None and self.c3.sc_fused) else None
        if ctx1 is not None:
            dy1, s1 = self.c2.backward(dy2, sv2, sums=s2, bn_next=ctx1)
        else:
            dy1 = self.c2.backward(dy2, sv2, sums=s2)
        if self.sc is not None:
            self.sc.backward(g, sv_s, dx_out=dx_out, dx_beta=dx_beta, sums=sc_sums)
        if prev_ctx is not None:      # (stride 2: the scattered data gradient, cvl_conv_igemm_dgrad_bnsum_res)
            _, s_prev = self.c1.backward(dy1, sv1, dx_out=dx_out, dx_beta=1.0, sums=s1, bn_next=prev_ctx)
            return dx_out, s_prev
        self.c1.backward(dy1, sv1, dx_out=dx_out, dx_beta=1.0, sums=s1)
        return dx_out, None


# Keras applications ResNet v1 depths (block counts of conv2_x .. conv5_x); the detectors tap the
# last block of conv3_x / conv4_x / conv5_x (RetinaNet/retinanet_module.py:32-52:
# conv3_block4_out / conv4_block23_out for ResNet101, conv3_block8_out / conv4_block36_out for
# ResNet152; FCOS/fcos.py:30-35 for ResNet50)
DEPTHS = {"resnet50": (3, 4, 6, 3), "resnet101": (3, 4, 23, 3), "resnet152": (3, 8, 36, 3)}


class ResNet50(object):
    """Keras ResNet50 / ResNet101 / ResNet152 (v1 bottleneck stacks; `depth` picks the block
    counts, the class name is kept for the default)."""
    STACKS = ((64, 3, 1), (128, 4, 2), (256, 6, 2), (512, 3, 2))
    tap_channels = (512, 1024, 2048)

    def __init__(self, store, depth="resnet50"):
        blocks = DEPTHS[depth.lower()]
        self.STACKS = tuple((f, nb, st) for (f, _, st), nb in zip(ResNet50.STACKS, blocks))
        self.stem = Stem(store)
        self.stages = []
        cin = 64
        for si, (f, nb, stride) in enumerate(self.STACKS):
            stage = []
            for bi in range(nb):
                stage.append(Bottleneck(store, "conv%d_block%d" % (si + 2, bi + 1), cin, f,
                                        stride if bi == 0 else 1, bi == 0))
                cin = 4 * f
            self.stages.append(stage)

    def convs(self):
        out = [self.stem.conv]
        for st in self.stages:
            for b in st:
                out += [u.conv for u in b.units()]
        return out

    def bns(self):
        out = [self.stem.bn]
        for st in self.stages:
            for b in st:
                out += [u.bn for u in b.units()]
        return out

    def pack_entries(self):
        out = [self.stem.pack_entry()]
        for st in self.stages:
            for b in st:
                out += [u.conv.pack_entry() for u in b.units()]
        return out

    def pack(self):
        self.stem.pack()
        for st in self.stages:
            for b in st:
                for u in b.units():
                    u.conv.pack()

    def forward(self, x, train=True):
        """x: fp32 NHWC [B,H,W,3] in [-1,1].  Returns [C3, C4, C5] bf16 NHWC and saved state."""
        B = x.shape[0]
        # forward BN statistics + (second half) the backward's fused first-pass sums: one memset
        arena = StatsArena(4 * B * sum(bn.c for bn in self.bns()), x.device)
        h, sv_stem = self.stem.forward(x, train, arena)
        H, W = h.shape[1], h.shape[2]
        saved, taps = [], []
        for st in self.stages:
            ssv = []
            for b in st:
                h, H, W, sv = b.forward(h, B, H, W, train, arena)
                ssv.append(sv)
            saved.append(ssv)
            taps.append((h, H, W))
        return taps[1:], (sv_stem, saved, arena)

    def backward(self, d_taps, saved, hook=None):
        """d_taps: gradients of [C3, C4, C5]; they are used in place as stage-output buffers.
        hook(name) fires when a stage's parameter gradients are final ("conv5" .. "conv3", then
        "conv2_stem")."""
        hook = hook or (lambda name: None)
        sv_stem, ssv = saved[0], saved[1]
        arena = saved[2] if len(saved) > 2 else None
        dC = {1: d_taps[0], 2: d_taps[1], 3: d_taps[2]}
        dh = dC[3]
        pending = None              # the next-processed block's conv3 BN first pass, fused upstream
        for si in range(3, -1, -1):
            st = self.stages[si]
            # the stage's 1x1 weight gradients: one batched launch at the stage's end (layers.wgrad_batch)
            with wgrad_batch():
                for bi in range(len(st) - 1, -1, -1):
                    # the predecessor's conv3 BN first pass rides on this block's conv1 dgrad -- across
                    # a stage boundary too (a stage's first block: the strided, scattered data gradient
                    # that completes the previous stage's output gradient)
                    if bi >= 1:
                        prev = st[bi - 1].c3.bn_res_ctx(ssv[si][bi - 1][3], arena)
                    elif si >= 1 and FUSE_BNSUM_RES_S2:
                        prev = self.stages[si - 1][-1].c3.bn_res_ctx(ssv[si - 1][-1][3], arena)
                    else:
                        prev = None
                    if bi == 0 and (si - 1) in dC:
                        # this block's input is the previous stage's tap (C3 / C4), whose buffer
                        # already holds the FPN lateral's gradient: accumulate into it
                        dh, pending = st[bi].backward(dh, ssv[si][bi], dx_out=dC[si - 1], dx_beta=1.0, arena=arena,
                                                      sums3=pending, prev_ctx=prev)
                    else:
                        dh, pending = st[bi].backward(dh, ssv[si][bi], arena=arena, sums3=pending, prev_ctx=prev)
            if si > 0:
                hook("conv%d" % (si + 2))     # this stage's weight gradients are final
        self.stem.backward(dh, sv_stem)
        hook("conv2_stem")
