"""CenterNet hourglass (CenterNet/tf_centernet_hourglass.py:87-353: build_model(n_classes, tmp_pi,
n_filters, n_stacks, n_repeats, seperable, batch_norm, norm_order); the reference defaults are
n_filters=128, n_stacks=1, n_repeats=2, seperable=True, batch_norm=True, norm_order="norm_first")
as an explicit forward/backward graph on the cvlite MFMA conv and HIP memory-bound kernels.
Every build option is supported: stacked hourglasses (the output of stack s is the input of
stack s + 1), Conv2D instead of SeparableConv2D (seperable=False), no BatchNormalization, and
norm_last (BN on each repeat's 2nf-channel output, before its ReLU).

MI355X mapping:
  * every SeparableConv2D (depthwise D, no bias; pointwise P + bias) runs as ONE dense conv on the
    implicit-GEMM MFMA kernels with the folded kernel W = D x P (exact for 1x1 — a per-channel
    scale of the GEMM's K rows — and a rank-structured 3x3 / 7x7 kernel otherwise); the fold and
    the gradient unfold of all 91 separable convs are one launch each (cvl_sep_fold_multi /
    cvl_sep_unfold_multi), the fold feeding the batched bf16 re-pack;
  * the 7x7/2 stem (3 channels) is im2col + one K=160 GEMM, like the ResNet stem;
  * BatchNorm statistics span a sub-batch of `group` images (one Keras forward per sub-batch in
    train_step :527-545), computed by a deterministic column-sum kernel;
  * the bilinear x2 up-sampling is fused with the decoder's skip add;
  * b_focal (tf_bias_layer.py) is folded into the output conv's bias.
Keras names are kept: `cnn_block_0`, `<blk>_bn_<r>`, `<blk>_{bot,cnn,out}_<r>`
(`/depthwise_kernel`, `/pointwise_kernel`, `/bias`), `cnn_out`, `b_focal`.
Reference quirk kept (cnn_block :103-155): from the second repeat on the residual adds the BN
OUTPUT (`tmp_input` is rebound to the normalised tensor before the convs).
"""
import math
import os

import torch

from . import ops_nn as nn
from .layers import BF16, BatchNorm, Conv, ParamStore, constant, glorot_uniform
from . import _lib

STEM_K = 7
STEM_KP = 160          # im2col K = 7*7*3 = 147 padded to a multiple of 32
BN_EPS = 1e-3          # Keras BatchNormalization default (the hourglass passes no epsilon)
BN_MOMENTUM = 0.99


def skey(s, name):
    """Key of a per-stack tensor (stack s, 1-based) in the forward / backward value maps."""
    return "%d:%s" % (s, name)


def block_graph(n_stacks=1):
    """(name, input, output) of every cnn_block in graph order (tf_centernet_hourglass.py:189-333);
    the tensors of stack s are keyed skey(s, ...)."""
    out = [("cnn_block_1", "blk0", "cnn1")]
    for s in range(1, n_stacks + 1):
        st = "stack_%d_" % s
        k = lambda n: skey(s, n)   # noqa: E731
        out += [(st + "enc_block_1", k("stack_in"), k("enc1")), (st + "enc_block_2", k("e1"), k("enc2")),
                (st + "enc_block_3", k("e2"), k("enc3")), (st + "enc_block_4a", k("e3"), k("enc4a")),
                (st + "enc_block_4b", k("enc4a"), k("enc4b")), (st + "enc_block_4", k("enc4b"), k("enc4")),
                (st + "dec_block_1", k("e3"), k("dec1")), (st + "dec_out_1", k("d1res"), k("o1")),
                (st + "dec_block_2", k("e2"), k("dec2")), (st + "dec_out_2", k("d2res"), k("o2")),
                (st + "dec_block_3", k("e1"), k("dec3")), (st + "dec_out_3", k("d3res"), k("o3")),
                (st + "dec_block_4", k("stack_in"), k("dec4")), (st + "dec_out_4", k("d4res"), k("o4"))]
    return out


# 3x3 separable convs on maps of at least this many pixels run SPLIT: depthwise kernel
# (cvl_depthwise_*, HBM-bound) + pointwise 1x1 GEMM, instead of the dense fold whose 3x3 GEMM does
# 9x the pointwise FLOPs; below it the fold's single launch wins (CVL_DISPATCH=sep_split_min_hw=<n>, 0 = never)
SPLIT_MIN_HW = _lib.dispatch("sep_split_min_hw", 128 * 128)


class _PointwiseOf(Conv):
    """The pointwise half of a split SeparableConv2D as a 1x1 Conv whose weight IS the layer's
    trainable pointwise_kernel [1,1,Cin,Cout] (HWIO of a 1x1 conv): packing reads it and the
    weight gradient lands in its gradient slot, with no fold / unfold."""

    def __init__(self, store, pwname, cin, cout):
        self.name, self.k, self.cin, self.cout, self.stride, self.pad = pwname, 1, cin, cout, 1, "same"
        self.cin_k = cin
        self.npad = max(32, (cout + 31) // 32 * 32)
        self.cout_pad = self.npad
        self.cin_pad = (cin + 31) // 32 * 32
        self.has_bias = False
        self.need_dgrad = True
        self.wname, self.bname = pwname, None
        self.store = store
        self.wf = self.wd = None


class SepConv(object):
    """Keras SeparableConv2D(cout, k, stride, "same") = dense conv with the folded kernel D x P.
    The trainable D / P / bias live in the model store; the folded kernel and its gradient in
    the `eff` store (not optimised).  3x3 / stride 1 convs on large maps run split instead
    (depthwise kernel on D + 1x1 GEMM on P, gradients written straight to D / P): `split` is
    decided on the first forward at a map size and fixes which of the two forms the model's
    fold / pack plans carry."""

    def __init__(self, store, eff, name, k, cin, cout, stride=1, cin_k=None, dgrad=True):
        self.name, self.k, self.cin, self.cout = name, k, cin, cout
        self.dwname = store.add(name + "/depthwise_kernel", (k, k, cin, 1), glorot_uniform(k * k * cin, k * k))
        self.pwname = store.add(name + "/pointwise_kernel", (1, 1, cin, cout), glorot_uniform(cin, cout))
        self.bname = store.add(name + "/bias", (cout,), constant(0.0))
        self.store = store
        self.conv = Conv(eff, name, k, cin, cout, stride, "same", bias=False, cin_k=cin_k, dgrad=dgrad)
        self.can_split = k == 3 and stride == 1 and cin % 8 == 0
        self.split = False
        self.pw = _PointwiseOf(store, self.pwname, cin, cout) if self.can_split else None
        self.on_mode_change = None         # the owning net's plan invalidation
        self.bias_sink = None              # the owning net's deferred bias-gradient list
        self._t = self._dt = None

    def want_split(self, H, W):
        return self.can_split and 0 < SPLIT_MIN_HW <= H * W

    @property
    def b(self):
        return self.store.p(self.bname)

    @property
    def db(self):
        return self.store.g(self.bname)

    def sep_entry(self):
        st = self.store
        return (st.p(self.dwname), st.p(self.pwname), self.conv.w, self.conv.dw, st.g(self.dwname),
                st.g(self.pwname))

    def _set_split(self, on):
        if on != self.split:
            self.split = on
            if on:
                self.pw.pack()                  # eager: the plans pick the pointwise up from now on
            if self.on_mode_change is not None:
                self.on_mode_change()

    def fwd(self, x, B, H, W, relu_out=False):
        self._set_split(self.want_split(H, W))
        if self.split:
            # depthwise (TF "same" 3x3: pad 1) then the pointwise GEMM with the layer's bias
            t = torch.empty((B, H, W, self.cin), dtype=BF16, device=x.device)
            nn.depthwise_fwd(x, self.store.p(self.dwname), t, 3, 1, 1, 1)
            self._t = t
            out = torch.empty((B, H, W, self.cout), dtype=BF16, device=x.device)
            d = self.pw.fwd_desc(B, [nn.seg(H, W, H, W, self.pw.wf, self.b)], ld_dst=self.cout, relu_out=relu_out)
            nn.conv_igemm(d, t, out)
            return out
        c = self.conv
        Ho, Wo, _, _ = c.out_hw(H, W)
        out = torch.empty((B, Ho, Wo, self.cout), dtype=BF16, device=x.device)
        d = c.fwd_desc(B, [nn.seg(Ho, Wo, H, W, c.wf, self.b)], ld_dst=self.cout, relu_out=relu_out)
        nn.conv_igemm(d, x, out)
        return out

    def wgrad(self, x, dy, B, H, W):
        HW = H * W
        if self.split:
            # dP = t^T dy; dt = dy P^T (kept for dgrad); dD = depthwise weight gradient of (x, dt)
            self.pw.wgrad(self._t, dy, B, H, W, bias=False)
            self._dt = self.pw.dgrad(dy, B, H, W)
            nn.depthwise_wgrad(x, self._dt, self.store.g(self.dwname), 3, 1, 1, 1)
        else:
            self.conv.wgrad(x, dy, B, H, W, bias=False)
        item = (dy, int(dy.shape[-1]), 0, self.cout, 0, HW, HW, B, self.db, 0.0)
        if self.bias_sink is not None:      # batched at the end of the net's backward
            self.bias_sink.append(item)
        else:
            nn.bias_grad(*item[:9])

    def dgrad(self, dy, B, H, W, out=None, beta=0.0):
        if self.split:
            assert self._dt is not None, "split SepConv: wgrad (which forms dt) runs before dgrad"
            if out is None:
                out = torch.empty((B, H, W, self.cin), dtype=BF16, device=dy.device)
            nn.depthwise_dgrad(self._dt, self.store.p(self.dwname), out, 3, 1, 1, 1, beta=beta)
            return out
        return self.conv.dgrad(dy, B, H, W, out=out, beta=beta)


class DenseConv(object):
    """Keras Conv2D(cout, k, stride, "same") with bias (build_model(seperable=False), :124-136,
    :174-182) behind SepConv's interface: the trainable HWIO kernel is packed directly."""
    split = False
    can_split = False

    def __init__(self, store, name, k, cin, cout, stride=1, cin_k=None, dgrad=True):
        self.name, self.k, self.cin, self.cout = name, k, cin, cout
        self.conv = Conv(store, name, k, cin, cout, stride, "same", bias=True, cin_k=cin_k, dgrad=dgrad)
        self.store = store
        self.on_mode_change = None
        self.bias_sink = None

    @property
    def b(self):
        return self.conv.b

    @property
    def db(self):
        return self.conv.db

    def fwd(self, x, B, H, W, relu_out=False):
        c = self.conv
        Ho, Wo, _, _ = c.out_hw(H, W)
        out = torch.empty((B, Ho, Wo, self.cout), dtype=BF16, device=x.device)
        d = c.fwd_desc(B, [nn.seg(Ho, Wo, H, W, c.wf, self.b)], ld_dst=self.cout, relu_out=relu_out)
        nn.conv_igemm(d, x, out)
        return out

    def wgrad(self, x, dy, B, H, W):
        self.conv.wgrad(x, dy, B, H, W, bias=False)
        HW = H * W
        item = (dy, int(dy.shape[-1]), 0, self.cout, 0, HW, HW, B, self.db, 0.0)
        if self.bias_sink is not None:
            self.bias_sink.append(item)
        else:
            nn.bias_grad(*item[:9])

    def dgrad(self, dy, B, H, W, out=None, beta=0.0):
        return self.conv.dgrad(dy, B, H, W, out=out, beta=beta)


def make_conv(seperable, store, eff, name, k, cin, cout, stride=1, cin_k=None, dgrad=True):
    if seperable:
        return SepConv(store, eff, name, k, cin, cout, stride=stride, cin_k=cin_k, dgrad=dgrad)
    return DenseConv(store, name, k, cin, cout, stride=stride, cin_k=cin_k, dgrad=dgrad)


class Stem(object):
    """cnn_block_0: SeparableConv2D (or Conv2D) (n_filters, 7x7, stride 2, "same") on the 3-channel
    image as im2col (TF-same pads) + one K=160 GEMM with the (folded) kernel [7][7][3][nf]."""

    def __init__(self, store, eff, nf, seperable=True):
        self.sep = make_conv(seperable, store, eff, "cnn_block_0", STEM_K, 3, nf, stride=2, cin_k=STEM_KP,
                             dgrad=False)
        self.nf = nf

    def pack_entry(self):
        c = self.sep.conv
        if c.wf is None:
            c.wf = torch.empty((self.nf, STEM_KP), dtype=BF16, device=c.store.flat.device)
        return (c.w, 1, 147, self.nf, STEM_KP, self.nf, c.wf, 0, 0, None)

    def _desc(self, B, Ho, Wo):
        return nn.make_desc(nn.FWD, B, STEM_KP, 1, 1, 1, 0, 0, self.nf, self.nf, self.nf,
                            [nn.seg(Ho, Wo, Ho, Wo, self.sep.conv.wf, self.sep.b)])

    def forward(self, x):
        B, H, W, _ = x.shape
        Ho, Wo, pt, pl = self.sep.conv.out_hw(H, W)
        A = torch.empty((B * Ho * Wo, STEM_KP), dtype=BF16, device=x.device)
        nn.im2col(x, STEM_K, STEM_K, 2, pt, pl, Ho, Wo, STEM_KP, A)
        z = torch.empty((B, Ho, Wo, self.nf), dtype=BF16, device=x.device)
        nn.conv_igemm(self._desc(B, Ho, Wo), A, z)
        return z, (A, B, Ho, Wo)

    def backward(self, dz, saved):
        A, B, Ho, Wo = saved
        dw = torch.empty((STEM_KP, self.nf), dtype=torch.float32, device=dz.device)
        nn.conv_wgrad(self._desc(B, Ho, Wo), A, dz, dw)
        nn.wgrad_flush()                             # dw is read right away (deferred reductions)
        self.sep.conv.dw.view(147, self.nf).copy_(dw[:147])
        HW = Ho * Wo
        nn.bias_grad(dz, self.nf, 0, self.nf, 0, HW, HW, B, self.sep.db)


class Repeat(object):
    """One cnn_block repeat (tf_centernet_hourglass.py:96-155): norm_first: BN -> conv 1x1 (nf) ->
    conv 3x3 (nf) -> conv 1x1 (2nf) -> ReLU, residual (r >= 1) adds the BN OUTPUT (the input is
    rebound to it); norm_last: conv 1x1 -> 3x3 -> 1x1 -> BN -> ReLU, residual adds the input;
    batch_norm=False drops the BN; the convs are SeparableConv2D or Conv2D (seperable)."""

    def __init__(self, store, eff, blk, r, cin, nf, seperable=True, batch_norm=True, norm_order="norm_first"):
        if norm_order not in ("norm_first", "norm_last"):
            raise ValueError("norm_order must be 'norm_first' or 'norm_last'")
        self.r = r
        self.norm_first = norm_order == "norm_first"
        self.bn = (BatchNorm(store, "%s_bn_%d" % (blk, r), cin if self.norm_first else 2 * nf, eps=BN_EPS,
                             momentum=BN_MOMENTUM) if batch_norm else None)
        self.bot = make_conv(seperable, store, eff, "%s_bot_%d" % (blk, r), 1, cin, nf)
        self.cnn = make_conv(seperable, store, eff, "%s_cnn_%d" % (blk, r), 3, nf, nf)
        self.out = make_conv(seperable, store, eff, "%s_out_%d" % (blk, r), 1, nf, 2 * nf)
        self.cin, self.cout = cin, 2 * nf

    def seps(self):
        return [self.bot, self.cnn, self.out]

    def _bn(self, t, B, HW, group, train, relu):
        c, bn = self.bn.c, self.bn
        mr = torch.empty((B, c, 2), dtype=torch.float32, device=t.device)
        if train:
            stats = nn.bn_acc(B, c, t.device, zero=False)
            nn.bn_stats(t, B, HW, c, stats)
            nn.bn_finalize_grouped(stats, mr, bn.run_mean, bn.run_var, B, c, HW, group, bn.eps, bn.momentum)
        else:                                     # Keras inference: moving statistics
            mr[:, :, 0] = bn.run_mean
            mr[:, :, 1] = torch.rsqrt(bn.run_var + bn.eps)
        a = torch.empty_like(t)
        nn.bn_apply(t, mr, bn.gamma, bn.beta, None, a, B, HW, c, relu)
        return a, mr

    def forward(self, t, B, H, W, group, train=True):
        HW = H * W
        mr = z = None
        a = t
        if self.bn is not None and self.norm_first:
            a, mr = self._bn(t, B, HW, group, train, False)
        u = self.bot.fwd(a, B, H, W)
        v = self.cnn.fwd(u, B, H, W)
        if self.bn is not None and not self.norm_first:
            z = self.out.fwd(v, B, H, W)
            y, mr = self._bn(z, B, HW, group, train, True)
        else:
            y = self.out.fwd(v, B, H, W, relu_out=True)
        if self.r == 0:
            o = y
        else:
            o = torch.empty_like(y)
            nn.add(y, a, o)
        return o, (t, mr, a, u, v, z, y, B, H, W, group)

    def backward(self, dout, saved, dx_out, dx_beta=0.0):
        """dout: grad of this repeat's output (clobbered when r >= 1: it becomes the residual
        addend's gradient); writes / accumulates (dx_beta) the grad of its input into dx_out."""
        t, mr, a, u, v, z, y, B, H, W, group = saved
        st = self.store_of()
        dz3 = torch.empty_like(y)
        if z is not None:                          # norm_last: ReLU -> BN backward onto the conv output
            nn.bn_backward_grouped(dout, z, mr, self.bn.gamma, dz3, st.g(self.bn.gname), st.g(self.bn.bname),
                                   B, H * W, self.cout, group, y_relu=y)
        else:
            nn.relu_backward(dout, y, dz3)
        self.out.wgrad(v, dz3, B, H, W)
        dv = self.out.dgrad(dz3, B, H, W)
        self.cnn.wgrad(u, dv, B, H, W)
        du = self.cnn.dgrad(dv, B, H, W)
        self.bot.wgrad(a, du, B, H, W)
        if self.bn is not None and self.norm_first:
            if self.r == 0:
                da = self.bot.dgrad(du, B, H, W)
            else:
                da = self.bot.dgrad(du, B, H, W, out=dout, beta=1.0)     # + residual branch (BN output)
            nn.bn_backward_grouped(da, t, mr, self.bn.gamma, dx_out, st.g(self.bn.gname), st.g(self.bn.bname),
                                   B, H * W, self.cin, group, dz_beta=dx_beta)
        elif self.r == 0:
            self.bot.dgrad(du, B, H, W, out=dx_out, beta=dx_beta)
        else:                                     # residual adds the input itself
            da = self.bot.dgrad(du, B, H, W, out=dout, beta=1.0)
            if dx_beta:
                nn.add(dx_out, da, dx_out)
            else:
                dx_out.copy_(da)
        return dx_out

    def store_of(self):
        return self.bot.store


class CnnBlock(object):
    def __init__(self, store, eff, name, cin, nf, n_repeats, **opts):
        self.name = name
        self.reps = []
        c = cin
        for r in range(n_repeats):
            self.reps.append(Repeat(store, eff, name, r, c, nf, **opts))
            c = 2 * nf
        self.cout = c

    def seps(self):
        return [s for r in self.reps for s in r.seps()]

    def bns(self):
        return [r.bn for r in self.reps if r.bn is not None]

    def forward(self, x, B, H, W, group, train=True):
        h, saved = x, []
        for rep in self.reps:
            h, sv = rep.forward(h, B, H, W, group, train)
            saved.append(sv)
        return h, saved

    def backward(self, dy, saved, dx_out, dx_beta=0.0):
        """dy is clobbered; the block-input gradient is written/accumulated into dx_out."""
        g = dy
        for i in range(len(self.reps) - 1, -1, -1):
            tgt = dx_out if i == 0 else torch.empty_like(saved[i][0])
            self.reps[i].backward(g, saved[i], tgt, dx_beta if i == 0 else 0.0)
            g = tgt
        return dx_out


class HourglassNet(object):
    """tf_centernet_hourglass.build_model(n_classes, tmp_pi, n_filters, n_stacks, n_repeats) on
    MI355X.  forward(x [B,H,W,3] fp32) -> [B,H/4,W/4,4+C] fp32; backward(d_out bf16)."""

    def __init__(self, n_classes, tmp_pi=0.99, n_filters=128, n_stacks=1, n_repeats=2, device="cuda", seed=0,
                 seperable=True, batch_norm=True, norm_order="norm_first"):
        self.C = n_classes
        self.nf = n_filters
        self.n_stacks = n_stacks
        self.device = torch.device(device)
        store, eff = ParamStore(), ParamStore()
        self._build(store, eff, n_classes, tmp_pi, n_filters, n_stacks, n_repeats,
                    dict(seperable=seperable, batch_norm=batch_norm, norm_order=norm_order))
        store.finalize(self.device, seed)
        eff.finalize(self.device, seed + 1)
        self.store, self.eff = store, eff
        for bn in self.bns():
            bn.init_buffers(self.device)
        for s in self.seps():
            s.on_mode_change = self._mode_changed
        self.cout_ld = (4 + n_classes + 31) // 32 * 32
        self.b_eff = torch.zeros(4 + n_classes, dtype=torch.float32, device=self.device)
        self.g_beff = torch.zeros(4 + n_classes, dtype=torch.float32, device=self.device)
        self._plan = None
        self.pack()

    def _build(self, store, eff, C, tmp_pi, nf, n_stacks, n_repeats, opts=None):
        opts = opts or {}
        self.stem = Stem(store, eff, nf, opts.get("seperable", True))
        self.blocks = {}
        for name, i, o in block_graph(n_stacks):       # only cnn_block_1 sees the stem's nf channels
            self.blocks[name] = CnnBlock(store, eff, name, nf if i == "blk0" else 2 * nf, nf, n_repeats, **opts)
        self.cnn_out = Conv(store, "cnn_out", 3, 2 * nf, 4 + C, bias=True)
        self.bfocal = store.add("b_focal", (1,), constant(math.log((1.0 - tmp_pi) / tmp_pi)))

    # ---- parameters ---------------------------------------------------------------------------
    def seps(self):
        out = [self.stem.sep]
        for b in self.blocks.values():
            out += b.seps()
        return out

    def bns(self):
        return [bn for b in self.blocks.values() for bn in b.bns()]

    def _make_plan(self):
        seps = self.seps()
        entries = [self.stem.pack_entry()] + [(s.pw if s.split else s.conv).pack_entry() for s in seps[1:]]
        entries.append(self.cnn_out.pack_entry())
        folds = [s.sep_entry() for s in seps if isinstance(s, SepConv) and not s.split]
        self._plan = (nn.SepPlan(folds, self.device) if folds else None, nn.PackPlan(entries, self.device))

    def _mode_changed(self):
        self._plan = None

    def pack(self):
        """fold every separable conv, fold b_focal, re-pack all bf16 conv weights (3 launches)."""
        if self._plan is None:
            self._make_plan()
        sep, pk = self._plan
        if sep is not None:
            sep.fold()
        pk.run()
        nn.bias_scalar_fold(self.cnn_out.b, self.store.p(self.bfocal), self.b_eff, 4)

    def unfold_grads(self):
        if self._plan[0] is not None:
            self._plan[0].unfold()

    def grad_groups(self):
        """One group: the separable-conv unfold finalises every gradient at the end of backward
        (2.6 M parameters, 10 MB: a single all-reduce)."""
        return [("all", list(self.store.offsets))]

    @staticmethod
    def out_hw(H, W):
        s2 = lambda n: -(-n // 2)    # noqa: E731  (SAME stride 2 / pool 2 "same")
        return s2(s2(H)), s2(s2(W))

    # ---- forward / backward -----------------------------------------------------------------
    def __call__(self, x, training=False, group=None):
        """Keras-style call: x [B,H,W,3] (array or tensor) -> [B,H/4,W/4,4+C] fp32."""
        x = torch.as_tensor(x, dtype=torch.float32).to(self.device).contiguous()
        return self.forward(x, group=group, train=training)

    def forward(self, x, group=None, train=True):
        """x fp32 NHWC [B,H,W,3]; group = BN sub-batch size (default: the whole batch)."""
        B, H, W, _ = x.shape
        group = B if group is None else int(group)
        dev = x.device
        v, hw, saved = {}, {}, {}
        v["blk0"], sv_stem = self.stem.forward(x)
        H0, W0 = v["blk0"].shape[1], v["blk0"].shape[2]
        hw["blk0"] = (H0, W0)

        def run(name):
            _, i, o = self._graph[name]
            h, w_ = hw[i]
            v[o], saved[name] = self.blocks[name].forward(v[i], B, h, w_, group, train)
            hw[o] = (h, w_)
            return v[o]

        def pool(src, key):
            h, w_ = hw[src]
            Ho, Wo = -(-h // 2), -(-w_ // 2)
            t = v[src]
            y = torch.empty((B, Ho, Wo, t.shape[3]), dtype=BF16, device=dev)
            arg = torch.empty((B, Ho, Wo, t.shape[3]), dtype=torch.uint8, device=dev)
            nn.maxpool2x2(t, y, arg)
            v[key], hw[key] = y, (Ho, Wo)
            saved["pool_" + key] = arg

        def res_add(a, b, key):
            o = torch.empty_like(v[a])
            nn.add(v[a], v[b], o)
            v[key], hw[key] = o, hw[a]

        def up_add(prev, other, key):
            o = torch.empty_like(v[other])
            nn.upsample_bilinear2x_add(v[prev], v[other], o)
            v[key], hw[key] = o, hw[other]

        self._graph = dict((b[0], b) for b in block_graph(self.n_stacks))
        run("cnn_block_1")
        pool("cnn1", skey(1, "stack_in"))
        for s in range(1, self.n_stacks + 1):
            st = "stack_%d_" % s
            k = lambda n: skey(s, n)   # noqa: E731
            run(st + "enc_block_1"); res_add(k("stack_in"), k("enc1"), k("e1res")); pool(k("e1res"), k("e1"))  # noqa: E702
            run(st + "enc_block_2"); res_add(k("e1"), k("enc2"), k("e2res")); pool(k("e2res"), k("e2"))        # noqa: E702
            run(st + "enc_block_3"); res_add(k("e2"), k("enc3"), k("e3res")); pool(k("e3res"), k("e3"))        # noqa: E702
            run(st + "enc_block_4a"); run(st + "enc_block_4b"); run(st + "enc_block_4")                         # noqa: E702
            res_add(k("e3"), k("enc4"), k("e4res")); pool(k("e4res"), k("e4"))                                  # noqa: E702
            run(st + "dec_block_1"); up_add(k("e4"), k("dec1"), k("d1res")); run(st + "dec_out_1")             # noqa: E702
            run(st + "dec_block_2"); up_add(k("o1"), k("dec2"), k("d2res")); run(st + "dec_out_2")             # noqa: E702
            run(st + "dec_block_3"); up_add(k("o2"), k("dec3"), k("d3res")); run(st + "dec_out_3")             # noqa: E702
            run(st + "dec_block_4"); up_add(k("o3"), k("dec4"), k("d4res")); run(st + "dec_out_4")             # noqa: E702
            if s < self.n_stacks:         # the stack's output is the next stack's input
                v[skey(s + 1, "stack_in")], hw[skey(s + 1, "stack_in")] = v[k("o4")], hw[k("o4")]
        v["o4"], hw["o4"] = v[skey(self.n_stacks, "o4")], hw[skey(self.n_stacks, "o4")]
        Ho, Wo = hw["o4"]
        c = self.cnn_out
        out = torch.empty((B, Ho, Wo, 4 + self.C), dtype=torch.float32, device=dev)
        d = c.fwd_desc(B, [nn.seg(Ho, Wo, Ho, Wo, c.wf, self.b_eff)], ld_dst=4 + self.C, dst_f32=True)
        nn.conv_igemm(d, v["o4"], out)
        self._saved = (sv_stem, saved, v, hw, B, group)
        if self._plan is None:        # a separable conv switched form at this map size: re-plan now
            self._make_plan()
        return out

    def backward(self, d_out, hook=None):
        """d_out: bf16 [B,Ho,Wo,cout_ld] gradient of the output (cvl_centernet_loss).  Writes every
        parameter gradient of the store (overwrite semantics)."""
        sv_stem, saved, v, hw, B, group = self._saved
        c = self.cnn_out
        Ho, Wo = hw["o4"]
        HW = Ho * Wo
        # the convs' bias gradients (column sums of their output gradients) are collected and run as
        # batched cvl_bias_grad_multi launches (16 per launch pair) at the end, instead of two
        # launches per conv (91 convs per stack)
        sink = [(d_out, int(d_out.shape[-1]), 0, 4 + self.C, 0, HW, HW, B, self.g_beff, 0.0)]
        for sc in self.seps()[1:]:
            sc.bias_sink = sink
        c.wgrad(v["o4"], d_out, B, Ho, Wo, bias=False)
        g = {}
        g[skey(self.n_stacks, "o4")] = c.dgrad(d_out, B, Ho, Wo)

        def blk(name, dy, dx_key, beta):
            _, i, _ = self._graph[name]
            if dx_key not in g:
                g[dx_key] = torch.empty_like(v[i])
                beta = 0.0
            self.blocks[name].backward(dy, saved[name], g[dx_key], beta)

        def unpool(key, src):                 # g[src] = maxpool backward of g[key]
            t = torch.empty_like(v[src])
            nn.maxpool2x2_backward(g[key], saved["pool_" + key], t)
            g[src] = t

        def upb(res, prev):                   # grad of the up-sampled input of a decoder merge
            t = torch.empty_like(v[prev])
            nn.upsample_bilinear2x_backward(g[res], t)
            g[prev] = t

        def acc(dst, src):                    # g[dst] += g[src] (or alias)
            if dst in g:
                nn.add(g[dst], g[src], g[dst])
            else:
                g[dst] = g[src].clone()

        for s in range(self.n_stacks, 0, -1):
            st = "stack_%d_" % s
            k = lambda n: skey(s, n)   # noqa: E731
            # decoder, last merge first: dX_res feeds both the dec block and the up-sampled input
            blk(st + "dec_out_4", g[k("o4")], k("d4res"), 0.0)
            upb(k("d4res"), k("o3"))
            blk(st + "dec_block_4", g[k("d4res")], k("stack_in"), 0.0)
            blk(st + "dec_out_3", g[k("o3")], k("d3res"), 0.0)
            upb(k("d3res"), k("o2"))
            blk(st + "dec_block_3", g[k("d3res")], k("e1"), 0.0)
            blk(st + "dec_out_2", g[k("o2")], k("d2res"), 0.0)
            upb(k("d2res"), k("o1"))
            blk(st + "dec_block_2", g[k("d2res")], k("e2"), 0.0)
            blk(st + "dec_out_1", g[k("o1")], k("d1res"), 0.0)
            upb(k("d1res"), k("e4"))
            blk(st + "dec_block_1", g[k("d1res")], k("e3"), 0.0)
            # encoder: x_res = x + cnn(x) -> pool
            unpool(k("e4"), k("e4res"))
            acc(k("e3"), k("e4res"))
            blk(st + "enc_block_4", g[k("e4res")], k("enc4b"), 0.0)
            blk(st + "enc_block_4b", g[k("enc4b")], k("enc4a"), 0.0)
            blk(st + "enc_block_4a", g[k("enc4a")], k("e3"), 1.0)
            unpool(k("e3"), k("e3res"))
            acc(k("e2"), k("e3res"))
            blk(st + "enc_block_3", g[k("e3res")], k("e2"), 1.0)
            unpool(k("e2"), k("e2res"))
            acc(k("e1"), k("e2res"))
            blk(st + "enc_block_2", g[k("e2res")], k("e1"), 1.0)
            unpool(k("e1"), k("e1res"))
            acc(k("stack_in"), k("e1res"))
            blk(st + "enc_block_1", g[k("e1res")], k("stack_in"), 1.0)
            if s > 1:                         # this stack's input is the previous stack's output
                g[skey(s - 1, "o4")] = g[k("stack_in")]
        unpool(skey(1, "stack_in"), "cnn1")
        blk("cnn_block_1", g["cnn1"], "blk0", 0.0)
        self.stem.backward(g["blk0"], sv_stem)
        for sc in self.seps()[1:]:
            sc.bias_sink = None
        nn.bias_grad_multi(sink)
        nn.bias_scalar_unfold(self.g_beff, c.db, self.store.g(self.bfocal), 4)
        self.unfold_grads()
        self._saved = None
        if hook is not None:
            hook("all")

    @staticmethod
    def param_dict(n_classes, seed=0, **kw):
        """Initial parameters (Keras names -> CPU fp32) without a GPU (for the CPU oracle)."""
        net = HourglassNet.__new__(HourglassNet)
        net.C = n_classes
        store, eff = ParamStore(), ParamStore()
        net._build(store, eff, n_classes, kw.get("tmp_pi", 0.99), kw.get("n_filters", 128),
                   kw.get("n_stacks", 1), kw.get("n_repeats", 2),
                   dict(seperable=kw.get("seperable", True), batch_norm=kw.get("batch_norm", True),
                        norm_order=kw.get("norm_order", "norm_first")))
        store.finalize("cpu", seed)
        return {k: store.p(k).clone() for k in store.offsets}
