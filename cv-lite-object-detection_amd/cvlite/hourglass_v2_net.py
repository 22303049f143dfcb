"""CenterNet v2 — the network CenterNet/train_hourglass_voc.py trains (tf_hourglass_net.build_model,
:115-394, with the script's n_filters=12, n_features=64, n_repeats=2, separable, norm_first BN) —
as an explicit forward / backward graph on the cvlite kernels.  The other build options are
supported too: Conv2D instead of SeparableConv2D (seperable=False), no BatchNormalization, and
norm_last (BN on each conv's output, before its ReLU: cnn_block :47-77, downsample_block :79-113).

Graph (nf = n_filters): a 3x3 separable conv on the image (no BN / ReLU), cnn_block_1 (nf), six
[downsample (BN -> separable 3x3/2 -> ReLU) + cnn_block + residual] encoder stages to 64 nf at
H/64, six decoder stages UpSampling2D(bilinear)(encoder residual + previous decoder output) ->
cnn_block, then the "pass through" (:307-344): the 12 encoder/decoder maps are tf.reshape'd to
[B, H/8, W/8, *] (a reinterpretation of the row-major NHWC bytes, Q36 — not space-to-depth) and
concatenated (189 nf channels), cnn_block "final_out" (n_features), the Conv2D head with
4 * (5 + C) channels read as [S, S, 4 scales, 5 + C]; sigmoid on the 4 box channels, the b_focal
BiasLayer on the rest (applied inside the fused loss / `outputs`).

MI355X mapping:
  * channel counts that are not multiples of 32 (nf = 12, 24, 48 and the 2268-wide concat) live
    with a zero-padded channel pitch cp(c) = round_up(c, 32): the MFMA conv kernels want 32-channel
    blocks.  Pads are exact zeros everywhere: the folded dense kernels are zero outside the real
    (cin, cout) block (fold with pitches, cvl_sep_item.cin_ld / cout_ld), BN of a zero channel is
    beta = 0, ReLU / residual / up-sampling keep zeros, and every pad receives a zero gradient.
    The BN gamma / beta and conv bias parameters are stored padded (pads never change); the
    depthwise / pointwise kernels keep their Keras shapes;
  * every SeparableConv2D is ONE dense conv with the folded kernel D x P (as hourglass_net.py);
    the first one (3 input channels) is im2col (K = 27 -> 32) + one GEMM;
  * UpSampling2D of a residual sum is one pass (cvl_upsample_bilinear2x_sum, taps of a + b in
    fp32); the reshape-concat and its adjoint are one gather / scatter launch each
    (cvl_reshape_concat[_backward]);
  * BatchNorm statistics over sub-batches of `group` images (one Keras forward per sub-batch in
    train_step :436-445);
  * b_focal folded into the head bias on every scale's class channels (periodic fold).
Keras names: `cnn_block_0`, `<blk>_bn_<r>` / `<blk>_cnn_<r>` (cnn_block), `down_block_<k>_bnorm` /
`down_block_<k>` (downsample_block), `dec_block_<k>`, `final_out`, `head_out`, `b_focal`.
"""
import math

import torch

from . import ops_nn as nn
from .hourglass_net import BN_EPS, BN_MOMENTUM
from .layers import BF16, BatchNorm, Conv, ParamStore, constant, glorot_uniform

STEM_KP = 32           # im2col K = 3*3*3 = 27 padded to 32


def cp(c):
    """Channel pitch of a c-channel map (multiple of 32)."""
    return (c + 31) // 32 * 32


class SepConvP(object):
    """Keras SeparableConv2D(cout, k, stride, "same") with channel-padded input / output maps:
    dense conv [k][k][cp(cin)][cp(cout)] (eff store, zero outside the real block)."""

    def __init__(self, store, eff, name, k, cin, cout, stride=1):
        self.name, self.k, self.cin, self.cout, self.stride = name, k, cin, cout, stride
        self.cpi, self.cpo = cp(cin), cp(cout)
        self.dwname = store.add(name + "/depthwise_kernel", (k, k, cin, 1), glorot_uniform(k * k * cin, k * k))
        self.pwname = store.add(name + "/pointwise_kernel", (1, 1, cin, cout), glorot_uniform(cin, cout))
        self.bname = store.add(name + "/bias", (self.cpo,), constant(0.0))
        self.store = store
        self.conv = Conv(eff, name, k, self.cpi, self.cpo, stride, "same", bias=False)

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

    def out_hw(self, H, W):
        Ho, Wo, _, _ = self.conv.out_hw(H, W)
        return Ho, Wo

    def fwd(self, x, B, H, W, relu_out=False):
        c = self.conv
        Ho, Wo = self.out_hw(H, W)
        out = torch.empty((B, Ho, Wo, self.cpo), dtype=BF16, device=x.device)
        d = c.fwd_desc(B, [nn.seg(Ho, Wo, H, W, c.wf, self.b)], ld_dst=self.cpo, relu_out=relu_out,
                       n_store=self.cpo)
        nn.conv_igemm(d, x, out)
        return out

    def wgrad(self, x, dy, B, H, W):
        self.conv.wgrad(x, dy, B, H, W, bias=False)
        Ho, Wo = self.out_hw(H, W)
        nn.bias_grad(dy, self.cpo, 0, self.cpo, 0, Ho * Wo, Ho * Wo, B, self.db)

    def dgrad(self, dy, B, H, W, out=None, beta=0.0):
        return self.conv.dgrad(dy, B, H, W, out=out, beta=beta)


def padded_glorot(k, cin, cout, cpi, cpo):
    """Glorot-uniform over the real [k,k,cin,cout] block of a channel-padded kernel, zero pads."""
    lim = math.sqrt(6.0 / (k * k * cin + k * k * cout))

    def init(gen, shape):
        w = torch.zeros(shape, dtype=torch.float32)
        w[:, :, :cin, :cout] = (torch.rand((k, k, cin, cout), generator=gen, dtype=torch.float64) * 2 - 1).mul_(lim).float()
        return w
    return init


class DenseConvP(SepConvP):
    """Keras Conv2D(cout, k, stride, "same") with bias (seperable=False) on channel-padded maps: the
    trainable kernel is kept at its padded shape [k][k][cp(cin)][cp(cout)] (zero pads, which get
    zero gradients), the bias padded to cp(cout) like every v2 per-channel parameter."""

    def __init__(self, store, name, k, cin, cout, stride=1):
        self.name, self.k, self.cin, self.cout, self.stride = name, k, cin, cout, stride
        self.cpi, self.cpo = cp(cin), cp(cout)
        self.conv = Conv(store, name, k, self.cpi, self.cpo, stride, "same", bias=False,
                         w_init=padded_glorot(k, cin, cout, self.cpi, self.cpo))
        self.bname = store.add(name + "/bias", (self.cpo,), constant(0.0))
        self.store = store

    def sep_entry(self):
        raise TypeError("a Conv2D has no separable fold")


def conv_p(seperable, store, eff, name, k, cin, cout, stride=1):
    if seperable:
        return SepConvP(store, eff, name, k, cin, cout, stride=stride)
    return DenseConvP(store, name, k, cin, cout, stride=stride)


class StemV2(object):
    """cnn_block_0 (:131-140): SeparableConv2D(nf, 3x3, "same") on the 3-channel image as im2col
    (K = 27 -> 32) + one GEMM with the folded kernel [3][3][3][nf]; output pitch cp(nf)."""

    def __init__(self, store, eff, nf, seperable=True):
        self.nf, self.cpo = nf, cp(nf)
        self.seperable = seperable
        name = "cnn_block_0"
        if seperable:
            self.dwname = store.add(name + "/depthwise_kernel", (3, 3, 3, 1), glorot_uniform(27, 9))
            self.pwname = store.add(name + "/pointwise_kernel", (1, 1, 3, nf), glorot_uniform(3, nf))
        self.bname = store.add(name + "/bias", (self.cpo,), constant(0.0))
        self.store = store
        # separable: the folded kernel in the eff store; Conv2D: the trainable kernel itself
        self.conv = Conv(eff if seperable else store, name, 3, 3, nf, 1, "same", bias=False, cin_k=STEM_KP,
                         npad=self.cpo, dgrad=False)

    def sep_entry(self):
        st = self.store
        return (st.p(self.dwname), st.p(self.pwname), self.conv.w, self.conv.dw, st.g(self.dwname),
                st.g(self.pwname))

    def pack_entry(self):
        c = self.conv
        if c.wf is None:
            c.wf = torch.empty((self.cpo, STEM_KP), dtype=BF16, device=c.store.flat.device)
        return (c.w, 1, 27, self.nf, STEM_KP, self.cpo, c.wf, 0, 0, None)

    def _desc(self, B, H, W):
        return nn.make_desc(nn.FWD, B, STEM_KP, 1, 1, 1, 0, 0, self.cpo, self.cpo, self.cpo,
                            [nn.seg(H, W, H, W, self.conv.wf, self.store.p(self.bname))])

    def forward(self, x):
        B, H, W, _ = x.shape
        A = torch.empty((B * H * W, STEM_KP), dtype=BF16, device=x.device)
        nn.im2col(x, 3, 3, 1, 1, 1, H, W, STEM_KP, A)
        z = torch.empty((B, H, W, self.cpo), dtype=BF16, device=x.device)
        nn.conv_igemm(self._desc(B, H, W), A, z)
        return z, (A, B, H, W)

    def backward(self, dz, saved):
        A, B, H, W = saved
        dw = torch.empty((STEM_KP, self.cpo), dtype=torch.float32, device=dz.device)
        nn.conv_wgrad(self._desc(B, H, W), A, dz, dw)
        nn.wgrad_flush()                             # dw is read right away (deferred reductions)
        self.conv.dw.view(27, self.nf).copy_(dw[:27, :self.nf])
        nn.bias_grad(dz, self.cpo, 0, self.cpo, 0, H * W, H * W, B, self.store.g(self.bname))


def _bn_forward(bn, t, B, HW, group, train, relu=False):
    c = bn.c
    mr = torch.empty((B, c, 2), dtype=torch.float32, device=t.device)
    if train:
        stats = nn.bn_acc(B, c, t.device, zero=False)
        nn.bn_stats(t, B, HW, c, stats)
        nn.bn_finalize_grouped(stats, mr, bn.run_mean, bn.run_var, B, c, HW, group, bn.eps, bn.momentum)
    else:                                        # Keras inference: moving statistics
        mr[:, :, 0] = bn.run_mean
        mr[:, :, 1] = torch.rsqrt(bn.run_var + bn.eps)
    a = torch.empty_like(t)
    nn.bn_apply(t, mr, bn.gamma, bn.beta, None, a, B, HW, c, relu)
    return a, mr


class _UnitV2(object):
    """A conv unit of tf_hourglass_net (:35-113): [BN (norm_first)] -> conv -> [BN (norm_last)] -> ReLU
    (batch_norm=False: no BN).  The norm_first BN is over the unit's input, the norm_last one over
    its output; both keep channel-padded parameters and the real channel count in bn_c."""

    def _init_unit(self, store, eff, bn_name, conv_name, cin, cout, stride, seperable, batch_norm, norm_order):
        if norm_order not in ("norm_first", "norm_last"):
            raise ValueError("norm_order must be 'norm_first' or 'norm_last'")
        self.norm_first = norm_order == "norm_first"
        self.bn_c = cin if self.norm_first else cout
        self.bn = BatchNorm(store, bn_name, cp(self.bn_c), eps=BN_EPS, momentum=BN_MOMENTUM) if batch_norm else None
        self.sep = conv_p(seperable, store, eff, conv_name, 3, cin, cout, stride)
        self.store = store

    def _unit_fwd(self, t, B, H, W, group, train):
        a, mr, z = t, None, None
        if self.bn is not None and self.norm_first:
            a, mr = _bn_forward(self.bn, t, B, H * W, group, train)
        if self.bn is not None and not self.norm_first:
            z = self.sep.fwd(a, B, H, W)
            Ho, Wo = self.sep.out_hw(H, W)
            y, mr = _bn_forward(self.bn, z, B, Ho * Wo, group, train, relu=True)
        else:
            y = self.sep.fwd(a, B, H, W, relu_out=True)
        return a, mr, z, y

    def _unit_bwd_to_a(self, dout, a, mr, z, y, B, H, W, group):
        """gradient of the conv's output (through ReLU [and the norm_last BN]) -> wgrad, returns du."""
        st = self.store
        du = torch.empty_like(y)
        if z is not None:
            Ho, Wo = self.sep.out_hw(H, W)
            nn.bn_backward_grouped(dout, z, mr, self.bn.gamma, du, st.g(self.bn.gname), st.g(self.bn.bname),
                                   B, Ho * Wo, self.bn.c, group, y_relu=y)
        else:
            nn.relu_backward(dout, y, du)
        self.sep.wgrad(a, du, B, H, W)
        return du

    def _input_grad(self, da, t, mr, B, H, W, group, dx_out, dx_beta):
        st = self.store
        if self.bn is not None and self.norm_first:
            nn.bn_backward_grouped(da, t, mr, self.bn.gamma, dx_out, st.g(self.bn.gname), st.g(self.bn.bname),
                                   B, H * W, self.bn.c, group, dz_beta=dx_beta)
        elif da is not dx_out:
            if dx_beta:
                nn.add(dx_out, da, dx_out)
            else:
                dx_out.copy_(da)


class RepeatV2(_UnitV2):
    """One cnn_block repeat (:35-77): norm_first: a = BN(t); y = ReLU(conv3x3(a)); out = y (r = 0) or
    y + a (the residual adds the BN OUTPUT: tmp_input is rebound to it); norm_last: y =
    ReLU(BN(conv3x3(t))), out = y or y + t."""

    def __init__(self, store, eff, blk, r, cin, nf, seperable=True, batch_norm=True, norm_order="norm_first"):
        self.r, self.cin, self.cout = r, cin, nf
        self._init_unit(store, eff, "%s_bn_%d" % (blk, r), "%s_cnn_%d" % (blk, r), cin, nf, 1, seperable, batch_norm,
                        norm_order)

    def forward(self, t, B, H, W, group, train=True):
        a, mr, z, y = self._unit_fwd(t, B, H, W, group, train)
        if self.r == 0:
            o = y
        else:
            o = torch.empty_like(y)
            nn.add(y, a, o)
        return o, (t, mr, a, z, y, B, H, W, group)

    def backward(self, dout, saved, dx_out, dx_beta=0.0):
        """dout is clobbered when r >= 1 (it becomes the residual addend's gradient)."""
        t, mr, a, z, y, B, H, W, group = saved
        du = self._unit_bwd_to_a(dout, a, mr, z, y, B, H, W, group)
        direct = self.r == 0 and not (self.bn is not None and self.norm_first)
        if direct:
            da = self.sep.dgrad(du, B, H, W, out=dx_out, beta=dx_beta)
        elif self.r == 0:
            da = self.sep.dgrad(du, B, H, W)
        else:
            da = self.sep.dgrad(du, B, H, W, out=dout, beta=1.0)       # + the residual branch
        self._input_grad(da, t, mr, B, H, W, group, dx_out, dx_beta)


class CnnBlockV2(object):
    def __init__(self, store, eff, name, cin, nf, n_repeats, **opts):
        self.name = name
        self.reps = [RepeatV2(store, eff, name, r, cin if r == 0 else nf, nf, **opts) for r in range(n_repeats)]
        self.cout = nf

    def seps(self):
        return [r.sep for r in self.reps]

    def bns(self):
        return [r.bn for r in self.reps if r.bn is not None]

    def units(self):
        return list(self.reps)

    def forward(self, x, B, H, W, group, train=True):
        h, saved = x, []
        for rep in self.reps:
            h, sv = rep.forward(h, B, H, W, group, train)
            saved.append(sv)
        return h, saved

    def backward(self, dy, saved, dx_out, dx_beta=0.0):
        """dy is clobbered; the block-input gradient is written / accumulated into dx_out."""
        g = dy
        for i in range(len(self.reps) - 1, -1, -1):
            tgt = dx_out if i == 0 else torch.empty_like(saved[i][0])
            self.reps[i].backward(g, saved[i], tgt, dx_beta if i == 0 else 0.0)
            g = tgt
        return dx_out


class DownV2(_UnitV2):
    """downsample_block (:79-113): [BN] -> conv 3x3 / 2 "same" -> [BN] -> ReLU."""

    def __init__(self, store, eff, name, cin, cout, seperable=True, batch_norm=True, norm_order="norm_first"):
        self._init_unit(store, eff, name + "_bnorm", name, cin, cout, 2, seperable, batch_norm, norm_order)
        self.cout = cout

    def seps(self):
        return [self.sep]

    def bns(self):
        return [self.bn] if self.bn is not None else []

    def units(self):
        return [self]

    def forward(self, t, B, H, W, group, train=True):
        a, mr, z, y = self._unit_fwd(t, B, H, W, group, train)
        return y, (t, mr, a, z, y, B, H, W, group)

    def backward(self, dout, saved, dx_out, dx_beta=0.0):
        t, mr, a, z, y, B, H, W, group = saved
        du = self._unit_bwd_to_a(dout, a, mr, z, y, B, H, W, group)
        if self.bn is not None and self.norm_first:
            da = self.sep.dgrad(du, B, H, W)
        else:
            da = self.sep.dgrad(du, B, H, W, out=dx_out, beta=dx_beta)
        self._input_grad(da, t, mr, B, H, W, group, dx_out, dx_beta)


CONCAT_ORDER = ("blk1", "blk2", "blk3", "blk4", "blk5", "blk6", "dec1", "dec2", "dec3", "dec4", "dec5", "dec6")


class HourglassV2Net(object):
    """tf_hourglass_net.build_model(n_filters, n_classes, tmp_pi, n_repeats, n_features) on MI355X.
    forward(x [B,H,W,3] fp32, H and W multiples of 64) -> head logits fp32 [B, H/8, W/8, ld]
    (channel sc*(5+C) + j; b_focal folded into the class channels' bias, no sigmoid);
    backward(d_out bf16 [B, H/8, W/8, ld])."""

    def __init__(self, n_classes, n_filters=12, tmp_pi=0.99, n_repeats=2, n_features=64, device="cuda", seed=0,
                 seperable=True, batch_norm=True, norm_order="norm_first"):
        assert n_filters % 4 == 0 and n_features % 32 == 0, "n_filters % 4, n_features % 32 (reshape / conv pitch)"
        self.C, self.nf, self.nfeat = n_classes, n_filters, n_features
        self.R = 5 + n_classes
        self.device = torch.device(device)
        store, eff = ParamStore(), ParamStore()
        self.opts = dict(seperable=seperable, batch_norm=batch_norm, norm_order=norm_order)
        self._build(store, eff, n_classes, tmp_pi, n_filters, n_repeats, n_features, self.opts)
        store.finalize(self.device, seed)
        eff.finalize(self.device, seed + 1)
        eff.flat.zero_()                     # folded kernels: zero outside the real (cin, cout) block
        self.store, self.eff = store, eff
        for bn in self.bns():
            bn.init_buffers(self.device)
        self.cout = 4 * self.R
        self.cout_ld = self.head.npad
        self.b_eff = torch.zeros(self.cout, dtype=torch.float32, device=self.device)
        self.g_beff = torch.zeros(self.cout, dtype=torch.float32, device=self.device)
        self._plan = None
        self._saved = None
        self.pack()

    def _build(self, store, eff, C, tmp_pi, nf, n_repeats, n_features, opts=None):
        o = opts or {}
        self.stem = StemV2(store, eff, nf, o.get("seperable", True))
        self.enc = [CnnBlockV2(store, eff, "cnn_block_1", nf, nf, n_repeats, **o)]
        self.down = [DownV2(store, eff, "down_block_1", nf, 2 * nf, **o)]
        for k in range(2, 7):
            c = (2 ** (k - 1)) * nf
            self.enc.append(CnnBlockV2(store, eff, "cnn_block_%d" % k, c, c, n_repeats, **o))
            self.down.append(DownV2(store, eff, "down_block_%d" % k, c, 2 * c, **o))
        self.dec = [CnnBlockV2(store, eff, "dec_block_%d" % k, (2 ** (7 - k)) * nf, (2 ** (6 - k)) * nf, n_repeats,
                               **o) for k in range(1, 7)]
        self.feat_c = 189 * nf                           # 63 nf encoder + 126 nf decoder channels
        self.final = CnnBlockV2(store, eff, "final_out", self.feat_c, n_features, n_repeats, **o)
        self.head = Conv(store, "head_out", 3, n_features, 4 * (5 + C), bias=True)
        self.bfocal = store.add("b_focal", (1,), constant(math.log((1.0 - tmp_pi) / tmp_pi)))

    # ---- parameters -------------------------------------------------------------------------
    def blocks(self):
        return self.enc + self.down + self.dec + [self.final]

    def seps(self):
        return [s for b in self.blocks() for s in b.seps()]

    def bns(self):
        return [bn for b in self.blocks() for bn in b.bns()]

    def _make_plan(self):
        seps = self.seps()
        entries = [self.stem.pack_entry()] + [s.conv.pack_entry() for s in seps] + [self.head.pack_entry()]
        folds = ([self.stem.sep_entry()] if self.stem.seperable else []) + \
            [s.sep_entry() for s in seps if not isinstance(s, DenseConvP)]
        self._plan = (nn.SepPlan(folds, self.device) if folds else None, nn.PackPlan(entries, self.device))

    def pack(self):
        """Fold every separable conv, fold b_focal, re-pack every bf16 conv kernel (3 launches)."""
        if self._plan is None:
            self._make_plan()
        sep, pk = self._plan
        if sep is not None:
            sep.fold()
        pk.run()
        nn.bias_scalar_fold_periodic(self.head.b, self.store.p(self.bfocal), self.b_eff, self.R, 4)

    def grad_groups(self):
        return [("all", list(self.store.offsets))]

    @staticmethod
    def out_hw(H, W):
        return H // 8, W // 8

    def real_params(self, grads=False):
        """The Keras-shaped parameters (or their gradients), channel pads stripped, CPU fp32: the
        oracle's view of the model."""
        get = self.store.g if grads else self.store.p
        out = {k: get(k).detach().cpu().clone() for k in self.store.offsets}
        cut = [(self.stem.bname, self.nf)]
        for blk in self.blocks():
            for u in blk.units():
                if u.bn is not None:
                    cut += [(u.bn.gname, u.bn_c), (u.bn.bname, u.bn_c)]
                cut.append((u.sep.bname, u.sep.cout))
                if isinstance(u.sep, DenseConvP):          # Conv2D kernel kept channel-padded
                    k = u.sep.conv.wname
                    out[k] = out[k][:, :, :u.sep.cin, :u.sep.cout].clone()
        for k, c in cut:
            out[k] = out[k][:c].clone()
        return out

    # ---- forward / backward -----------------------------------------------------------------
    def __call__(self, x, training=False, group=None):
        x = torch.as_tensor(x, dtype=torch.float32).to(self.device).contiguous()
        return self.outputs(self.forward(x, group=group, train=training))

    def outputs(self, logits):
        """The Keras model output [B,S,S,4,5+C]: sigmoid box channels, class logits + b_focal
        (b_focal is already in the head bias)."""
        B, S0, S1, _ = logits.shape
        o = logits[..., :self.cout].reshape(B, S0, S1, 4, self.R)
        return torch.cat([torch.sigmoid(o[..., :4]), o[..., 4:]], -1)

    def forward(self, x, group=None, train=True):
        B, H, W, _ = x.shape
        assert H % 64 == 0 and W % 64 == 0, "tf_hourglass_net needs H, W multiples of 64 (6 stride-2 stages)"
        group = B if group is None else int(group)
        dev = x.device
        v, sv, hw = {}, {}, {}
        v["blk0"], sv["stem"] = self.stem.forward(x)
        v["cnn1"], sv["cnn1"] = self.enc[0].forward(v["blk0"], B, H, W, group, train)
        hw["blk0"] = (H, W)
        v["blk1"], sv["d1"] = self.down[0].forward(v["cnn1"], B, H, W, group, train)
        hw["blk1"] = (H // 2, W // 2)
        for k in range(2, 7):
            h, w = hw["blk%d" % (k - 1)]
            c, sv["cnn%d" % k] = self.enc[k - 1].forward(v["blk%d" % (k - 1)], B, h, w, group, train)
            s = torch.empty_like(c)
            nn.add(v["blk%d" % (k - 1)], c, s)
            v["in%d" % k] = s
            v["blk%d" % k], sv["d%d" % k] = self.down[k - 1].forward(s, B, h, w, group, train)
            hw["blk%d" % k] = (h // 2, w // 2)
        h, w = hw["blk6"]
        u = torch.empty((B, 2 * h, 2 * w, v["blk6"].shape[-1]), dtype=BF16, device=dev)
        nn.upsample_bilinear2x_sum(v["blk6"], None, u)
        v["ups1"] = u
        v["dec1"], sv["dec1"] = self.dec[0].forward(u, B, 2 * h, 2 * w, group, train)
        for k in range(2, 7):
            a, b = v["in%d" % (8 - k)], v["dec%d" % (k - 1)]
            h, w = a.shape[1], a.shape[2]
            u = torch.empty((B, 2 * h, 2 * w, a.shape[-1]), dtype=BF16, device=dev)
            nn.upsample_bilinear2x_sum(a, b, u)
            v["ups%d" % k] = u
            v["dec%d" % k], sv["dec%d" % k] = self.dec[k - 1].forward(u, B, 2 * h, 2 * w, group, train)
        S0, S1 = H // 8, W // 8
        feats = torch.empty((B, S0, S1, cp(self.feat_c)), dtype=BF16, device=dev)
        nn.reshape_concat([(v[k], self._real_c(k)) for k in CONCAT_ORDER], feats)
        hfin, sv["final"] = self.final.forward(feats, B, S0, S1, group, train)
        hd = self.head
        out = torch.empty((B, S0, S1, self.cout_ld), dtype=torch.float32, device=dev)
        d = hd.fwd_desc(B, [nn.seg(S0, S1, S0, S1, hd.wf, self.b_eff)], ld_dst=self.cout_ld, dst_f32=True)
        nn.conv_igemm(d, hfin, out)
        v["feats"], v["final"] = feats, hfin
        self._saved = (v, sv, B, S0, S1)
        return out

    def _real_c(self, key):
        nf = self.nf
        if key.startswith("blk"):
            return (2 ** int(key[3:])) * nf
        return (2 ** (6 - int(key[3:]))) * nf

    def backward(self, d_out, hook=None):
        """d_out bf16 [B,S,S,cout_ld] (cvl_hourglass_v2_loss).  Writes every parameter gradient of
        the store (overwrite semantics)."""
        v, sv, B, S0, S1 = self._saved
        hd = self.head
        hd.wgrad(v["final"], d_out, B, S0, S1, bias=False)
        nn.bias_grad(d_out, int(d_out.shape[-1]), 0, self.cout, 0, S0 * S1, S0 * S1, B, self.g_beff)
        nn.bias_scalar_unfold_periodic(self.g_beff, hd.db, self.store.g(self.bfocal), self.R, 4)
        g_h = hd.dgrad(d_out, B, S0, S1)
        g_feats = torch.empty_like(v["feats"])
        self.final.backward(g_h, sv["final"], g_feats, 0.0)
        g = {k: torch.empty_like(v[k]) for k in CONCAT_ORDER}
        nn.reshape_concat_backward([(g[k], self._real_c(k), 0.0) for k in CONCAT_ORDER], g_feats)
        # decoder, last stage first: ups_k = up(in_{8-k} + dec_{k-1})
        for k in range(6, 1, -1):
            gu = torch.empty_like(v["ups%d" % k])
            self.dec[k - 1].backward(g["dec%d" % k], sv["dec%d" % k], gu, 0.0)
            a = "in%d" % (8 - k)
            g[a] = torch.empty_like(v[a])
            nn.upsample_bilinear2x_backward(gu, g[a], beta=0.0)
            nn.upsample_bilinear2x_backward(gu, g["dec%d" % (k - 1)], beta=1.0)
        gu = torch.empty_like(v["ups1"])
        self.dec[0].backward(g["dec1"], sv["dec1"], gu, 0.0)
        nn.upsample_bilinear2x_backward(gu, g["blk6"], beta=1.0)
        # encoder: blk_k = down_k(in_k); in_k = blk_{k-1} + cnn_k(blk_{k-1})
        for k in range(6, 1, -1):
            self.down[k - 1].backward(g["blk%d" % k], sv["d%d" % k], g["in%d" % k], 1.0)
            b = "blk%d" % (k - 1)
            nn.add(g[b], g["in%d" % k], g[b])
            self.enc[k - 1].backward(g["in%d" % k], sv["cnn%d" % k], g[b], 1.0)
        g["cnn1"] = torch.empty_like(v["cnn1"])
        self.down[0].backward(g["blk1"], sv["d1"], g["cnn1"], 0.0)
        g["blk0"] = torch.empty_like(v["blk0"])
        self.enc[0].backward(g["cnn1"], sv["cnn1"], g["blk0"], 0.0)
        self.stem.backward(g["blk0"], sv["stem"])
        if self._plan[0] is not None:
            self._plan[0].unfold()
        self._saved = None
        if hook is not None:
            hook("all")
