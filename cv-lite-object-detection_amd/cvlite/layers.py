"""Parameter store and layer objects of the explicit (tape-free) training graph.

All trainable fp32 parameters live in ONE flat device buffer (and so do their gradients and the
SGD momentum): the optimizer is one fused launch, data-parallel all-reduce is one bucketed
collective, and checkpoints are one tensor.  Each conv keeps bf16 packed copies of its weights
(forward and data-gradient layouts) refreshed after every update.  Names follow the Keras layer
names of the reference graph (e.g. `conv2_block1_1_conv/kernel`, `cls_layer_1/kernel`,
`logits_output_1/bias`) so a TF checkpoint can be mapped onto the store.
"""
import math

import os

import torch

from . import ops_nn as nn
from . import _lib

BF16 = torch.bfloat16
F32 = torch.float32


def act_dtype(precision=None):
    """Activation / activation-gradient storage type of a network: "bf16" (production: bf16
    storage, bf16 MFMA convs, fp32 accumulation and master weights) or "fp32" (the parity mode of
    SURVEY.md §8b: fp32 everywhere, for whole-graph parity with the reference's fp32 Keras graph).
    None reads CVL_PRECISION (default bf16)."""
    p = (precision or os.environ.get("CVL_PRECISION", "bf16")).lower()
    if p not in ("bf16", "fp32"):
        raise ValueError("precision must be 'bf16' or 'fp32'")
    return F32 if p == "fp32" else BF16


def glorot_uniform(fan_in, fan_out):
    lim = math.sqrt(6.0 / (fan_in + fan_out))

    def init(gen, shape):
        return (torch.rand(shape, generator=gen, dtype=torch.float64) * 2 - 1).mul_(lim).float()
    return init


def constant(v):
    def init(gen, shape):
        return torch.full(shape, float(v), dtype=torch.float32)
    return init


def same_pad(n, k, s):
    """TF 'same': output size and leading pad (asymmetric: extra pad goes bottom/right)."""
    out = -(-n // s)
    total = max((out - 1) * s + k - n, 0)
    return out, total // 2


class ParamStore(object):
    """Flat fp32 parameter / gradient / momentum buffers with named views."""

    def __init__(self):
        self.specs = []      # (name, shape, init)
        self.index = {}
        self.finalized = False
        self.act = BF16      # activation storage type of the network (act_dtype)

    def add(self, name, shape, init):
        assert not self.finalized and name not in self.index
        self.index[name] = len(self.specs)
        self.specs.append((name, tuple(shape), init))
        return name

    def finalize(self, device, seed=0):
        sizes = [int(math.prod(s)) for _, s, _ in self.specs]
        # 16-element alignment keeps every view 64-byte aligned
        offs, o = [], 0
        for n in sizes:
            offs.append(o)
            o += (n + 15) // 16 * 16
        self.numel = o
        self.flat = torch.zeros(o, dtype=torch.float32, device=device)
        self.grad = torch.zeros(o, dtype=torch.float32, device=device)
        self.mom = torch.zeros(o, dtype=torch.float32, device=device)
        gen = torch.Generator().manual_seed(seed)
        host = torch.zeros(o, dtype=torch.float32)
        self.offsets = {}
        for (name, shape, init), off, n in zip(self.specs, offs, sizes):
            host[off:off + n] = init(gen, shape).reshape(-1)
            self.offsets[name] = (off, n, shape)
        self.flat.copy_(host.to(device))
        self.finalized = True

    def p(self, name):
        off, n, shape = self.offsets[name]
        return self.flat[off:off + n].view(shape)

    def g(self, name):
        off, n, shape = self.offsets[name]
        return self.grad[off:off + n].view(shape)

    @property
    def n_params(self):
        return sum(n for (off, n, _) in self.offsets.values())

    def state_dict(self):
        return {name: self.p(name).detach().cpu().clone() for name in self.offsets}

    def load_state_dict(self, sd):
        for name, t in sd.items():
            self.p(name).copy_(t.to(self.flat.device))


class Conv(object):
    """Keras Conv2D (HWIO kernel, glorot-uniform init, zero bias) on the segmented MFMA conv.

    pad: 'same' (TF padding), 'valid', or an explicit leading pad int (ZeroPadding2D + valid)."""

    def __init__(self, store, name, k, cin, cout, stride=1, pad="same", bias=True, bias_init=0.0,
                 cin_k=None, npad=None, cout_pad=None, dgrad=True, init_fan_out=None, w_init=None):
        self.name, self.k, self.cin, self.cout, self.stride, self.pad = name, k, cin, cout, stride, pad
        self.cin_k = cin if cin_k is None else cin_k       # channels per tap in the forward pack
        self.npad = npad if npad is not None else max(32, (cout + 31) // 32 * 32)
        self.cout_pad = cout_pad if cout_pad is not None else self.npad   # dgrad pack K-channels
        self.cin_pad = (cin + 31) // 32 * 32
        self.has_bias = bias
        self.need_dgrad = dgrad
        fan_out = k * k * cout if init_fan_out is None else init_fan_out
        self.wname = store.add(name + "/kernel", (k, k, cin, cout),
                               w_init if w_init is not None else glorot_uniform(k * k * cin, fan_out))
        self.bname = store.add(name + "/bias", (cout,), constant(bias_init)) if bias else None
        self.store = store
        self.wf = self.wd = None

    # ---- geometry -----------------------------------------------------------------------------
    def out_hw(self, H, W):
        if self.pad == "same":
            (Ho, pt), (Wo, pl) = same_pad(H, self.k, self.stride), same_pad(W, self.k, self.stride)
        elif self.pad == "valid":
            Ho, Wo, pt, pl = (H - self.k) // self.stride + 1, (W - self.k) // self.stride + 1, 0, 0
        else:
            p = int(self.pad)
            Ho, Wo = (H + 2 * p - self.k) // self.stride + 1, (W + 2 * p - self.k) // self.stride + 1
            pt = pl = p
        return Ho, Wo, pt, pl

    # ---- parameters ---------------------------------------------------------------------------
    @property
    def w(self):
        return self.store.p(self.wname)

    @property
    def b(self):
        return self.store.p(self.bname) if self.bname else None

    @property
    def dw(self):
        return self.store.g(self.wname)

    @property
    def db(self):
        return self.store.g(self.bname) if self.bname else None

    def bias_arg(self):
        # every conv kernel reads bias[n] only for n < n_store (= cout): no padded copy needed
        return self.b if self.has_bias else None

    def alloc_packed(self):
        dev = self.store.flat.device
        K = self.k * self.k * self.cin_k
        if self.wf is None:      # packed operand copies in the activation type (fp32 in parity mode)
            self.wf = torch.empty((self.npad, K), dtype=self.store.act, device=dev)
            if self.need_dgrad:
                self.wd = torch.empty((self.cin_pad, self.k * self.k * self.cout_pad), dtype=self.store.act, device=dev)

    def pack_entry(self):
        """Row of an ops_nn.PackPlan (the batched re-pack of every conv)."""
        self.alloc_packed()
        return (self.w, self.k * self.k, self.cin, self.cout, self.cin_k, self.npad, self.wf,
                self.cin_pad, self.cout_pad, self.wd if self.need_dgrad else None)

    def pack_entries(self):
        return [self.pack_entry()]

    def pack(self):
        self.alloc_packed()
        nn.pack_conv_weights(self.w, self.k, self.k, self.cin, self.cout, self.cin_k, self.npad, self.wf,
                             self.cin_pad, self.cout_pad, self.wd if self.need_dgrad else None)

    # ---- descriptors ----------------------------------------------------------------------------
    def fwd_desc(self, B, segs, ld_dst=None, dst_coff=0, dst_f32=False, relu_out=False, relu_in=False,
                 beta=0.0, n_store=None, npad=None):
        """npad: the GEMM's N padding when it differs from the packed weights' (a weight gradient of a
        conv whose forward pack is wider than its dY rows, e.g. the FCOS heads)."""
        _, _, pt, pl = self.out_hw(segs[0]["Hs"], segs[0]["Ws"])
        return nn.make_desc(nn.FWD, B, self.cin_k, self.k, self.k, self.stride, pt, pl,
                            self.npad if npad is None else npad,
                            self.cout if n_store is None else n_store,
                            self.npad if ld_dst is None else ld_dst, segs, dst_coff=dst_coff,
                            dst_f32=dst_f32, relu_out=relu_out, relu_in=relu_in, beta=beta)

    def dgrad_desc(self, B, segs, ld_dst=None, beta=0.0):
        """segs in dgrad form: Hr/Wr = input map (dX), Hs/Ws = output map (dY)."""
        Ho, Wo = segs[0]["Hs"], segs[0]["Ws"]
        _, _, pt, pl = self.out_hw(segs[0]["Hr"], segs[0]["Wr"])
        return nn.make_desc(nn.DGRAD, B, self.cout_pad, self.k, self.k, self.stride, pt, pl, self.cin_pad,
                            self.cin, self.cin if ld_dst is None else ld_dst, segs, beta=beta)

    # ---- plain single-map helpers -----------------------------------------------------------------
    def fwd(self, x, B, H, W, out=None, stats=None, relu_out=False, relu_in=False):
        Ho, Wo, _, _ = self.out_hw(H, W)
        if out is None:
            out = torch.empty((B, Ho, Wo, self.cout), dtype=x.dtype, device=x.device)
        d = self.fwd_desc(B, [nn.seg(Ho, Wo, H, W, self.wf, self.bias_arg())], ld_dst=self.cout,
                          relu_out=relu_out, relu_in=relu_in)
        nn.conv_igemm(d, x, out, stats)
        return out, Ho, Wo

    def wgrad(self, x, dy, B, H, W, relu_in=False, dw=None, beta=0.0, bias=True):
        Ho, Wo, _, _ = self.out_hw(H, W)
        d = self.fwd_desc(B, [nn.seg(Ho, Wo, H, W, self.wf, None)], ld_dst=self.cout_pad_ld(dy),
                          relu_in=relu_in)
        if _wgb is not None and self.k in (1, 3) and beta == 0.0 and not relu_in and x.dtype == BF16:
            _wgb.append((d, x, dy, self.dw if dw is None else dw))     # launched by flush_wgrad_batch()
        else:
            nn.conv_wgrad(d, x, dy, self.dw if dw is None else dw, beta)
        if self.has_bias and bias:
            nn.bias_grad(dy, self.cout_pad_ld(dy), 0, self.cout, 0, Ho * Wo, Ho * Wo, B, self.db)

    def cout_pad_ld(self, dy):
        return int(dy.shape[-1])

    def dgrad(self, dy, B, H, W, out=None, beta=0.0, bn_next=None):
        """dX (= out, beta accumulate).  bn_next = (z, mean_rstd, gamma, beta, zeroed sums or None) of the BN -> ReLU unit
        whose dy this is: returns (dX, sums) with that BN backward's first pass fused into the
        epilogue (sums None when the launch could not fuse)."""
        Ho, Wo, _, _ = self.out_hw(H, W)
        if out is None:
            out = torch.empty((B, H, W, self.cin), dtype=dy.dtype, device=dy.device)
        d = self.dgrad_desc(B, [nn.seg(H, W, Ho, Wo, self.wd)], ld_dst=self.cin, beta=beta)
        if bn_next is None:
            nn.conv_igemm(d, dy, out)
            return out
        z, mr, ga, be, sums = bn_next[:5]
        y = bn_next[5] if len(bn_next) > 5 else None       # residual unit: mask y > 0 (bn_res_ctx)
        zero = sums is None
        if zero:
            sums = nn.bn_acc(B, self.cin, dy.device, zero=False)
        if y is not None:
            fused = nn.conv_igemm_dgrad_bnsum_res(d, dy, out, y, z, mr, ga, be, sums, zero=zero)
        else:
            fused = nn.conv_igemm_dgrad_bnsum(d, dy, out, z, mr, ga, be, sums, zero=zero)
        return out, (sums if fused else None)


# the BN backward's first pass fused into the producing data gradient (CVL_DISPATCH=no_bnsum_fuse: off,
# for A/B measurement)
FUSE_BNSUM = not _lib.dispatch("no_bnsum_fuse")
# ... and a residual unit's (BN3) first pass into the next block's conv1 data gradient (CVL_DISPATCH=no_bnsum_res: off)
FUSE_BNSUM_RES = FUSE_BNSUM and not _lib.dispatch("no_bnsum_res")
# ... and a projection shortcut BN's first pass into the residual unit's second pass (no_sc_bnsum: off)
FUSE_SC_BNSUM = FUSE_BNSUM_RES and not _lib.dispatch("no_sc_bnsum")

# Batched weight gradients (round 6; CVL_DISPATCH=no_wgrad_batch: off).  Inside `with wgrad_batch():`
# Conv.wgrad collects its 1x1 / 3x3 bf16 problems (keeping their x / dy alive) instead of launching
# them; the exit (or flush_wgrad_batch()) hands all of them to ONE cvl_conv_wgrad_batch call: one
# launch per ResNet stage and kernel instead of one per conv, with fewer splits per problem.
WGRAD_BATCH = not _lib.dispatch("no_wgrad_batch")
_wgb = None


class wgrad_batch(object):
    def __enter__(self):
        global _wgb
        self.own = _wgb is None and WGRAD_BATCH
        if self.own:
            _wgb = []
        return self

    def __exit__(self, exc_type, *exc):
        global _wgb
        if self.own:
            try:
                if exc_type is None:
                    flush_wgrad_batch()
            finally:
                _wgb = None
        return False


def conv_wgrad(d, x, dy, dw):
    """nn.conv_wgrad (beta 0), collected instead while a wgrad_batch is open (bf16 operands)."""
    if _wgb is not None and x.dtype == BF16:
        _wgb.append((d, x, dy, dw))
    else:
        nn.conv_wgrad(d, x, dy, dw)


def flush_wgrad_batch():
    """Launch the collected weight gradients (no-op outside wgrad_batch / when none)."""
    if _wgb:
        items = list(_wgb)
        del _wgb[:]
        nn.conv_wgrad_batch([i[0] for i in items], [i[1] for i in items], [i[2] for i in items],
                            [i[3] for i in items])


class StatsArena(object):
    """One zeroed buffer holding the (sum, sumsq) BN statistics of every conv of a forward pass as
    BN accumulators (nn.bn_acc: [B][C][2][S] in the library's mode), one memset per step instead of
    one per BN.  n_stats = statistics (2 per image and channel) it can hand out."""

    def __init__(self, n_stats, device):
        self.slots = nn.acc_slots()
        self.buf = torch.zeros(n_stats * self.slots, dtype=torch.int64, device=device)
        self.off = 0

    def take(self, B, c):
        n = B * c * 2 * self.slots
        assert self.off + n <= self.buf.numel(), "stats arena too small"
        v = self.buf[self.off:self.off + n].view(B, c, 2, self.slots)
        self.off += n
        return v


class BatchNorm(object):
    """Keras BatchNormalization(axis=-1) in training mode with per-image statistics."""

    def __init__(self, store, name, c, eps=1.001e-5, momentum=0.99):
        self.name, self.c, self.eps, self.momentum = name, c, eps, momentum
        self.gname = store.add(name + "/gamma", (c,), constant(1.0))
        self.bname = store.add(name + "/beta", (c,), constant(0.0))
        self.store = store
        self.run_mean = self.run_var = None

    def init_buffers(self, device):
        self.run_mean = torch.zeros(self.c, dtype=torch.float32, device=device)
        self.run_var = torch.ones(self.c, dtype=torch.float32, device=device)

    def moving_mean_rstd(self, B):
        """Keras training=False: normalise with the moving statistics (same for every image),
        as [B][C][2] (mean, rstd) for cvl_bn_apply."""
        mr = torch.empty((B, self.c, 2), dtype=torch.float32, device=self.run_mean.device)
        mr[:, :, 0] = self.run_mean
        mr[:, :, 1] = torch.rsqrt(self.run_var + self.eps)
        return mr

    def normalize(self, z, stats, B, HW, relu, residual=None, train=True, residual_bn=None):
        """y = BN(z) (+ residual) (ReLU): training mode from the conv's fused per-image statistics
        (and the moving-average update), inference mode from the moving statistics.
        residual_bn: a deferred unit's (z, stats, mean_rstd out, BatchNorm) -- the residual is that
        BN's output, formed in the same launch (cvl_bn_finalize_apply_bnres), never stored."""
        y = torch.empty_like(z)
        if train and residual_bn is not None:
            rz, rstats, rmr, rbn = residual_bn
            mr = torch.empty((B, self.c, 2), dtype=torch.float32, device=z.device)
            nn.bn_finalize_apply_bnres(stats, mr, self.run_mean, self.run_var, z, self.gamma, self.beta, rstats, rmr,
                                       rbn.run_mean, rbn.run_var, rz, rbn.gamma, rbn.beta, rbn.eps, rbn.momentum, y,
                                       B, HW, self.c, relu, self.eps, self.momentum)
        elif train:
            mr = torch.empty((B, self.c, 2), dtype=torch.float32, device=z.device)
            nn.bn_finalize_apply(stats, mr, self.run_mean, self.run_var, z, self.gamma, self.beta, residual, y, B,
                                 HW, self.c, relu, self.eps, self.momentum)
        else:
            mr = self.moving_mean_rstd(B)
            nn.bn_apply(z, mr, self.gamma, self.beta, residual, y, B, HW, self.c, relu)
        return y, mr

    @property
    def gamma(self):
        return self.store.p(self.gname)

    @property
    def beta(self):
        return self.store.p(self.bname)


class ConvBN(object):
    """conv -> BN (-> + residual) (-> ReLU): the Keras ResNet50 unit."""

    def __init__(self, store, name, k, cin, cout, stride=1, pad="same", dgrad=True, cin_k=None,
                 bn_name=None):
        self.conv = Conv(store, name + "_conv" if bn_name is None else name, k, cin, cout, stride, pad,
                         bias=True, dgrad=dgrad, cin_k=cin_k)
        self.bn = BatchNorm(store, (name + "_bn") if bn_name is None else bn_name, cout)

    def forward(self, x, B, H, W, relu=True, residual=None, train=True, arena=None, defer=False,
                residual_bn=None):
        """defer (training, no ReLU): the BN is not applied here -- returns (pending, saved) where
        pending = (z, stats, mean_rstd, BatchNorm) is the consumer's residual_bn, which forms this
        unit's output and finalize inside its own BN launch (the projection shortcut).  Its saved
        y is None: the backward of such a unit reads z only (no ReLU mask, no residual)."""
        c = self.conv.cout
        Ho, Wo, _, _ = self.conv.out_hw(H, W)
        stats = None
        if train:
            stats = arena.take(B, c) if arena is not None else nn.bn_acc(B, c, x.device)
        z, _, _ = self.conv.fwd(x, B, H, W, stats=stats)
        if defer:
            assert train and residual is None and not relu, "defer: the projection shortcut's BN only"
            mr = torch.empty((B, c, 2), dtype=torch.float32, device=z.device)
            return (z, stats, mr, self.bn), (x, z, None, mr, B, H, W, Ho, Wo, relu, False)
        y, mr = self.bn.normalize(z, stats, B, Ho * Wo, relu, residual=residual, train=train,
                                  residual_bn=residual_bn)
        return y, (x, z, y, mr, B, H, W, Ho, Wo, relu, residual is not None or residual_bn is not None)

    def bn_next_ctx(self, saved, arena=None):
        """What a producer of this unit's dy needs to fuse the BN backward's first pass into its
        data-gradient epilogue (conv_igemm_dgrad_bnsum); None unless BN -> ReLU without residual.
        The sums buffer comes zeroed from the step's StatsArena when one is given."""
        x, z, y, mr, B, H, W, Ho, Wo, relu, has_res = saved
        if not relu or has_res or not FUSE_BNSUM or z.dtype != BF16:      # (fp32 parity mode: two passes)
            return None
        return (z, mr, self.bn.gamma, self.bn.beta, arena.take(B, self.bn.c) if arena is not None else None)

    def bn_res_ctx(self, saved, arena=None):
        """As bn_next_ctx for a residual unit (BN -> + shortcut -> ReLU, the bottleneck's conv3): its dy
        is completed by the next block's first 1x1 data gradient accumulating into the block-output
        gradient, whose epilogue then forms this BN backward's first pass with the mask y > 0."""
        x, z, y, mr, B, H, W, Ho, Wo, relu, has_res = saved
        if not relu or not has_res or not FUSE_BNSUM_RES or z.dtype != BF16:
            return None
        return (z, mr, self.bn.gamma, self.bn.beta, arena.take(B, self.bn.c) if arena is not None else None, y)

    def backward(self, dy, saved, dx_out=None, dx_beta=0.0, g_out=None, need_dx=True, sums=None, bn_next=None,
                 sc_fuse=None):
        """dz = BN backward of dy, the conv's weight gradient, and (need_dx) its data gradient.
        sums: this unit's BN-backward first pass, already formed by the producer of dy (skip it).
        bn_next: the NEXT unit's bn_next_ctx -- the data gradient then also forms that unit's first
        pass, and the return value is (dx, sums or None) instead of dx.
        sc_fuse: (z_sc, mean_rstd_sc, sc_sums) of a projection shortcut whose dy is g_out: with the
        fused first pass (sums given) the second pass also forms the shortcut BN's first pass into
        sc_sums; self.sc_fused then says whether it did."""
        x, z, y, mr, B, H, W, Ho, Wo, relu, has_res = saved
        c = self.conv.cout
        dz = torch.empty_like(z)
        st = self.bn.store
        self.sc_fused = False
        if sums is not None and has_res and sc_fuse is not None and g_out is not None:
            assert relu                                  # + the projection shortcut BN's first pass
            nn.bn_backward_res_sums_sc(dy, y, z, mr, self.bn.gamma, sums, dz, g_out, st.g(self.bn.gname),
                                       st.g(self.bn.bname), sc_fuse[0], sc_fuse[1], sc_fuse[2], B, Ho * Wo, c,
                                       conv_dbias=self.conv.db)
            self.sc_fused = True
        elif sums is not None and has_res:               # residual unit, first pass fused upstream
            assert relu
            nn.bn_backward_res_sums(dy, y, z, mr, self.bn.gamma, sums, dz, g_out, st.g(self.bn.gname),
                                    st.g(self.bn.bname), B, Ho * Wo, c, conv_dbias=self.conv.db)
        elif sums is not None and not relu:              # BN without ReLU (the shortcut), first pass done
            nn.bn_backward_sums(dy, z, mr, self.bn.gamma, sums, dz, st.g(self.bn.gname), st.g(self.bn.bname),
                                B, Ho * Wo, c, conv_dbias=self.conv.db)
        elif sums is not None:                           # first pass fused upstream
            assert relu and not has_res and g_out is None
            nn.bn_backward_relu_sums(dy, z, mr, self.bn.gamma, self.bn.beta, sums, dz, st.g(self.bn.gname),
                                     st.g(self.bn.bname), B, Ho * Wo, c, conv_dbias=self.conv.db)
        elif relu and not has_res and g_out is None:    # ReLU mask rebuilt from z: y is not read
            nn.bn_backward_relu(dy, z, mr, self.bn.gamma, self.bn.beta, dz, st.g(self.bn.gname),
                                st.g(self.bn.bname), B, Ho * Wo, c, conv_dbias=self.conv.db)
        elif sc_fuse is not None and relu and has_res and g_out is not None and y is not None:
            # both passes here, the second one also forming the projection shortcut BN's first pass
            nn.bn_backward_sc(dy, y, z, mr, self.bn.gamma, dz, g_out, st.g(self.bn.gname), st.g(self.bn.bname),
                              sc_fuse[0], sc_fuse[1], sc_fuse[2], B, Ho * Wo, c, conv_dbias=self.conv.db)
            self.sc_fused = True
        else:
            # the mask comes from y: a deferred unit (saved y None) has no ReLU (ConvBN.forward)
            assert y is not None or not relu, "ReLU unit without its saved output"
            nn.bn_backward(dy, y if relu else None, z, mr, self.bn.gamma, dz, g_out, st.g(self.bn.gname),
                           st.g(self.bn.bname), B, Ho * Wo, c, conv_dbias=self.conv.db)
        self.conv.wgrad(x, dz, B, H, W, bias=False)
        if not need_dx:
            return None
        if bn_next is None:
            return self.conv.dgrad(dz, B, H, W, out=dx_out, beta=dx_beta)
        # beta-accumulating producers take the residual (y-mask) form only (bn_res_ctx)
        assert dx_beta == 0.0 or len(bn_next) > 5
        dx = self.conv.dgrad(dz, B, H, W, out=dx_out, beta=dx_beta, bn_next=bn_next)
        return dx
