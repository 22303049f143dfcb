"""Device ops of the conv/BN/FPN training graph: thin torch-tensor wrappers over the C ABI
(include/cvlite.h).  Tensors are raw storage (bf16 activations NHWC, fp32 params); no autograd.

fp32 parity mode (CVL_PRECISION=fp32, layers.act_dtype): the same wrappers take fp32 activations
and dispatch on the tensor dtype -- convolutions through cvl_conv_desc.prec = CVL_PREC_F32, the
memory-bound ops through their *_f32 entry points."""
import ctypes

import torch

from . import _lib
from ._lib import ptr, stream

c_int, c_int64, c_float, c_void_p = ctypes.c_int, ctypes.c_int64, ctypes.c_float, ctypes.c_void_p
BF16 = torch.bfloat16
FWD, DGRAD = 0, 1
MAX_SEG = 10        # CVL_CONV_MAX_SEG (include/cvlite.h): cls + reg towers x 5 levels in one launch


class ConvSeg(ctypes.Structure):
    _fields_ = [("Hr", c_int), ("Wr", c_int), ("Hs", c_int), ("Ws", c_int),
                ("src_base", c_int64), ("src_img", c_int64), ("dst_base", c_int64), ("dst_img", c_int64),
                ("w", c_void_p), ("bias", c_void_p)]


class ConvDesc(ctypes.Structure):
    _fields_ = [("mode", c_int), ("B", c_int), ("Cin", c_int), ("KH", c_int), ("KW", c_int),
                ("stride", c_int), ("pad_t", c_int), ("pad_l", c_int), ("Npad", c_int),
                ("n_store", c_int), ("ld_dst", c_int), ("dst_coff", c_int), ("dst_f32", c_int),
                ("relu_out", c_int), ("relu_in", c_int), ("beta", c_float), ("nseg", c_int),
                ("seg", ConvSeg * MAX_SEG), ("prec", c_int)]


PREC_BF16, PREC_F32 = 0, 1      # cvl_conv_desc.prec


def _is_f32(t):
    return t is not None and t.dtype == torch.float32


def _prec(desc, src):
    """The descriptor's operand precision follows its source tensor (bf16: production MFMA path;
    fp32: the parity mode, whose weights are packed fp32)."""
    desc.prec = PREC_F32 if _is_f32(src) else PREC_BF16


def seg(Hr, Wr, Hs, Ws, w, bias=None, src_base=0, src_img=None, dst_base=0, dst_img=None):
    return dict(Hr=Hr, Wr=Wr, Hs=Hs, Ws=Ws, w=w, bias=bias, src_base=src_base,
                src_img=Hs * Ws if src_img is None else src_img, dst_base=dst_base,
                dst_img=Hr * Wr if dst_img is None else dst_img)


def make_desc(mode, B, Cin, KH, KW, stride, pad_t, pad_l, Npad, n_store, ld_dst, segs, dst_coff=0,
              dst_f32=False, relu_out=False, relu_in=False, beta=0.0):
    d = ConvDesc()
    d.mode, d.B, d.Cin, d.KH, d.KW = mode, B, Cin, KH, KW
    d.stride, d.pad_t, d.pad_l, d.Npad, d.n_store = stride, pad_t, pad_l, Npad, n_store
    d.ld_dst, d.dst_coff, d.dst_f32 = ld_dst, dst_coff, int(bool(dst_f32))
    d.relu_out, d.relu_in, d.beta = int(bool(relu_out)), int(bool(relu_in)), float(beta)
    d.nseg = len(segs)
    keep = []
    for i, s in enumerate(segs):
        q = d.seg[i]
        q.Hr, q.Wr, q.Hs, q.Ws = s["Hr"], s["Wr"], s["Hs"], s["Ws"]
        q.src_base, q.src_img, q.dst_base, q.dst_img = s["src_base"], s["src_img"], s["dst_base"], s["dst_img"]
        q.w = s["w"].data_ptr()
        q.bias = s["bias"].data_ptr() if s["bias"] is not None else None
        keep.append((s["w"], s["bias"]))
    d._keep = keep   # keep weight tensors alive as long as the descriptor
    return d


def conv_igemm(desc, src, dst, stats=None):
    _prec(desc, src)
    n = int(_lib.load().cvl_conv_igemm_workspace_size(ctypes.byref(desc)))
    ws = torch.empty(n, dtype=torch.uint8, device=src.device) if n > 16 else None
    _lib.call("cvl_conv_igemm", ctypes.byref(desc), ptr(src), ptr(dst), acc_ptr(stats), ptr(ws),
              n if ws is not None else 0, stream())


def conv_igemm_relu_mask(desc, src, dst, y):
    """Data gradient through a ReLU: dst = dgrad(src) * (y > 0), y laid out as dst (the X32 register
    epilogue applies the mask; other kernels get the separate ReLU backward).  Bit-identical to
    conv_igemm + relu_backward."""
    _prec(desc, src)
    n = int(_lib.load().cvl_conv_igemm_workspace_size(ctypes.byref(desc)))
    ws = torch.empty(n, dtype=torch.uint8, device=src.device) if n > 16 else None
    _lib.call("cvl_conv_igemm_relu_mask", ctypes.byref(desc), ptr(src), ptr(dst), ptr(y), ptr(ws),
              n if ws is not None else 0, stream())


def probe_arm(slot):
    """Time the next conv_igemm launch from inside if it runs the tower kernel (slot: uint64 [4]
    device tensor, zeroed; cvl_probe_arm)."""
    _lib.call("cvl_probe_arm", ptr(slot))


def probe_seconds(slot):
    """Mean seconds per probed launch over every probed launch since the slot was zeroed, and the count."""
    hz = _lib.load().cvl_probe_clock_hz()
    ticks, n = (int(v) for v in slot[1:3].cpu().tolist())
    return (ticks / n / hz if n and hz > 0 else None), n


# workspaces of the weight gradients whose split reductions are pending (cvl_wgrad_defer); None =
# deferral off.  Kept alive until the flush has been enqueued.
_wgrad_pending = None


class deferred_wgrad(object):
    """with deferred_wgrad(): the split-M weight-gradient reductions of the block are batched into
    one launch per wgrad_flush() (and one at exit); dW is final only after the flush."""

    def __enter__(self):
        global _wgrad_pending
        self.outer = _wgrad_pending is not None
        if not self.outer:
            _wgrad_pending = []
            _lib.call("cvl_wgrad_defer", 1, stream())
        return self

    def __exit__(self, *exc):
        global _wgrad_pending
        if not self.outer:
            _lib.call("cvl_wgrad_defer", 0, stream())
            _wgrad_pending = None
        return False


def wgrad_flush():
    """Reduce every pending weight gradient (no-op when none / deferral off)."""
    if _wgrad_pending is not None:
        _lib.call("cvl_wgrad_flush", stream())
        del _wgrad_pending[:]


def conv_wgrad(desc, x, dy, dw, beta=0.0):
    _prec(desc, x)
    lib = _lib.load()
    n = int(lib.cvl_conv_wgrad_workspace_size(ctypes.byref(desc)))
    ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
    _lib.call("cvl_conv_wgrad", ctypes.byref(desc), ptr(x), ptr(dy), ptr(dw), float(beta), ptr(ws),
              ws.numel(), stream())
    if _wgrad_pending is not None:
        _wgrad_pending.append(ws)


def conv_wgrad_grouped(desc, x, dy, dws, beta=0.0):
    """Weight gradients of `len(dws)` segment groups in one launch (cvl_conv_wgrad_grouped): the
    descriptor's segments split into equal consecutive groups, group g summed into dws[g]."""
    _prec(desc, x)
    lib = _lib.load()
    n = int(lib.cvl_conv_wgrad_grouped_workspace_size(ctypes.byref(desc), len(dws)))
    ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
    arr = (c_void_p * len(dws))(*[t.data_ptr() for t in dws])
    _lib.call("cvl_conv_wgrad_grouped", ctypes.byref(desc), len(dws), ptr(x), ptr(dy), arr, float(beta), ptr(ws),
              ws.numel(), stream())
    if _wgrad_pending is not None:
        _wgrad_pending.append(ws)


def conv_wgrad_batch(descs, xs, dys, dws, beta=0.0):
    """Weight gradients of several convolutions in one call (cvl_conv_wgrad_batch): every 1x1 bf16
    problem of the list shares one launch, the rest run one by one -- as conv_wgrad for each."""
    n = len(descs)
    if n == 0:
        return
    for d, x in zip(descs, xs):
        _prec(d, x)
    lib = _lib.load()
    darr = (c_void_p * n)(*[ctypes.addressof(d) for d in descs])
    nb = int(lib.cvl_conv_wgrad_batch_workspace_size(darr, n))
    ws = torch.empty(max(nb, 16), dtype=torch.uint8, device=xs[0].device)
    xa = (c_void_p * n)(*[t.data_ptr() for t in xs])
    ya = (c_void_p * n)(*[t.data_ptr() for t in dys])
    wa = (c_void_p * n)(*[t.data_ptr() for t in dws])
    _lib.call("cvl_conv_wgrad_batch", darr, n, xa, ya, wa, float(beta), ptr(ws), ws.numel(), stream())
    if _wgrad_pending is not None:
        _wgrad_pending.append(ws)


def pack_conv_weights(w_hwio, KH, KW, Cin, Cout, Cin_k, Npad, w_fwd, Cin_pad=0, Cout_pad=0, w_dgrad=None):
    _lib.call("cvl_pack_conv_weights", ptr(w_hwio), KH, KW, Cin, Cout, Cin_k, Npad, ptr(w_fwd),
              Cin_pad, Cout_pad, ptr(w_dgrad), stream())


class PackItem(ctypes.Structure):
    _fields_ = [("w", c_void_p), ("w_fwd", c_void_p), ("w_dgrad", c_void_p), ("KHW", c_int), ("Cin", c_int),
                ("Cout", c_int), ("Cin_k", c_int), ("Npad", c_int), ("Cin_pad", c_int), ("Cout_pad", c_int),
                ("f32_out", c_int)]


class PackPlan(object):
    """Device tables for cvl_pack_conv_weights_multi: every conv's fwd/dgrad bf16 re-pack in one
    launch.  entries: (w_hwio fp32, KHW, Cin, Cout, Cin_k, Npad, w_fwd, Cin_pad, Cout_pad, w_dgrad)."""

    def __init__(self, entries, device):
        items = (PackItem * len(entries))()
        tiles = []
        self._keep = []
        for i, (w, khw, cin, cout, cin_k, npad, wf, cin_pad, cout_pad, wd) in enumerate(entries):
            it = items[i]
            it.w = w.data_ptr()
            it.w_fwd = wf.data_ptr() if wf is not None else None
            it.w_dgrad = wd.data_ptr() if wd is not None else None
            it.KHW, it.Cin, it.Cout, it.Cin_k, it.Npad = khw, cin, cout, cin_k, npad
            it.Cin_pad, it.Cout_pad = (cin_pad, cout_pad) if wd is not None else (0, 0)
            it.f32_out = int(_is_f32(wf if wf is not None else wd))       # parity-mode fp32 packs
            self._keep.append((w, wf, wd))
            ci_hi = max(cin_k, it.Cin_pad)
            co_hi = max(npad, it.Cout_pad)
            for tap in range(khw):
                for ci0 in range(0, ci_hi, 64):
                    for co0 in range(0, co_hi, 64):
                        tiles.append((i, tap, ci0, co0))
        raw = bytes(items)
        self.host_items = items          # geometry of every entry (host copy of the device table)
        self.items = torch.frombuffer(bytearray(raw), dtype=torch.uint8).to(device)
        self.tiles = torch.tensor(tiles, dtype=torch.int32, device=device)
        self.ntiles = len(tiles)

    def run(self):
        _lib.call("cvl_pack_conv_weights_multi", ptr(self.items), ptr(self.tiles), self.ntiles, stream())


def stem_conv7x7s2(img, w_packed, bias, z, stats=None):
    """ResNet conv1 from the fp32 NHWC image (cvl_stem_conv7x7s2): z [B][Ho][Wo][64] bf16 (+ BN stats)."""
    B, H, W, C = img.shape
    assert C == 3 and img.dtype == torch.float32 and img.is_contiguous()
    _lib.call("cvl_stem_conv7x7s2", ptr(img), B, H, W, ptr(w_packed), ptr(bias), ptr(z), acc_ptr(stats), stream())


def stem_wgrad(img, dz, dw, beta=0.0):
    """dw [192][64] fp32 (padded K order, cvl_stem_wgrad) = beta*dw + the stem's weight gradient."""
    B, H, W, _ = img.shape
    n = int(_lib.load().cvl_stem_wgrad_workspace_size(B, H, W))
    ws = torch.empty(max(n, 16), dtype=torch.uint8, device=img.device)
    _lib.call("cvl_stem_wgrad", ptr(img), B, H, W, ptr(dz), ptr(dw), float(beta), ptr(ws), ws.numel(), stream())
    if _wgrad_pending is not None:
        _wgrad_pending.append(ws)


def im2col(x, KH, KW, stride, pad_t, pad_l, Ho, Wo, Kp, out):
    B, H, W, C = x.shape
    _lib.call("cvl_im2col", ptr(x), B, H, W, C, KH, KW, stride, pad_t, pad_l, Ho, Wo, Kp, ptr(out), stream())


# BN statistics accumulators (include/cvlite.h "BN accumulators"; csrc/bn_acc.h): a (B, C) buffer
# is int64 [B][C][2][S].  S = 1 by default (one float64 per statistic, fp64 atomics); S = ACC_SLOTS
# in the exact mode (7 exponent bins + a non-finite count: bit-identical whatever order the atomics
# land in), chosen with set_bn_exact(True) -- or CVL_BN_EXACT=1 -- before any buffer is made.
ACC_SLOTS = 8
ACC_BINS, ACC_W, ACC_E0 = 7, 22, 27


_SLOTS = [None]          # cached cvl_bn_acc_slots() of the current mode


def set_bn_exact(on):
    """Library-wide BN accumulator mode (cvl_bn_set_exact); buffers made before a switch are invalid
    -- and rejected: every entry point that takes a BN accumulator buffer checks its slot dimension
    against the mode (acc_ptr)."""
    _lib.call("cvl_bn_set_exact", 1 if on else 0)
    _SLOTS[0] = None


def acc_slots():
    """uint64 slots per statistic of the current mode (cvl_bn_acc_slots): 1 or ACC_SLOTS."""
    if _SLOTS[0] is None:
        _SLOTS[0] = int(_lib.load().cvl_bn_acc_slots())
    return _SLOTS[0]


def acc_ptr(t):
    """Pointer of a BN accumulator buffer ([..., 2, S] int64, as bn_acc / StatsArena make them) after
    checking S against the library's current mode: a buffer made in the other mode would be indexed
    as [..][2][8] vs [..][2][1] by the kernels (out-of-bounds atomics), so it is refused here."""
    if t is None:
        return None
    if t.dtype != torch.int64 or t.dim() < 2 or int(t.shape[-1]) != acc_slots():
        raise _lib.CvlError("BN accumulator buffer of shape %s / %s does not match the current mode (%d slots "
                            "per statistic): made before a cvl_bn_set_exact switch?" % (tuple(t.shape), t.dtype,
                                                                                     acc_slots()))
    return ptr(t)


def bn_acc(B, C, device, zero=True):
    """A (B, C) BN statistics buffer ((sum, sumsq) or (sum g, sum g*xhat)) for the producing kernels."""
    f = torch.zeros if zero else torch.empty
    return f((B, C, 2, acc_slots()), dtype=torch.int64, device=device)


def bn_acc_value(acc):
    """float64 values [..., 2] of a BN accumulator buffer [..., 2, ACC_SLOTS] (cvl_bn_acc_decode)."""
    acc = acc.contiguous()
    out = torch.empty(acc.shape[:-1], dtype=torch.float64, device=acc.device)
    _lib.call("cvl_bn_acc_decode", acc_ptr(acc), ptr(out), out.numel(), stream())
    return out


def _acc_add_f32(bins, f):
    """bins[..., k] += the exact integer of float32 f in bin k (bn_acc.h acc_split), torch ops."""
    u = f.contiguous().view(torch.int32).to(torch.int64) & 0xffffffff
    e = (u >> 23) & 0xff
    r = e - ACC_E0
    k = torch.div(r.clamp(min=0), ACC_W, rounding_mode="floor")
    bad = (e == 255) | ((e != 0) & (r >= 0) & (k >= ACC_BINS))
    ok = (e != 0) & (r >= 0) & (k < ACC_BINS)
    m = ((u & 0x7fffff) | 0x800000) << (r - k * ACC_W).clamp(min=0)
    v = torch.where((u >> 31) == 1, -m, m)
    bins.scatter_add_(-1, torch.where(ok, k, 0).unsqueeze(-1), torch.where(ok, v, 0).unsqueeze(-1))
    bins[..., ACC_BINS] += bad.to(torch.int64)


def bn_acc_encode(values, exact=None):
    """float64 statistic values [..., 2] -> an accumulator buffer [..., 2, S] of the library's mode
    (exact=None) or of the given one: the float64 bits (S = 1), or each value split into three float32
    pieces added into the bins as bn_acc.h acc_add_f64 (S = ACC_SLOTS).  For callers that hold the
    sums already."""
    v = values.to(torch.float64)
    if exact is None:
        exact = acc_slots() == ACC_SLOTS
    if not exact:
        return v.contiguous().view(torch.int64).unsqueeze(-1).clone()
    out = torch.zeros(v.shape + (ACC_SLOTS,), dtype=torch.int64, device=v.device)
    hi = v.to(torch.float32)
    r = v - hi.double()
    mid = r.to(torch.float32)
    lo = (r - mid.double()).to(torch.float32)
    for piece in (hi, mid, lo):
        _acc_add_f32(out, piece)
    return out


def bn_finalize(stats, mean_rstd, run_mean, run_var, B, C, HW, eps, momentum):
    _lib.call("cvl_bn_finalize", acc_ptr(stats), ptr(mean_rstd), ptr(run_mean), ptr(run_var), B, C, HW,
              float(eps), float(momentum), stream())


def bn_apply(z, mean_rstd, gamma, beta, residual, y, B, HW, C, relu):
    _lib.call("cvl_bn_apply_f32" if _is_f32(z) else "cvl_bn_apply", ptr(z), ptr(mean_rstd), ptr(gamma), ptr(beta), ptr(residual), ptr(y),
              B, HW, C, int(relu), stream())          # relu: 0 none, 1 ReLU, 2 ReLU6


def bn_finalize_apply(stats, mean_rstd, run_mean, run_var, z, gamma, beta, residual, y, B, HW, C, relu, eps,
                      momentum):
    _lib.call("cvl_bn_finalize_apply_f32" if _is_f32(z) else "cvl_bn_finalize_apply", acc_ptr(stats), ptr(mean_rstd), ptr(run_mean), ptr(run_var), ptr(z), ptr(gamma),
              ptr(beta), ptr(residual), ptr(y), B, HW, C, int(relu), float(eps), float(momentum), stream())


def bn_finalize_apply_bnres(stats, mean_rstd, run_mean, run_var, z, gamma, beta, res_stats, res_mean_rstd,
                            res_run_mean, res_run_var, res_z, res_gamma, res_beta, res_eps, res_momentum, y, B,
                            HW, C, relu, eps, momentum):
    """y = act(BN(z) + BN_res(res_z)) with both finalizes in one launch (cvl_bn_finalize_apply_bnres)."""
    _lib.call("cvl_bn_finalize_apply_bnres", acc_ptr(stats), ptr(mean_rstd), ptr(run_mean), ptr(run_var), ptr(z),
              ptr(gamma), ptr(beta), acc_ptr(res_stats), ptr(res_mean_rstd), ptr(res_run_mean), ptr(res_run_var),
              ptr(res_z), ptr(res_gamma), ptr(res_beta), float(res_eps), float(res_momentum), ptr(y), B, HW, C,
              int(relu), float(eps), float(momentum), stream())


def bn_backward(dy, y_relu, z, mean_rstd, gamma, dz, g_out, dgamma, dbeta, B, HW, C, beta_acc=0.0,
                conv_dbias=None):
    if _is_f32(dy):
        return bn_backward_f32(dy, y_relu, z, mean_rstd, gamma, None, dz, g_out, dgamma, dbeta, B, HW, C, beta_acc,
                               conv_dbias)
    n = int(_lib.load().cvl_bn_backward_workspace_size(B, HW, C))
    ws = torch.empty(n, dtype=torch.uint8, device=dy.device)
    _lib.call("cvl_bn_backward", ptr(dy), ptr(y_relu), ptr(z), ptr(mean_rstd), ptr(gamma), ptr(ws), n,
              ptr(dz), ptr(g_out), ptr(dgamma), ptr(dbeta), float(beta_acc), ptr(conv_dbias), B, HW, C,
              stream())


def bn_backward_f32(dy, y_relu, z, mean_rstd, gamma, bn_beta, dz, g_out, dgamma, dbeta, B, HW, C, beta_acc=0.0,
                    conv_dbias=None, act_hi=float("inf")):
    """fp32 parity form of bn_backward (y_relu given) / bn_backward_relu (bn_beta given)."""
    n = int(_lib.load().cvl_bn_backward_f32_workspace_size(B, C))
    ws = torch.empty(n, dtype=torch.uint8, device=dy.device)
    _lib.call("cvl_bn_backward_f32", ptr(dy), ptr(y_relu), ptr(z), ptr(mean_rstd), ptr(gamma), ptr(bn_beta), ptr(ws), n,
              ptr(dz), ptr(g_out), ptr(dgamma), ptr(dbeta), float(beta_acc), ptr(conv_dbias), float(act_hi), B, HW, C,
              stream())


def bn_backward_relu6(dy, z, mean_rstd, gamma, beta, dz, dgamma, dbeta, B, HW, C, beta_acc=0.0, conv_dbias=None):
    """bn_backward of a BN -> ReLU6 unit without a residual (mask 0 < bn(z) < 6 rebuilt from z)."""
    n = int(_lib.load().cvl_bn_backward_workspace_size(B, HW, C))
    ws = torch.empty(n, dtype=torch.uint8, device=dy.device)
    _lib.call("cvl_bn_backward_relu6", ptr(dy), ptr(z), ptr(mean_rstd), ptr(gamma), ptr(beta), ptr(ws), n, ptr(dz),
              ptr(dgamma), ptr(dbeta), float(beta_acc), ptr(conv_dbias), B, HW, C, stream())


def _dw_shapes(x, Ho, Wo):
    B, H, W, C = x.shape
    return B, H, W, C, Ho, Wo


def depthwise_fwd(x, w, y, k, stride, pad_t, pad_l):
    """Keras DepthwiseConv2D: x [B,H,W,C] bf16, w [k,k,C(,1)] fp32 -> y [B,Ho,Wo,C] bf16."""
    B, H, W, C = x.shape
    Ho, Wo = y.shape[1], y.shape[2]
    _lib.call("cvl_depthwise_fwd", ptr(x), ptr(w), ptr(y), B, H, W, C, int(k), int(stride), int(pad_t), int(pad_l),
              Ho, Wo, stream())


def depthwise_dgrad(dy, w, dx, k, stride, pad_t, pad_l, beta=0.0):
    B, H, W, C = dx.shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    _lib.call("cvl_depthwise_dgrad", ptr(dy), ptr(w), ptr(dx), B, H, W, C, int(k), int(stride), int(pad_t),
              int(pad_l), Ho, Wo, float(beta), stream())


def depthwise_wgrad(x, dy, dw, k, stride, pad_t, pad_l, beta=0.0):
    B, H, W, C = x.shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    n = int(_lib.load().cvl_depthwise_wgrad_workspace_size(B, Ho, Wo, C, int(k)))
    ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
    _lib.call("cvl_depthwise_wgrad", ptr(x), ptr(dy), ptr(dw), float(beta), B, H, W, C, int(k), int(stride),
              int(pad_t), int(pad_l), Ho, Wo, ptr(ws), ws.numel(), stream())


def conv_igemm_dgrad_bnsum(desc, src, dst, z, mean_rstd, gamma, beta, sums, act_hi=float("inf"), zero=True):
    """DGRAD conv whose epilogue also forms the next BN's backward first pass into `sums`
    (bn_acc [B][C][2][S], zeroed here first unless zero=False: the caller's buffer is already zero).
    Returns True when fused; False = the plain data gradient ran and `sums` is untouched (run the
    two-pass BN backward)."""
    _prec(desc, src)
    n = int(_lib.load().cvl_conv_igemm_workspace_size(ctypes.byref(desc)))
    ws = torch.empty(n, dtype=torch.uint8, device=src.device) if n > 16 else None
    if zero:
        sums.zero_()
    flag = ctypes.c_int32(0)
    _lib.call("cvl_conv_igemm_dgrad_bnsum", ctypes.byref(desc), ptr(src), ptr(dst), ptr(z), ptr(mean_rstd), ptr(gamma),
              ptr(beta), float(act_hi), acc_ptr(sums), ctypes.addressof(flag), ptr(ws), n if ws is not None else 0,
              stream())
    return bool(flag.value)


def conv_igemm_dgrad_bnsum_res(desc, src, dst, y, z, mean_rstd, gamma, beta, sums, zero=True):
    """Residual-unit form of conv_igemm_dgrad_bnsum: a beta-accumulating 1x1 DGRAD that completes dy of
    a BN -> (+ shortcut) -> ReLU unit with output y; its epilogue forms that BN backward's first pass
    (mask y > 0) into `sums`.  True when fused, else the plain data gradient ran."""
    _prec(desc, src)
    n = int(_lib.load().cvl_conv_igemm_workspace_size(ctypes.byref(desc)))
    ws = torch.empty(n, dtype=torch.uint8, device=src.device) if n > 16 else None
    if zero:
        sums.zero_()
    flag = ctypes.c_int32(0)
    _lib.call("cvl_conv_igemm_dgrad_bnsum_res", ctypes.byref(desc), ptr(src), ptr(dst), ptr(y), ptr(z),
              ptr(mean_rstd), ptr(gamma), ptr(beta), acc_ptr(sums), ctypes.addressof(flag), ptr(ws),
              n if ws is not None else 0, stream())
    return bool(flag.value)


def bn_backward_res_sums(dy, y, z, mean_rstd, gamma, sums, dz, g_out, dgamma, dbeta, B, HW, C, beta_acc=0.0,
                         conv_dbias=None):
    """Second pass of a residual unit's BN backward (mask y > 0, g_out = masked dy) from the fused sums."""
    _lib.call("cvl_bn_backward_res_sums", ptr(dy), ptr(y), ptr(z), ptr(mean_rstd), ptr(gamma), acc_ptr(sums), ptr(dz),
              ptr(g_out), ptr(dgamma), ptr(dbeta), float(beta_acc), ptr(conv_dbias), B, HW, C, stream())


def bn_backward_res_sums_sc(dy, y, z, mean_rstd, gamma, sums, dz, g_out, dgamma, dbeta, z_sc, mean_rstd_sc, sc_sums,
                            B, HW, C, beta_acc=0.0, conv_dbias=None):
    """bn_backward_res_sums that also forms the projection shortcut BN's first pass (its dy = g_out)
    into sc_sums [B][C][2] (float64 values); bn_backward_sums then runs the shortcut's second pass."""
    n = int(_lib.load().cvl_bn_backward_res_sums_sc_workspace_size(B, HW, C))
    ws = torch.empty(n, dtype=torch.uint8, device=dy.device)
    _lib.call("cvl_bn_backward_res_sums_sc", ptr(dy), ptr(y), ptr(z), ptr(mean_rstd), ptr(gamma), acc_ptr(sums),
              ptr(dz), ptr(g_out), ptr(dgamma), ptr(dbeta), float(beta_acc), ptr(conv_dbias), ptr(z_sc),
              ptr(mean_rstd_sc), ptr(ws), n, ptr(sc_sums), B, HW, C, stream())


def bn_backward_sc(dy, y, z, mean_rstd, gamma, dz, g_out, dgamma, dbeta, z_sc, mean_rstd_sc, sc_sums, B, HW, C,
                   beta_acc=0.0, conv_dbias=None):
    """bn_backward (mask y > 0, g_out) whose second pass also forms the projection shortcut BN's first
    pass into sc_sums [B][C][2] (float64 values)."""
    n = int(_lib.load().cvl_bn_backward_sc_workspace_size(B, HW, C))
    ws = torch.empty(n, dtype=torch.uint8, device=dy.device)
    _lib.call("cvl_bn_backward_sc", ptr(dy), ptr(y), ptr(z), ptr(mean_rstd), ptr(gamma), ptr(ws), n, ptr(dz),
              ptr(g_out), ptr(dgamma), ptr(dbeta), float(beta_acc), ptr(conv_dbias), ptr(z_sc), ptr(mean_rstd_sc),
              ptr(sc_sums), B, HW, C, stream())


def bn_backward_sums(dy, z, mean_rstd, gamma, sums, dz, dgamma, dbeta, B, HW, C, beta_acc=0.0, conv_dbias=None):
    """Second pass of a BN without ReLU from first-pass sums [B][C][2] (float64 values)."""
    _lib.call("cvl_bn_backward_sums", ptr(dy), ptr(z), ptr(mean_rstd), ptr(gamma), ptr(sums), ptr(dz), ptr(dgamma),
              ptr(dbeta), float(beta_acc), ptr(conv_dbias), B, HW, C, stream())


def bn_backward_relu_sums(dy, z, mean_rstd, gamma, beta, sums, dz, dgamma, dbeta, B, HW, C, beta_acc=0.0,
                          conv_dbias=None, act_hi=float("inf")):
    """Second pass of bn_backward_relu from the fused first-pass sums (conv_igemm_dgrad_bnsum)."""
    _lib.call("cvl_bn_backward_relu_sums", ptr(dy), ptr(z), ptr(mean_rstd), ptr(gamma), ptr(beta), acc_ptr(sums), ptr(dz),
              ptr(dgamma), ptr(dbeta), float(beta_acc), ptr(conv_dbias), float(act_hi), B, HW, C, stream())


def bn_backward_relu(dy, z, mean_rstd, gamma, beta, dz, dgamma, dbeta, B, HW, C, beta_acc=0.0, conv_dbias=None):
    """bn_backward of a BN -> ReLU unit without a residual add: the mask is rebuilt from z."""
    if _is_f32(dy):
        return bn_backward_f32(dy, None, z, mean_rstd, gamma, beta, dz, None, dgamma, dbeta, B, HW, C, beta_acc,
                               conv_dbias)
    n = int(_lib.load().cvl_bn_backward_workspace_size(B, HW, C))
    ws = torch.empty(n, dtype=torch.uint8, device=dy.device)
    _lib.call("cvl_bn_backward_relu", ptr(dy), ptr(z), ptr(mean_rstd), ptr(gamma), ptr(beta), ptr(ws), n, ptr(dz),
              ptr(dgamma), ptr(dbeta), float(beta_acc), ptr(conv_dbias), B, HW, C, stream())


def bn_relu_maxpool3x3s2(z, mean_rstd, gamma, beta, y, argmax):
    """The stem's BN -> ReLU -> pad 1 -> max-pool 3x3/2 from the pre-BN z (bf16), no full-size BN output."""
    B, H, W, C = z.shape
    _lib.call("cvl_bn_relu_maxpool3x3s2", ptr(z), ptr(mean_rstd), ptr(gamma), ptr(beta), ptr(y), ptr(argmax), B, H,
              W, C, stream())


def maxpool3x3s2(x, y, argmax):
    B, H, W, C = x.shape
    _lib.call("cvl_maxpool3x3s2_f32" if _is_f32(x) else "cvl_maxpool3x3s2", ptr(x), ptr(y), ptr(argmax), B, H, W, C, stream())


def maxpool3x3s2_backward(dy, argmax, dx):
    B, H, W, C = dx.shape
    _lib.call("cvl_maxpool3x3s2_backward_f32" if _is_f32(dy) else "cvl_maxpool3x3s2_backward", ptr(dy), ptr(argmax), ptr(dx), B, H, W, C, stream())


def maxpool3x3s2_backward_bn_relu(dp, argmax, z, mean_rstd, gamma, beta, dy, dz, dgamma, dbeta, beta_acc=0.0,
                                  conv_dbias=None):
    """maxpool3x3s2_backward + bn_backward_relu of the ResNet stem (C = 64, bf16) with the BN
    backward's first pass fused into the pool kernel; dy is the pool's input gradient (stored)."""
    B, H, W, C = z.shape
    n = int(_lib.load().cvl_maxpool3x3s2_backward_bn_relu_workspace_size(B, H, W, C))
    ws = torch.empty(n, dtype=torch.uint8, device=z.device)
    _lib.call("cvl_maxpool3x3s2_backward_bn_relu", ptr(dp), ptr(argmax), ptr(z), ptr(mean_rstd), ptr(gamma),
              ptr(beta), ptr(ws), n, ptr(dy), ptr(dz), ptr(dgamma), ptr(dbeta), float(beta_acc), ptr(conv_dbias),
              B, H, W, C, stream())


def upsample2x_add(a, b, out, B, H, W, C):
    _lib.call("cvl_upsample2x_add_f32" if _is_f32(a) else "cvl_upsample2x_add", ptr(a), ptr(b), ptr(out), B, H, W, C, stream())


def upsample2x_backward(dout, db, B, H, W, C, beta=0.0):
    _lib.call("cvl_upsample2x_backward_f32" if _is_f32(dout) else "cvl_upsample2x_backward", ptr(dout), ptr(db), B, H, W, C, float(beta), stream())


def relu_backward(dy, y, dx, beta=0.0):
    _lib.call("cvl_relu_backward_f32" if _is_f32(dy) else "cvl_relu_backward", ptr(dy), ptr(y), ptr(dx), dy.numel(), float(beta), stream())


def add(a, b, out):
    _lib.call("cvl_add_f32" if _is_f32(a) else "cvl_add", ptr(a), ptr(b), ptr(out), a.numel(), stream())


def bias_grad(dy, ld, coff, ncol, base, img_stride, HW, B, db, beta=0.0):
    if _is_f32(dy):
        return bias_grad_multi([(dy, ld, coff, ncol, base, img_stride, HW, B, db, beta)])
    n = int(_lib.load().cvl_bias_grad_workspace_size(ncol, HW, B))
    ws = torch.empty(max(n, 16), dtype=torch.uint8, device=dy.device)
    _lib.call("cvl_bias_grad", ptr(dy), ld, coff, ncol, int(base), int(img_stride), HW, B, ptr(ws), ws.numel(),
              ptr(db), float(beta), stream())


class BiasItem(ctypes.Structure):
    _fields_ = [("dy", c_void_p), ("db", c_void_p), ("base", ctypes.c_int64), ("img_stride", ctypes.c_int64),
                ("ld", c_int), ("coff", c_int), ("ncol", c_int), ("HW", c_int), ("B", c_int), ("beta", ctypes.c_float)]


BIAS_MAX_ITEMS = 16


def bias_grad_multi(items):
    """Several bias gradients in one launch pair (cvl_bias_grad_multi).  items: list of
    (dy, ld, coff, ncol, base, img_stride, HW, B, db, beta) -- bias_grad's arguments."""
    for k in range(0, len(items), BIAS_MAX_ITEMS):
        chunk = items[k:k + BIAS_MAX_ITEMS]
        arr = (BiasItem * len(chunk))()
        dev = chunk[0][0].device
        for i, (dy, ld, coff, ncol, base, img_stride, HW, B, db, beta) in enumerate(chunk):
            _lib.require_cuda(dy, db)
            arr[i] = BiasItem(dy.data_ptr(), db.data_ptr(), int(base), int(img_stride), int(ld), int(coff), int(ncol),
                              int(HW), int(B), float(beta))
        if _is_f32(chunk[0][0]):
            assert all(_is_f32(it[0]) for it in chunk)
            _lib.call("cvl_bias_grad_multi_f32", arr, len(chunk), stream())
            continue
        n = int(_lib.load().cvl_bias_grad_multi_workspace_size(arr, len(chunk)))
        if n == 0:
            raise _lib.CvlError("cvl_bias_grad_multi: invalid items")
        ws = torch.empty(n, dtype=torch.uint8, device=dev)
        _lib.call("cvl_bias_grad_multi", arr, len(chunk), ptr(ws), ws.numel(), stream())


SUMSQ_WS = 1025     # include/cvlite.h CVL_SUMSQ_WS: norm total + per-block partials (float64)


def sgd_clip_update(w, g, v, lr_dev, momentum, inv_bs, clip, ws=None):
    if ws is None:
        ws = torch.empty(SUMSQ_WS, dtype=torch.float64, device=w.device)
    assert ws.numel() >= SUMSQ_WS
    _lib.call("cvl_sgd_clip_update", ptr(w), ptr(g), ptr(v), w.numel(), ptr(lr_dev), float(momentum),
              float(inv_bs), float(clip), ptr(ws), stream())


def lr_schedule(step_dev, lr_dev, init_lr, min_lr, decay_rate, decay_step, max_decays=None):
    if max_decays is None:
        _lib.call("cvl_lr_schedule", ptr(step_dev), ptr(lr_dev), float(init_lr), float(min_lr),
                  float(decay_rate), int(decay_step), stream())
    else:
        _lib.call("cvl_lr_schedule_capped", ptr(step_dev), ptr(lr_dev), float(init_lr), float(min_lr),
                  float(decay_rate), int(decay_step), int(max_decays), stream())


class L2Reg(object):
    """Device l2_params_reg of a ParamStore (train_fcos.py:118-120): sum over the trainable
    tensors of sqrt(tf.nn.l2_loss(v)); graph-capturable, result in self.out (device float)."""

    def __init__(self, store):
        dev = store.flat.device
        offs = [o for (o, n, _) in store.offsets.values()]
        cnts = [n for (o, n, _) in store.offsets.values()]
        self.store = store
        self.offs = torch.tensor(offs, dtype=torch.int64, device=dev)
        self.cnts = torch.tensor(cnts, dtype=torch.int64, device=dev)
        self.terms = torch.zeros(len(offs), dtype=torch.float32, device=dev)
        self.out = torch.zeros(1, dtype=torch.float32, device=dev)

    def run(self):
        _lib.call("cvl_l2_params_reg", ptr(self.store.flat), ptr(self.offs), ptr(self.cnts), int(self.offs.numel()),
                  ptr(self.terms), ptr(self.out), stream())
        return self.out


def select_first_nonzero(counts, k, idx, weight):
    _lib.call("cvl_select_first_nonzero", ptr(counts), int(counts.numel()), int(k), ptr(idx), ptr(weight), stream())


def gather_rows(src, idx, dst):
    """dst[i] = src[idx[i]] along dim 0 (contiguous tensors, same row size)."""
    row_bytes = src[0].numel() * src.element_size()
    assert dst[0].numel() * dst.element_size() == row_bytes and src.is_contiguous() and dst.is_contiguous()
    _lib.call("cvl_gather_rows", ptr(src), int(row_bytes), ptr(idx), int(idx.numel()), ptr(dst), stream())


# ---- CenterNet hourglass ops (include/cvlite.h "CenterNet hourglass training path") -------------
def bn_stats(x, B, HW, C, stats):
    n = int(_lib.load().cvl_bn_stats_workspace_size(B, HW, C))
    ws = torch.empty(max(n, 16), dtype=torch.uint8, device=x.device)
    _lib.call("cvl_bn_stats", ptr(x), B, HW, C, acc_ptr(stats), ptr(ws), ws.numel(), stream())


def bn_finalize_grouped(stats, mean_rstd, run_mean, run_var, B, C, HW, group, eps, momentum):
    _lib.call("cvl_bn_finalize_grouped", acc_ptr(stats), ptr(mean_rstd), ptr(run_mean), ptr(run_var), B, C, HW,
              int(group), float(eps), float(momentum), stream())


def bn_backward_grouped(dy, z, mean_rstd, gamma, dz, dgamma, dbeta, B, HW, C, group, dz_beta=0.0, y_relu=None):
    n = int(_lib.load().cvl_bn_backward_grouped_workspace_size(B, HW, C))
    ws = torch.empty(n, dtype=torch.uint8, device=dy.device)
    _lib.call("cvl_bn_backward_grouped", ptr(dy), ptr(y_relu), ptr(z), ptr(mean_rstd), ptr(gamma), ptr(ws), n,
              ptr(dz), float(dz_beta), ptr(dgamma), ptr(dbeta), B, HW, C, int(group), stream())


def maxpool2x2(x, y, argmax):
    B, H, W, C = x.shape
    _lib.call("cvl_maxpool2x2", ptr(x), ptr(y), ptr(argmax), B, H, W, C, stream())


def maxpool2x2_backward(dy, argmax, dx):
    B, H, W, C = dx.shape
    _lib.call("cvl_maxpool2x2_backward", ptr(dy), ptr(argmax), ptr(dx), B, H, W, C, stream())


def upsample_bilinear2x_add(prev, other, out):
    B, h, w, C = prev.shape
    assert tuple(other.shape) == (B, 2 * h, 2 * w, C) and out.shape == other.shape
    _lib.call("cvl_upsample_bilinear2x_add", ptr(prev), ptr(other), ptr(out), B, h, w, C, stream())


def upsample_bilinear2x_backward(dout, dprev, beta=0.0):
    B, h, w, C = dprev.shape
    assert tuple(dout.shape) == (B, 2 * h, 2 * w, C)
    _lib.call("cvl_upsample_bilinear2x_backward", ptr(dout), ptr(dprev), B, h, w, C, float(beta), stream())


class SepItem(ctypes.Structure):
    _fields_ = [("dw", c_void_p), ("pw", c_void_p), ("weff", c_void_p), ("gweff", c_void_p), ("gdw", c_void_p),
                ("gpw", c_void_p), ("taps", c_int), ("cin", c_int), ("cout", c_int),
                ("cin_ld", c_int), ("cout_ld", c_int), ("pad_", c_int)]


class SepPlan(object):
    """Device tables of cvl_sep_fold_multi / cvl_sep_unfold_multi: every SeparableConv2D's dense
    fold (forward) and gradient unfold (backward) in one launch each.
    entries: (dw [kh,kw,Cin,1], pw [1,1,Cin,Cout], weff, gweff, gdw, gpw) fp32 device tensors;
    weff / gweff may be channel-padded [kh,kw,Cin_p,Cout_p] (pads stay as they are, i.e. zero)."""

    def __init__(self, entries, device):
        items = (SepItem * len(entries))()
        rows = []
        self._keep = []
        for i, (dw, pw, weff, gweff, gdw, gpw) in enumerate(entries):
            kh, kw, cin, _ = dw.shape
            cout = pw.shape[3]
            assert tuple(weff.shape[:2]) == (kh, kw) and weff.shape[2] >= cin and weff.shape[3] >= cout
            assert gweff.shape == weff.shape
            it = items[i]
            it.cin_ld, it.cout_ld = int(weff.shape[2]), int(weff.shape[3])
            it.dw, it.pw, it.weff = dw.data_ptr(), pw.data_ptr(), weff.data_ptr()
            it.gweff, it.gdw, it.gpw = gweff.data_ptr(), gdw.data_ptr(), gpw.data_ptr()
            it.taps, it.cin, it.cout = kh * kw, cin, cout
            self._keep.append((dw, pw, weff, gweff, gdw, gpw))
            rows += [(i, ci) for ci in range(cin)]
        self.items = torch.frombuffer(bytearray(bytes(items)), dtype=torch.uint8).to(device)
        self.rows = torch.tensor(rows, dtype=torch.int32, device=device)
        self.nrows = len(rows)

    def fold(self):
        _lib.call("cvl_sep_fold_multi", ptr(self.items), ptr(self.rows), self.nrows, stream())

    def unfold(self):
        _lib.call("cvl_sep_unfold_multi", ptr(self.items), ptr(self.rows), self.nrows, stream())


def bias_scalar_fold(bias, scalar, b_eff, c0):
    _lib.call("cvl_bias_scalar_fold", ptr(bias), ptr(scalar), ptr(b_eff), int(bias.numel()), int(c0), stream())


def bias_scalar_unfold(g_eff, g_bias, g_scalar, c0):
    _lib.call("cvl_bias_scalar_unfold", ptr(g_eff), ptr(g_bias), ptr(g_scalar), int(g_eff.numel()), int(c0), stream())


def bias_scalar_fold_periodic(bias, scalar, b_eff, period, c0):
    _lib.call("cvl_bias_scalar_fold_periodic", ptr(bias), ptr(scalar), ptr(b_eff), int(bias.numel()), int(period),
              int(c0), stream())


def bias_scalar_unfold_periodic(g_eff, g_bias, g_scalar, period, c0):
    _lib.call("cvl_bias_scalar_unfold_periodic", ptr(g_eff), ptr(g_bias), ptr(g_scalar), int(g_eff.numel()),
              int(period), int(c0), stream())


def upsample_bilinear2x_sum(a, b, out):
    """out = UpSampling2D(bilinear)(a + b) (b may be None): one pass, taps summed in fp32."""
    B, h, w, C = a.shape
    assert tuple(out.shape) == (B, 2 * h, 2 * w, C) and (b is None or b.shape == a.shape)
    _lib.call("cvl_upsample_bilinear2x_sum", ptr(a), ptr(b), ptr(out), B, h, w, C, stream())


class RcItem(ctypes.Structure):
    _fields_ = [("src", c_void_p), ("dsrc", c_void_p), ("c", c_int), ("c_ld", c_int), ("hw", c_int),
                ("beta", ctypes.c_float)]


def _rc_items(maps):
    items = (RcItem * len(maps))()
    for k, (src, dsrc, c, beta) in enumerate(maps):
        t = src if src is not None else dsrc
        it = items[k]
        it.src = src.data_ptr() if src is not None else None
        it.dsrc = dsrc.data_ptr() if dsrc is not None else None
        it.c, it.c_ld, it.hw, it.beta = int(c), int(t.shape[-1]), int(t.shape[1] * t.shape[2]), float(beta)
    return items


def reshape_concat(maps, dst):
    """maps: [(src [B,h,w,c_ld] bf16, c_real)]; dst [B,S,S,ld] bf16 (tf_hourglass_net.py:307-344)."""
    B, S0, S1, ld = dst.shape
    items = _rc_items([(m, None, c, 0.0) for m, c in maps])
    _lib.call("cvl_reshape_concat", ctypes.cast(items, c_void_p), len(maps), B, S0 * S1, ptr(dst), ld, stream())


def reshape_concat_backward(maps, d_dst):
    """maps: [(dsrc [B,h,w,c_ld] bf16, c_real, beta)]: dsrc = beta*dsrc + gather(d_dst)."""
    B, S0, S1, ld = d_dst.shape
    items = _rc_items([(None, d, c, beta) for d, c, beta in maps])
    _lib.call("cvl_reshape_concat_backward", ctypes.cast(items, c_void_p), len(maps), B, S0 * S1, ptr(d_dst), ld, stream())


def adam_clip_update(w, g, m, v, lr_dev, iterations, beta1, beta2, eps, inv_bs, clip, ws=None):
    if ws is None:
        ws = torch.empty(1, dtype=torch.float64, device=w.device)
    _lib.call("cvl_adam_clip_update", ptr(w), ptr(g), ptr(m), ptr(v), w.numel(), ptr(lr_dev), ptr(iterations),
              float(beta1), float(beta2), float(eps), float(inv_bs), float(clip), ptr(ws), stream())
