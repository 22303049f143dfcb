"""Teacher-forced per-launch parity of a production training step (TEST INFRASTRUCTURE).

`LaunchParity` wraps every device op of `cvlite.ops_nn` (and the fused target / loss ops of
`cvlite.ops_targets`) while one real trainer step runs eagerly on the production dispatch (the
same Python calls the step's HIP graphs capture, so the same kernels, planner choices and
workspaces).  Around each launch it snapshots the GPU's OWN inputs (and any beta-accumulated
destination), lets the HIP kernel run, then recomputes that launch in float64 torch from the
snapshot and compares:

* convolutions (forward, data gradient, weight gradient; segmented / grouped / split-K /
  deferred-reduction forms; the fused BN-statistics, BN-backward-first-pass and residual
  epilogues): an explicit float64 im2col (`F.unfold` / `F.fold`) + matmul restatement of
  `cvl_conv_desc` (include/cvlite.h), weights decoded from the packed bf16 operand the kernel read;
* BatchNorm finalize / apply / backward (all mask sources), the stem pool forms, max-pool,
  nearest / bilinear up-sampling, ReLU backward, adds, bias gradients, the clip + SGD / Adam
  updates, the weight re-pack, the FCOS / RetinaNet / CenterNet fused losses (float64 autograd of
  oracle/fcos_torch.py) -- float64 restatements of the kernels' documented semantics.

Tolerances: bf16 outputs rel-L2 <= 1e-2, fp32 outputs rel-L2 <= 1e-4;
reductions whose terms cancel (bias / BN-parameter gradients, BN-backward sums) are normalised by
the same reduction over |terms| (`red`), because a relative error of a near-zero sum says nothing
about the kernel; exact ops (pooling values / argmax, im2col, re-pack) must match bit-for-bit.

The wrapper also hooks `_lib.call` and records every C entry point launched, so a test can assert
that no launch of the step went unchecked.  Weight-gradient launches flush their deferred split
reduction right after the call (the batched reduction runs with one record; its multi-record
ordering is covered by tests/test_gpu_conv.py::test_conv_wgrad_deferred_reduction).
"""
import collections
import math

import torch
import torch.nn.functional as F

F64 = torch.float64
TOL_BF16, TOL_F32 = 1e-2, 1e-4

# entry points that launch nothing, or only size / configure (not compute on tensors)
NON_COMPUTE = {
    "cvl_wgrad_defer", "cvl_wgrad_flush", "cvl_probe_arm",
    "cvl_bn_acc_decode",          # the harness's own reads of BN accumulator buffers
}
CK_NAMES = {0: "none", 1: "BASE", 2: "BASE_SPLITK", 3: "L64", 4: "L128", 5: "L256", 6: "X256", 7: "X32",
            8: "WG_S", 9: "WG_L128", 10: "WG_L256", 11: "WG_X", 12: "X32H", 13: "WG_SN", 14: "H64", 15: "WG_H",
            16: "P"}


def rel_l2(got, ref):
    got, ref = got.double(), ref.double()
    d = float((got - ref).norm())
    n = float(ref.norm())
    return d / n if n > 0 else d


def red_err(got, ref, ref_abs):
    """|got - ref| over the same reduction of |terms| (cancellation-safe error of a sum)."""
    d = float((got.double() - ref.double()).norm())
    n = float(ref_abs.double().norm())
    return d / n if n > 0 else d


def _rows(t, ld):
    flat = t.reshape(-1)
    return flat[: flat.numel() // ld * ld].view(-1, ld)


def _gather(rows, base, img, imgs, H, W):
    """[len(imgs), H, W, C] of the rows of images `imgs` (row base + b*img + y*W + x)."""
    return torch.stack([rows[base + b * img: base + b * img + H * W] for b in imgs]).view(len(imgs), H, W, -1)


def _row_index(base, img, imgs, HW, device):
    q = torch.arange(HW, device=device, dtype=torch.int64)
    return torch.cat([base + b * img + q for b in imgs])


def _pad_crop(x, KH, KW, stride, pt, pl, Ho, Wo):
    """NCHW input padded (TF 'same' leading pads given) / cropped to exactly the rows the Ho x Wo
    outputs read: (Ho-1)*stride + KH."""
    nh, nw = (Ho - 1) * stride + KH, (Wo - 1) * stride + KW
    H, W = x.shape[2], x.shape[3]
    x = F.pad(x, (pl, max(0, nw - W - pl), pt, max(0, nh - H - pt)))
    return x[:, :, :nh, :nw]


def _chunks(n, per_img_bytes, cap=1 << 31):
    step = max(1, int(cap // max(per_img_bytes, 1)))
    return [(i, min(n, i + step)) for i in range(0, n, step)]


def conv_fwd64(x, w, stride, pt, pl, Ho, Wo):
    """x [B,H,W,Ci] f64, w [O,KH,KW,Ci] (OHWI) f64 -> [B,Ho,Wo,O]."""
    B, H, W, Ci = x.shape
    O, KH, KW, _ = w.shape
    w2 = w.permute(0, 3, 1, 2).reshape(O, Ci * KH * KW)
    out = torch.empty((B, O, Ho * Wo), dtype=F64, device=x.device)
    for a, b in _chunks(B, Ci * KH * KW * Ho * Wo * 8):
        xp = _pad_crop(x[a:b].permute(0, 3, 1, 2), KH, KW, stride, pt, pl, Ho, Wo)
        cols = F.unfold(xp, (KH, KW), stride=stride)
        out[a:b] = torch.matmul(w2, cols)
    return out.view(B, O, Ho, Wo).permute(0, 2, 3, 1)


def conv_dgrad64(dy, w, stride, pt, pl, H, W):
    """dy [B,Ho,Wo,O], w [O,KH,KW,Ci] (the FORWARD weight) -> dx [B,H,W,Ci]."""
    B, Ho, Wo, O = dy.shape
    _, KH, KW, Ci = w.shape
    w2t = w.permute(0, 3, 1, 2).reshape(O, Ci * KH * KW).t()
    nh, nw = (Ho - 1) * stride + KH, (Wo - 1) * stride + KW
    dx = torch.empty((B, H, W, Ci), dtype=F64, device=dy.device)
    for a, b in _chunks(B, Ci * KH * KW * Ho * Wo * 8):
        cols = torch.matmul(w2t, dy[a:b].permute(0, 3, 1, 2).reshape(b - a, O, Ho * Wo))
        dxp = F.fold(cols, (nh, nw), (KH, KW), stride=stride)          # padded-input coordinates
        dxp = F.pad(dxp, (0, max(0, pl + W - nw), 0, max(0, pt + H - nh)))
        dx[a:b] = dxp[:, :, pt:pt + H, pl:pl + W].permute(0, 2, 3, 1)
    return dx


def conv_wgrad64(x, dy, KH, KW, stride, pt, pl):
    """x [B,H,W,Ci], dy [B,Ho,Wo,O] -> dW [KH,KW,Ci,O] (HWIO)."""
    B, H, W, Ci = x.shape
    _, Ho, Wo, O = dy.shape
    acc = torch.zeros((O, Ci * KH * KW), dtype=F64, device=x.device)
    for a, b in _chunks(B, Ci * KH * KW * Ho * Wo * 8):
        xp = _pad_crop(x[a:b].permute(0, 3, 1, 2), KH, KW, stride, pt, pl, Ho, Wo)
        cols = F.unfold(xp, (KH, KW), stride=stride)                  # [b, Ci*KK, L]
        g = dy[a:b].permute(0, 3, 1, 2).reshape(b - a, O, Ho * Wo)
        acc += torch.einsum("bol,bkl->ok", g, cols)
    return acc.view(O, Ci, KH, KW).permute(2, 3, 1, 0)


def bn_affine32(z, m, rs, ga, be):
    """cvl's fma(gamma, (z - mean) * rstd, beta): (z - m) * rs in fp32 (two IEEE ops), the fma
    evaluated exactly in fp64 (a 24x24-bit product is exact there) and rounded once to fp32."""
    xh = (z.float() - m.float()) * rs.float()
    return (ga.double() * xh.double() + be.double()).float(), xh


class Record(object):
    __slots__ = ("op", "detail", "kernel", "what", "err", "tol", "ok")

    def __init__(self, op, detail, kernel, what, err, tol):
        self.op, self.detail, self.kernel, self.what, self.err, self.tol = op, detail, kernel, what, err, tol
        self.ok = (err <= tol) if not (isinstance(err, float) and math.isnan(err)) else False

    def line(self):
        return "%-30s %-34s %-14s %-10s %.3e (tol %.0e) %s" % (self.op, self.detail[:34], self.kernel, self.what,
                                                               self.err, self.tol, "ok" if self.ok else "FAIL")


class LaunchParity(object):
    """Context manager: patch the device ops, check every launch, collect Records.

    imgs: how many images (first and last first) the forward / data-gradient references cover
    (None = all); weight gradients, BN statistics and reductions always cover the whole batch."""

    def __init__(self, imgs=2):
        self.nimg = imgs
        self.records = []
        self.calls = collections.Counter()
        self.checked_calls = collections.Counter()
        self._saved = []
        self.depth = 0

    # ---- bookkeeping ----------------------------------------------------------------------
    def img_set(self, B):
        if self.nimg is None or self.nimg >= B:
            return list(range(B))
        s = [0, B - 1] + list(range(1, B - 1))
        return sorted(s[:self.nimg])

    def add(self, op, detail, what, err, tol, kernel=""):
        self.records.append(Record(op, detail, kernel, what, float(err), tol))

    def cmp(self, op, detail, what, got, ref, kernel="", tol=None):
        if tol is None:
            tol = TOL_F32 if got.dtype in (torch.float32, torch.float64) else TOL_BF16
        self.add(op, detail, what, rel_l2(got, ref), tol, kernel)

    def exact(self, op, detail, what, got, ref, kernel="", frac_tol=0.0):
        bad = float((got.double() != ref.double()).float().mean()) if got.numel() else 0.0
        self.add(op, detail, what, bad, frac_tol, kernel)

    def failures(self):
        return [r for r in self.records if not r.ok]

    def table(self):
        return "\n".join(r.line() for r in self.records)

    def unchecked_calls(self):
        return {k: v for k, v in self.calls.items() if k not in NON_COMPUTE and k not in self.checked_calls}

    # ---- patching ---------------------------------------------------------------------------
    def _patch(self, mod, name, fn):
        orig = getattr(mod, name)
        self._saved.append((mod, name, orig))
        setattr(mod, name, fn(orig))

    def __enter__(self):
        from cvlite import _lib, ops_nn, ops_targets
        self.lib, self.nn, self.ot = _lib, ops_nn, ops_targets
        lp = self

        def call_wrap(orig):
            def call(name, *a):
                lp.calls[name] += 1
                if lp.depth > 0:
                    lp.checked_calls[name] += 1
                return orig(name, *a)
            return call
        self._patch(_lib, "call", call_wrap)
        for name in CHECKS:
            if hasattr(ops_nn, name):
                self._patch(ops_nn, name, self._wrap(name, CHECKS[name]))
        for name in TARGET_CHECKS:
            if hasattr(ops_targets, name):
                self._patch(ops_targets, name, self._wrap(name, TARGET_CHECKS[name]))
        for cls, meth, chk in ((ops_nn.PackPlan, "run", check_packplan), (ops_nn.SepPlan, "fold", check_sep_fold),
                               (ops_nn.SepPlan, "unfold", check_sep_unfold), (ops_nn.L2Reg, "run", check_l2reg)):
            self._patch(cls, meth, self._wrap_method(meth, chk))
        return self

    def __exit__(self, *exc):
        for mod, name, orig in reversed(self._saved):
            setattr(mod, name, orig)
        self._saved = []
        return False

    def _wrap(self, name, chk):
        lp = self

        def wrap(orig):
            def run(*a, **k):
                def launch(*aa, **kk):
                    lp.depth += 1
                    try:
                        return orig(*aa, **kk)
                    finally:
                        lp.depth -= 1
                torch.cuda.synchronize()
                out = chk(lp, name, launch, *a, **k)
                torch.cuda.synchronize()
                return out
            return run
        return wrap

    def _wrap_method(self, name, chk):
        lp = self

        def wrap(orig):
            def run(obj, *a, **k):
                def launch():
                    lp.depth += 1
                    try:
                        return orig(obj, *a, **k)
                    finally:
                        lp.depth -= 1
                torch.cuda.synchronize()
                out = chk(lp, name, launch, obj)
                torch.cuda.synchronize()
                return out
            return run
        return wrap

    def orig(self, name):
        """The unwrapped ops_nn function (a check may run a reference launch with it)."""
        for mod, n, fn in self._saved:
            if mod is self.nn and n == name:
                return fn
        return getattr(self.nn, name)

    def last_kernel(self):
        """Short name of the conv kernel the last launch used (include/cvlite.h CVL_CK_*)."""
        return CK_NAMES.get(int(self.lib.load().cvl_conv_igemm_last_kernel()), "?")

    def flush_wgrad(self):
        self.depth += 1
        try:
            self.lib.call("cvl_wgrad_flush", self.lib.stream())
        finally:
            self.depth -= 1


# ================================================================================================
# convolutions
# ================================================================================================
def _segs(desc):
    out = []
    for i in range(desc.nseg):
        q = desc.seg[i]
        w, bias = desc._keep[i]
        out.append(dict(Hr=q.Hr, Wr=q.Wr, Hs=q.Hs, Ws=q.Ws, sb=q.src_base, si=q.src_img, db=q.dst_base,
                        di=q.dst_img, w=w, bias=bias))
    return out


def _w_fwd(desc, wpack):
    """packed forward operand [Npad][KH*KW*Cin] -> OHWI float64."""
    return wpack.view(desc.Npad, desc.KH, desc.KW, desc.Cin).double()


def _w_from_dgrad(desc, wpack):
    """packed data-gradient operand [Cin_pad][KH*KW*Cout_pad] (desc.Npad = Cin_pad, desc.Cin =
    Cout_pad) -> the FORWARD weight OHWI [Cout_pad, KH, KW, Cin_pad] float64."""
    return wpack.view(desc.Npad, desc.KH, desc.KW, desc.Cin).permute(3, 1, 2, 0).double()


def _detail(desc, s, B):
    kind = "fwd" if desc.mode == 0 else "dgrad"
    return "%s %dx%d/%d %d->%d %dx%d B%d%s" % (kind, desc.KH, desc.KW, desc.stride,
                                                desc.Cin if desc.mode == 0 else desc.Cin,
                                                desc.n_store, s["Hr"], s["Wr"], B,
                                                " seg%d" % desc.nseg if desc.nseg > 1 else "")


def _conv_ref_seg(lp, desc, s, srows, imgs):
    if desc.mode == 0:
        x = _gather(srows, s["sb"], s["si"], imgs, s["Hs"], s["Ws"]).double()
        if desc.relu_in:
            x = x.clamp_min(0)
        out = conv_fwd64(x, _w_fwd(desc, s["w"]), desc.stride, desc.pad_t, desc.pad_l, s["Hr"], s["Wr"])
        out = out[..., :desc.n_store]
        if s["bias"] is not None:
            out = out + s["bias"][:desc.n_store].double()
        if desc.relu_out:
            out = out.clamp_min(0)
        return out
    assert not desc.relu_in and not desc.relu_out
    dy = _gather(srows, s["sb"], s["si"], imgs, s["Hs"], s["Ws"]).double()
    dx = conv_dgrad64(dy, _w_from_dgrad(desc, s["w"]), desc.stride, desc.pad_t, desc.pad_l, s["Hr"], s["Wr"])
    return dx[..., :desc.n_store]


def _conv_check_dst(lp, name, desc, src, dst, old, kern, imgs_all=False):
    """Compare every segment's destination block with the float64 restatement; returns the list of
    (segment, image list, fp64 reference [n, Hr, Wr, n_store]) for epilogue checks."""
    srows = _rows(src, desc.Cin)
    drows = _rows(dst, desc.ld_dst)
    orows = _rows(old, desc.ld_dst) if old is not None else None
    out = []
    for s in _segs(desc):
        imgs = list(range(desc.B)) if imgs_all else lp.img_set(desc.B)
        ref = _conv_ref_seg(lp, desc, s, srows, imgs)
        idx = _row_index(s["db"], s["di"], imgs, s["Hr"] * s["Wr"], dst.device)
        cols = slice(desc.dst_coff, desc.dst_coff + desc.n_store)
        got = drows[idx, cols]
        r = ref.reshape(-1, desc.n_store)
        if orows is not None and desc.beta != 0.0:
            r = r + desc.beta * orows[idx, cols].double()
        lp.cmp(name, _detail(desc, s, desc.B), "dst", got, r, kern,
               tol=TOL_F32 if desc.dst_f32 or got.dtype == torch.float32 else TOL_BF16)
        out.append((s, imgs, idx, cols))
    return out


def check_conv_igemm(lp, name, launch, desc, src, dst, stats=None):
    old = dst.clone() if desc.beta != 0.0 else None
    st0 = stats.clone() if stats is not None else None
    launch(desc, src, dst, stats)
    kern = lp.last_kernel()
    _conv_check_dst(lp, name, desc, src, dst, old, kern)
    if stats is not None:
        # fused BN statistics: per (image, channel) (sum, sumsq) of the stored (rounded) output
        assert desc.nseg == 1 and desc.mode == 0
        s = _segs(desc)[0]
        drows = _rows(dst, desc.ld_dst)
        got = _acc(stats, desc.B, desc.n_store) - _acc(st0, desc.B, desc.n_store)
        HW = s["Hr"] * s["Wr"]
        for b in range(desc.B):
            z = drows[s["db"] + b * s["di"]: s["db"] + b * s["di"] + HW, desc.dst_coff:desc.dst_coff + desc.n_store]
            z = z.double()
            ref = torch.stack([z.sum(0), (z * z).sum(0)], -1)
            rabs = torch.stack([z.abs().sum(0), (z * z).sum(0)], -1)
            lp.add(name, _detail(desc, s, desc.B) + " img%d" % b, "bn_stats", red_err(got[b], ref, rabs), 1e-6, kern)


def check_conv_igemm_relu_mask(lp, name, launch, desc, src, dst, y):
    """The data gradient with the ReLU mask in its epilogue: the plain launch (checked against the
    float64 restatement as conv_igemm) masked by y > 0 must equal it bit for bit."""
    launch(desc, src, dst, y)
    kern = lp.last_kernel()
    plain = torch.empty_like(dst)
    lp.orig("conv_igemm")(desc, src, plain)
    _conv_check_dst(lp, name, desc, src, plain, None, lp.last_kernel())
    exp = torch.where(y.reshape(plain.shape).float() > 0, plain, torch.zeros_like(plain))
    lp.exact(name, _detail(desc, _segs(desc)[0], desc.B) + " relu(y)", "dst", dst, exp, kern)


def _wgrad_ref(desc, segs, x, dy):
    xrows = _rows(x, desc.Cin)
    drows = _rows(dy, desc.ld_dst)
    acc = None
    for s in segs:
        imgs = list(range(desc.B))
        xs = _gather(xrows, s["sb"], s["si"], imgs, s["Hs"], s["Ws"]).double()
        if desc.relu_in:
            xs = xs.clamp_min(0)
        g = _gather(drows, s["db"], s["di"], imgs, s["Hr"], s["Wr"])[..., desc.dst_coff:desc.dst_coff + desc.n_store]
        r = conv_wgrad64(xs, g.double(), desc.KH, desc.KW, desc.stride, desc.pad_t, desc.pad_l)
        acc = r if acc is None else acc + r
    return acc.reshape(-1, desc.n_store)


def _wgrad_detail(desc, segs, ng=1):
    s = segs[0]
    return "wgrad %dx%d/%d %d->%d %dx%d B%d%s" % (desc.KH, desc.KW, desc.stride, desc.Cin, desc.n_store,
                                                   s["Hr"], s["Wr"], desc.B,
                                                   " seg%d/g%d" % (desc.nseg, ng) if desc.nseg > 1 else "")


def _check_dw(lp, name, detail, kern, dw, old, beta, ref):
    got = dw.reshape(-1)
    n = min(got.numel() // ref.shape[1], ref.shape[0]) * ref.shape[1]
    r = ref.reshape(-1)[:n]
    if beta != 0.0:
        r = r + beta * old.reshape(-1)[:n].double()
    lp.cmp(name, detail, "dW", got[:n], r, kern, tol=TOL_F32)


def check_conv_wgrad(lp, name, launch, desc, x, dy, dw, beta=0.0):
    old = dw.clone() if beta != 0.0 else None
    launch(desc, x, dy, dw, beta)
    kern = lp.last_kernel()
    lp.flush_wgrad()
    segs = _segs(desc)
    _check_dw(lp, name, _wgrad_detail(desc, segs), kern, dw, old, beta, _wgrad_ref(desc, segs, x, dy))


def check_conv_wgrad_grouped(lp, name, launch, desc, x, dy, dws, beta=0.0):
    olds = [d.clone() for d in dws] if beta != 0.0 else [None] * len(dws)
    launch(desc, x, dy, dws, beta)
    kern = lp.last_kernel()
    lp.flush_wgrad()
    segs = _segs(desc)
    per = len(segs) // len(dws)
    for g, dw in enumerate(dws):
        sg = segs[g * per:(g + 1) * per]
        _check_dw(lp, name, _wgrad_detail(desc, segs, len(dws)) + " grp%d" % g, kern, dw, olds[g], beta,
                  _wgrad_ref(desc, sg, x, dy))


def check_conv_wgrad_batch(lp, name, launch, descs, xs, dys, dws, beta=0.0):
    """cvl_conv_wgrad_batch: every problem's dW against its own float64 restatement."""
    olds = [d.clone() for d in dws] if beta != 0.0 else [None] * len(dws)
    launch(descs, xs, dys, dws, beta)
    kern = lp.last_kernel()
    lp.flush_wgrad()
    for i, (desc, x, dy, dw) in enumerate(zip(descs, xs, dys, dws)):
        segs = _segs(desc)
        _check_dw(lp, name, _wgrad_detail(desc, segs) + " batch%d/%d" % (i, len(descs)), kern, dw, olds[i], beta,
                  _wgrad_ref(desc, segs, x, dy))


def _bnsum_ref(lp, name, detail, kern, sums, dst_rows, idx_b, z, mr, gamma, beta, act_hi, ymask, B, C, HW):
    """(sum g, sum g*xhat) per (image, channel); g = dst * mask (mask from y > 0, or rebuilt from
    z as the kernels do), computed on the launch's own stored destination."""
    got = _acc(sums, B, C)
    errs = []
    for b in range(B):
        zz = z.reshape(B, HW, -1)[b, :, :C]
        g = dst_rows[idx_b[b]].double()[:, :C]
        m, rs = mr[b, :C, 0], mr[b, :C, 1]
        a, xh = bn_affine32(zz, m, rs, gamma[:C], beta[:C])
        if ymask is not None:
            mask = ymask.reshape(B, HW, -1)[b, :, :C].float() > 0
        else:
            mask = (a > 0) & (a < act_hi)
        g = g * mask.double()
        ref = torch.stack([g.sum(0), (g * xh.double()).sum(0)], -1)
        rabs = torch.stack([g.abs().sum(0), (g * xh.double()).abs().sum(0)], -1)
        errs.append(red_err(got[b], ref, rabs))
    lp.add(name, detail, "bn_sums", max(errs), 1e-4, kern)


def check_dgrad_bnsum(lp, name, launch, desc, src, dst, z, mean_rstd, gamma, beta, sums, act_hi=float("inf"),
                      zero=True):
    fused = launch(desc, src, dst, z, mean_rstd, gamma, beta, sums, act_hi=act_hi, zero=zero)
    kern = lp.last_kernel()
    res = _conv_check_dst(lp, name, desc, src, dst, None, kern)
    if fused:
        s = res[0][0]
        HW = s["Hr"] * s["Wr"]
        drows = _rows(dst, desc.ld_dst)
        idx_b = [_row_index(s["db"], s["di"], [b], HW, dst.device) for b in range(desc.B)]
        _bnsum_ref(lp, name, _detail(desc, s, desc.B), kern, sums, drows, idx_b, z, mean_rstd, gamma, beta,
                   act_hi, None, desc.B, desc.n_store, HW)
    return fused


def check_dgrad_bnsum_res(lp, name, launch, desc, src, dst, y, z, mean_rstd, gamma, beta, sums, zero=True):
    old = dst.clone()
    fused = launch(desc, src, dst, y, z, mean_rstd, gamma, beta, sums, zero=zero)
    kern = lp.last_kernel()
    res = _conv_check_dst(lp, name, desc, src, dst, old, kern)
    if fused:
        s = res[0][0]
        HW = s["Hr"] * s["Wr"]
        drows = _rows(dst, desc.ld_dst)
        idx_b = [_row_index(s["db"], s["di"], [b], HW, dst.device) for b in range(desc.B)]
        _bnsum_ref(lp, name, _detail(desc, s, desc.B) + " res", kern, sums, drows, idx_b, z, mean_rstd, gamma,
                   beta, float("inf"), y, desc.B, desc.n_store, HW)
    return fused


def check_im2col(lp, name, launch, x, KH, KW, stride, pad_t, pad_l, Ho, Wo, Kp, out):
    launch(x, KH, KW, stride, pad_t, pad_l, Ho, Wo, Kp, out)
    B, H, W, C = x.shape
    xp = _pad_crop(x.double().permute(0, 3, 1, 2), KH, KW, stride, pad_t, pad_l, Ho, Wo)
    cols = F.unfold(xp, (KH, KW), stride=stride)                       # [B, C*KH*KW (c, kh, kw), L]
    cols = cols.view(B, C, KH * KW, Ho * Wo).permute(0, 3, 2, 1).reshape(B * Ho * Wo, KH * KW * C)
    ref = torch.zeros((B * Ho * Wo, Kp), dtype=F64, device=x.device)
    ref[:, :KH * KW * C] = cols
    lp.exact(name, "im2col %dx%d/%d %dx%dx%d B%d" % (KH, KW, stride, H, W, C, B), "cols",
             out.view(-1, Kp), ref.to(torch.bfloat16))


def _stem_cols(img, Ho, Wo):
    """[B*Ho*Wo, 192] float64 patch rows of the bf16-rounded image in the stem kernels' K order
    (k = ky*24 + kx*3 + c; 21..23 of each kernel row and 168..191 zero)."""
    B = img.shape[0]
    x = F.pad(img.to(torch.bfloat16).double().permute(0, 3, 1, 2), (3, 3, 3, 3))     # ZeroPadding2D(3)
    cols = F.unfold(x, 7, stride=2)                                                  # [B, (c, ky, kx), L]
    L = cols.shape[-1]
    assert L == Ho * Wo
    cols = cols.view(B, 3, 7, 7, L).permute(0, 4, 2, 3, 1).reshape(B * L, 7, 21)   # [px, ky, (kx, c)]
    out = torch.zeros((B * L, 8, 24), dtype=F64, device=img.device)
    out[:, :7, :21] = cols
    return out.view(B * L, 192)


def check_stem_conv(lp, name, launch, img, w_packed, bias, z, stats=None):
    st0 = stats.clone() if stats is not None else None
    launch(img, w_packed, bias, z, stats)
    B, H, W, _ = img.shape
    Ho, Wo = z.shape[1], z.shape[2]
    cols = _stem_cols(img, Ho, Wo)
    wk = torch.zeros((192, 64), dtype=F64, device=img.device)
    wk[:168] = w_packed.double().t()
    ref = cols @ wk + (bias.double() if bias is not None else 0.0)
    detail = "stem 7x7/2 %dx%d B%d" % (H, W, B)
    lp.cmp(name, detail, "z", z.reshape(-1, 64), ref, "STEM", tol=TOL_BF16)
    if stats is not None:
        got = _acc(stats, B, 64) - _acc(st0, B, 64)
        zz = z.double().reshape(B, Ho * Wo, 64)
        r = torch.stack([zz.sum(1), (zz * zz).sum(1)], -1)
        rabs = torch.stack([zz.abs().sum(1), (zz * zz).sum(1)], -1)
        lp.add(name, detail, "bn_stats", max(red_err(got[b], r[b], rabs[b]) for b in range(B)), 1e-6, "STEM")


def check_stem_wgrad(lp, name, launch, img, dz, dw, beta=0.0):
    old = dw.clone() if beta != 0.0 else None
    launch(img, dz, dw, beta)
    lp.flush_wgrad()
    B, H, W, _ = img.shape
    Ho, Wo = dz.shape[1], dz.shape[2]
    ref = _stem_cols(img, Ho, Wo).t() @ dz.double().reshape(-1, 64)
    if beta != 0.0:
        ref = ref + beta * old.double()
    lp.cmp(name, "stem wgrad 7x7/2 %dx%d B%d" % (H, W, B), "dW", dw, ref, "STEM", tol=TOL_F32)


def check_packplan(lp, name, launch, plan):
    launch()
    for i, (w, wf, wd) in enumerate(plan._keep):
        _check_pack(lp, "PackPlan.run", w, wf, wd, plan.host_items[i])


def _check_pack(lp, name, w, wf, wd, it):
    """bf16 (or parity-mode fp32) re-pack of HWIO master weights: forward [Npad][KHW][Cin_k] and
    data-gradient [Cin_pad][KHW][Cout_pad] images, zero outside the real channels, bit-exact."""
    khw, cin, cout, cin_k, npad, cin_pad, cout_pad = it.KHW, it.Cin, it.Cout, it.Cin_k, it.Npad, it.Cin_pad, it.Cout_pad
    W = w.reshape(khw, cin, cout)
    dt = wf.dtype if wf is not None else wd.dtype
    if wf is not None:
        ref = torch.zeros((npad, khw, cin_k), dtype=torch.float32, device=w.device)
        ref[:cout, :, :cin] = W.permute(2, 0, 1)
        lp.exact(name, "fwd pack %dx%d->%d" % (khw, cin, cout), "w_fwd", wf.view(npad, khw, cin_k), ref.to(dt))
    if wd is not None:
        ref = torch.zeros((cin_pad, khw, cout_pad), dtype=torch.float32, device=w.device)
        ref[:cin, :, :cout] = W.permute(1, 0, 2)
        lp.exact(name, "dgrad pack %dx%d->%d" % (khw, cin, cout), "w_dgrad", wd.view(cin_pad, khw, cout_pad),
                 ref.to(dt))


def check_pack_conv_weights(lp, name, launch, w_hwio, KH, KW, Cin, Cout, Cin_k, Npad, w_fwd, Cin_pad=0, Cout_pad=0,
                            w_dgrad=None):
    launch(w_hwio, KH, KW, Cin, Cout, Cin_k, Npad, w_fwd, Cin_pad, Cout_pad, w_dgrad)
    from cvlite.ops_nn import PackItem
    it = PackItem(KHW=KH * KW, Cin=Cin, Cout=Cout, Cin_k=Cin_k, Npad=Npad, Cin_pad=Cin_pad, Cout_pad=Cout_pad)
    _check_pack(lp, name, w_hwio, w_fwd, w_dgrad, it)


# ================================================================================================
# BatchNorm
# ================================================================================================
def _acc(acc, B, C):
    """float64 (B, C, 2) values of a BN accumulator buffer (ops_nn.bn_acc layout)."""
    from cvlite import ops_nn as nn
    return nn.bn_acc_value(acc).view(B, C, 2)


def _moments(stats, B, C, HW, eps):
    s = _acc(stats, B, C)
    m = s[..., 0] / HW
    var = (s[..., 1] / HW - m * m).clamp_min(0)
    return m, var, 1.0 / torch.sqrt(var + float(eps))


def _check_finalize(lp, name, detail, stats, mr, rm0, rv0, run_mean, run_var, B, C, HW, eps, momentum, group=1):
    s = _acc(stats, B, C)
    if group > 1:          # sub-batch statistics: sums of each group of `group` images
        ng = (B + group - 1) // group
        sg = torch.stack([s[g * group:(g + 1) * group].sum(0) for g in range(ng)])
        cnt = torch.tensor([min(group, B - g * group) for g in range(ng)], dtype=F64, device=s.device)
        m = sg[..., 0] / (HW * cnt[:, None])
        var = (sg[..., 1] / (HW * cnt[:, None]) - m * m).clamp_min(0)
        rs = 1.0 / torch.sqrt(var + float(eps))
        gi = torch.arange(B, device=s.device) // group
        mm, rr = m[gi], rs[gi]
        n_each = HW * cnt
        ema_m, ema_v = m, var * n_each[:, None] / (n_each[:, None] - 1)
    else:
        mm, var, rr = _moments(stats, B, C, HW, eps)
        ema_m, ema_v = mm, var * HW / (HW - 1.0) if HW > 1 else var
    if mr is not None:
        got = mr.view(B, C, 2)
        lp.cmp(name, detail, "mean", got[..., 0], mm, tol=1e-6)
        lp.cmp(name, detail, "rstd", got[..., 1], rr, tol=1e-6)
    if run_mean is not None:
        rm, rv = rm0.double(), rv0.double()
        for k in range(ema_m.shape[0]):
            rm = rm * momentum + ema_m[k] * (1 - momentum)
            rv = rv * momentum + ema_v[k] * (1 - momentum)
        lp.cmp(name, detail, "run_mean", run_mean, rm, tol=1e-5)
        lp.cmp(name, detail, "run_var", run_var, rv, tol=1e-5)


def _apply_ref(z, mr, gamma, beta, residual, relu, B, HW, C):
    zz = z.reshape(B, HW, C).double()
    m, rs = mr.view(B, C, 2)[..., 0].double(), mr.view(B, C, 2)[..., 1].double()
    y = gamma.double() * (zz - m[:, None]) * rs[:, None] + beta.double()
    if residual is not None:
        y = y + residual.reshape(B, HW, C).double()
    if relu:
        y = y.clamp_min(0)
    if relu == 2:
        y = y.clamp_max(6)
    return y


def check_bn_finalize(lp, name, launch, stats, mean_rstd, run_mean, run_var, B, C, HW, eps, momentum):
    rm0 = run_mean.clone() if run_mean is not None else None
    rv0 = run_var.clone() if run_var is not None else None
    launch(stats, mean_rstd, run_mean, run_var, B, C, HW, eps, momentum)
    _check_finalize(lp, name, "C%d HW%d B%d" % (C, HW, B), stats, mean_rstd, rm0, rv0, run_mean, run_var, B, C, HW,
                    eps, momentum)


def check_bn_finalize_apply(lp, name, launch, stats, mean_rstd, run_mean, run_var, z, gamma, beta, residual, y, B, HW,
                            C, relu, eps, momentum):
    rm0 = run_mean.clone() if run_mean is not None else None
    rv0 = run_var.clone() if run_var is not None else None
    zr, rr = _keep_inputs(y, z, residual)
    launch(stats, mean_rstd, run_mean, run_var, z, gamma, beta, residual, y, B, HW, C, relu, eps, momentum)
    d = "C%d HW%d B%d relu%d%s" % (C, HW, B, relu, " +res" if residual is not None else "")
    _check_finalize(lp, name, d, stats, mean_rstd, rm0, rv0, run_mean, run_var, B, C, HW, eps, momentum)
    lp.cmp(name, d, "y", y.reshape(B, HW, C), _apply_ref(zr, mean_rstd, gamma, beta, rr, relu, B, HW, C))


def check_bn_finalize_apply_bnres(lp, name, launch, stats, mean_rstd, run_mean, run_var, z, gamma, beta, res_stats,
                                  res_mean_rstd, res_run_mean, res_run_var, res_z, res_gamma, res_beta, res_eps,
                                  res_momentum, y, B, HW, C, relu, eps, momentum):
    rm0, rv0 = _clone(run_mean, run_var)
    rrm0, rrv0 = _clone(res_run_mean, res_run_var)
    zr, rzr = _keep_inputs(y, z, res_z)
    launch(stats, mean_rstd, run_mean, run_var, z, gamma, beta, res_stats, res_mean_rstd, res_run_mean, res_run_var,
           res_z, res_gamma, res_beta, res_eps, res_momentum, y, B, HW, C, relu, eps, momentum)
    d = "C%d HW%d B%d relu%d +bn-res" % (C, HW, B, relu)
    _check_finalize(lp, name, d, stats, mean_rstd, rm0, rv0, run_mean, run_var, B, C, HW, eps, momentum)
    _check_finalize(lp, name, d + " (res)", res_stats, res_mean_rstd, rrm0, rrv0, res_run_mean, res_run_var, B, C,
                    HW, res_eps, res_momentum)
    res = _apply_ref(rzr, res_mean_rstd, res_gamma, res_beta, None, 0, B, HW, C)
    lp.cmp(name, d, "y", y.reshape(B, HW, C), _apply_ref(zr, mean_rstd, gamma, beta, res, relu, B, HW, C))


def check_bn_apply(lp, name, launch, z, mean_rstd, gamma, beta, residual, y, B, HW, C, relu):
    zr, rr = _keep_inputs(y, z, residual)
    launch(z, mean_rstd, gamma, beta, residual, y, B, HW, C, relu)
    d = "C%d HW%d B%d relu%d%s" % (C, HW, B, relu, " +res" if residual is not None else "")
    lp.cmp(name, d, "y", y.reshape(B, HW, C), _apply_ref(zr, mean_rstd, gamma, beta, rr, relu, B, HW, C))


def _bn_bwd_ref(dy, z, mr, gamma, B, HW, C, mask, sums=None, group=1):
    """dz, g, per-image (sum g, sum g*xhat) of a BN backward; mask [B,HW,C] bool or None;
    sums: the kernel's own per-image first-pass sums (teacher-forced second pass) or None."""
    g = dy.reshape(B, HW, C).double()
    if mask is not None:
        g = g * mask.double()
    m, rs = mr.view(B, C, 2)[..., 0], mr.view(B, C, 2)[..., 1]
    xh = ((z.reshape(B, HW, C).float() - m[:, None].float()) * rs[:, None].float()).double()
    if sums is None:
        s1, s2 = g.sum(1), (g * xh).sum(1)
    else:                                   # accumulator buffer, or plain float64 [B][C][2] values
        sv = sums.view(B, C, 2).double() if sums.dtype == F64 else _acc(sums, B, C)
        s1, s2 = sv[..., 0], sv[..., 1]
    if group > 1:
        ng = (B + group - 1) // group
        gi = torch.arange(B, device=g.device) // group
        t1 = torch.stack([s1[k * group:(k + 1) * group].sum(0) for k in range(ng)])[gi]
        t2 = torch.stack([s2[k * group:(k + 1) * group].sum(0) for k in range(ng)])[gi]
        cnt = torch.tensor([min(group, B - (int(i) // group) * group) for i in range(B)], dtype=F64,
                           device=g.device)
        n = HW * cnt[:, None]
    else:
        t1, t2, n = s1, s2, float(HW)
    dz = gamma.double() * rs.double()[:, None] * (g - (t1 / n)[:, None] - xh * (t2 / n)[:, None])
    return dz, g, s1, s2, xh


def _check_bn_bwd(lp, name, d, dy, z, mr, gamma, dz, dz_old, dz_beta, g_out, dgamma, dbeta, dg0, db0, beta_acc,
                  conv_dbias, B, HW, C, mask, sums=None, group=1):
    rdz, g, s1, s2, xh = _bn_bwd_ref(dy, z, mr, gamma, B, HW, C, mask, sums, group)
    if dz_beta:
        rdz = rdz + dz_beta * dz_old.reshape(B, HW, C).double()
    lp.cmp(name, d, "dz", dz.reshape(B, HW, C), rdz)
    if g_out is not None:
        lp.cmp(name, d, "g_out", g_out.reshape(B, HW, C), g)
    if dgamma is not None:
        rg, rb = s2.sum(0), s1.sum(0)
        ag = (g * xh).abs().sum((0, 1)) if sums is None else s2.abs().sum(0)
        ab = g.abs().sum((0, 1)) if sums is None else s1.abs().sum(0)
        if beta_acc:
            rg, rb = rg + beta_acc * dg0.double(), rb + beta_acc * db0.double()
            ag, ab = ag + abs(beta_acc) * dg0.double().abs(), ab + abs(beta_acc) * db0.double().abs()
        lp.add(name, d, "dgamma", red_err(dgamma, rg, ag), TOL_F32)
        lp.add(name, d, "dbeta", red_err(dbeta, rb, ab), TOL_F32)
    if conv_dbias is not None:
        lp.add(name, d, "conv_dbias", float(conv_dbias.abs().max()), 0.0)


def _mask_relu_z(z, mr, gamma, beta, B, HW, C, act_hi=float("inf")):
    m, rs = mr.view(B, C, 2)[..., 0], mr.view(B, C, 2)[..., 1]
    a, _ = bn_affine32(z.reshape(B, HW, C), m[:, None], rs[:, None], gamma, beta)
    return (a > 0) & (a < act_hi)


def _clone(*ts):
    return [t.clone() if t is not None else None for t in ts]


def _keep_inputs(out, *ins):
    """Inputs that share storage with the launch's output are snapshotted first (in-place forms);
    the kernel still reads the original tensors."""
    res = []
    for t in ins:
        if t is not None and out is not None and t.untyped_storage().data_ptr() == out.untyped_storage().data_ptr():
            t = t.clone()
        res.append(t)
    return res


def check_bn_backward(lp, name, launch, dy, y_relu, z, mean_rstd, gamma, dz, g_out, dgamma, dbeta, B, HW, C,
                      beta_acc=0.0, conv_dbias=None):
    dg0, db0 = _clone(dgamma, dbeta)
    dyr, zr = _keep_inputs(dz, dy, z)
    (yr,) = _keep_inputs(dz, y_relu)
    launch(dy, y_relu, z, mean_rstd, gamma, dz, g_out, dgamma, dbeta, B, HW, C, beta_acc=beta_acc,
           conv_dbias=conv_dbias)
    mask = (yr.reshape(B, HW, C).float() > 0) if yr is not None else None
    _check_bn_bwd(lp, name, "C%d HW%d B%d%s" % (C, HW, B, " relu(y)" if mask is not None else ""), dyr, zr, mean_rstd,
                  gamma, dz, None, 0.0, g_out, dgamma, dbeta, dg0, db0, beta_acc, conv_dbias, B, HW, C, mask)


def check_bn_backward_relu(lp, name, launch, dy, z, mean_rstd, gamma, beta, dz, dgamma, dbeta, B, HW, C, beta_acc=0.0,
                           conv_dbias=None):
    dg0, db0 = _clone(dgamma, dbeta)
    dyr, zr = _keep_inputs(dz, dy, z)
    launch(dy, z, mean_rstd, gamma, beta, dz, dgamma, dbeta, B, HW, C, beta_acc=beta_acc, conv_dbias=conv_dbias)
    mask = _mask_relu_z(zr, mean_rstd, gamma, beta, B, HW, C)
    _check_bn_bwd(lp, name, "C%d HW%d B%d relu(z)" % (C, HW, B), dyr, zr, mean_rstd, gamma, dz, None, 0.0, None, dgamma,
                  dbeta, dg0, db0, beta_acc, conv_dbias, B, HW, C, mask)


def check_bn_backward_relu6(lp, name, launch, dy, z, mean_rstd, gamma, beta, dz, dgamma, dbeta, B, HW, C,
                            beta_acc=0.0, conv_dbias=None):
    dg0, db0 = _clone(dgamma, dbeta)
    dyr, zr = _keep_inputs(dz, dy, z)
    launch(dy, z, mean_rstd, gamma, beta, dz, dgamma, dbeta, B, HW, C, beta_acc=beta_acc, conv_dbias=conv_dbias)
    mask = _mask_relu_z(zr, mean_rstd, gamma, beta, B, HW, C, 6.0)
    _check_bn_bwd(lp, name, "C%d HW%d B%d relu6(z)" % (C, HW, B), dyr, zr, mean_rstd, gamma, dz, None, 0.0, None,
                  dgamma, dbeta, dg0, db0, beta_acc, conv_dbias, B, HW, C, mask)


def check_bn_backward_relu_sums(lp, name, launch, dy, z, mean_rstd, gamma, beta, sums, dz, dgamma, dbeta, B, HW, C,
                                beta_acc=0.0, conv_dbias=None, act_hi=float("inf")):
    dg0, db0 = _clone(dgamma, dbeta)
    dyr, zr = _keep_inputs(dz, dy, z)
    launch(dy, z, mean_rstd, gamma, beta, sums, dz, dgamma, dbeta, B, HW, C, beta_acc=beta_acc, conv_dbias=conv_dbias,
           act_hi=act_hi)
    mask = _mask_relu_z(zr, mean_rstd, gamma, beta, B, HW, C, act_hi)
    _check_bn_bwd(lp, name, "C%d HW%d B%d sums" % (C, HW, B), dyr, zr, mean_rstd, gamma, dz, None, 0.0, None, dgamma,
                  dbeta, dg0, db0, beta_acc, conv_dbias, B, HW, C, mask, sums=sums)


def check_bn_backward_res_sums(lp, name, launch, dy, y, z, mean_rstd, gamma, sums, dz, g_out, dgamma, dbeta, B, HW, C,
                               beta_acc=0.0, conv_dbias=None):
    dg0, db0 = _clone(dgamma, dbeta)
    dyr, zr = _keep_inputs(dz, dy, z)
    (yr,) = _keep_inputs(dz, y)
    launch(dy, y, z, mean_rstd, gamma, sums, dz, g_out, dgamma, dbeta, B, HW, C, beta_acc=beta_acc,
           conv_dbias=conv_dbias)
    mask = yr.reshape(B, HW, C).float() > 0
    _check_bn_bwd(lp, name, "C%d HW%d B%d res sums" % (C, HW, B), dyr, zr, mean_rstd, gamma, dz, None, 0.0, g_out,
                  dgamma, dbeta, dg0, db0, beta_acc, conv_dbias, B, HW, C, mask, sums=sums)


def check_bn_backward_res_sums_sc(lp, name, launch, dy, y, z, mean_rstd, gamma, sums, dz, g_out, dgamma, dbeta,
                                  z_sc, mean_rstd_sc, sc_sums, B, HW, C, beta_acc=0.0, conv_dbias=None):
    """check_bn_backward_res_sums, plus the projection shortcut BN's first pass formed on the way:
    sc_sums = per-image (sum g_out, sum g_out * xhat_sc) against float64."""
    dg0, db0 = _clone(dgamma, dbeta)
    dyr, zr = _keep_inputs(dz, dy, z)
    (yr,) = _keep_inputs(dz, y)
    launch(dy, y, z, mean_rstd, gamma, sums, dz, g_out, dgamma, dbeta, z_sc, mean_rstd_sc, sc_sums, B, HW, C,
           beta_acc=beta_acc, conv_dbias=conv_dbias)
    mask = yr.reshape(B, HW, C).float() > 0
    d = "C%d HW%d B%d res sums +sc" % (C, HW, B)
    _check_bn_bwd(lp, name, d, dyr, zr, mean_rstd, gamma, dz, None, 0.0, g_out, dgamma, dbeta, dg0, db0, beta_acc,
                  conv_dbias, B, HW, C, mask, sums=sums)
    g = g_out.reshape(B, HW, C).double()
    ms, rss = mean_rstd_sc.view(B, C, 2)[..., 0], mean_rstd_sc.view(B, C, 2)[..., 1]
    xh = ((z_sc.reshape(B, HW, C).float() - ms[:, None].float()) * rss[:, None].float()).double()
    ref = torch.stack([g.sum(1), (g * xh).sum(1)], -1)
    rabs = torch.stack([g.abs().sum(1), (g * xh).abs().sum(1)], -1)
    lp.add(name, d, "sc_sums", red_err(sc_sums.view(B, C, 2).double(), ref, rabs), 1e-6)


def check_bn_backward_sc(lp, name, launch, dy, y, z, mean_rstd, gamma, dz, g_out, dgamma, dbeta, z_sc, mean_rstd_sc,
                         sc_sums, B, HW, C, beta_acc=0.0, conv_dbias=None):
    """check_bn_backward (mask y > 0, g_out), plus the projection shortcut BN's first-pass sums."""
    dg0, db0 = _clone(dgamma, dbeta)
    dyr, zr = _keep_inputs(dz, dy, z)
    (yr,) = _keep_inputs(dz, y)
    launch(dy, y, z, mean_rstd, gamma, dz, g_out, dgamma, dbeta, z_sc, mean_rstd_sc, sc_sums, B, HW, C,
           beta_acc=beta_acc, conv_dbias=conv_dbias)
    mask = yr.reshape(B, HW, C).float() > 0
    d = "C%d HW%d B%d relu(y) +sc" % (C, HW, B)
    _check_bn_bwd(lp, name, d, dyr, zr, mean_rstd, gamma, dz, None, 0.0, g_out, dgamma, dbeta, dg0, db0, beta_acc,
                  conv_dbias, B, HW, C, mask)
    g = g_out.reshape(B, HW, C).double()
    ms, rss = mean_rstd_sc.view(B, C, 2)[..., 0], mean_rstd_sc.view(B, C, 2)[..., 1]
    xh = ((z_sc.reshape(B, HW, C).float() - ms[:, None].float()) * rss[:, None].float()).double()
    ref = torch.stack([g.sum(1), (g * xh).sum(1)], -1)
    rabs = torch.stack([g.abs().sum(1), (g * xh).abs().sum(1)], -1)
    lp.add(name, d, "sc_sums", red_err(sc_sums.view(B, C, 2).double(), ref, rabs), 1e-6)


def check_bn_backward_sums(lp, name, launch, dy, z, mean_rstd, gamma, sums, dz, dgamma, dbeta, B, HW, C, beta_acc=0.0,
                           conv_dbias=None):
    dg0, db0 = _clone(dgamma, dbeta)
    dyr, zr = _keep_inputs(dz, dy, z)
    launch(dy, z, mean_rstd, gamma, sums, dz, dgamma, dbeta, B, HW, C, beta_acc=beta_acc, conv_dbias=conv_dbias)
    _check_bn_bwd(lp, name, "C%d HW%d B%d sums, no mask" % (C, HW, B), dyr, zr, mean_rstd, gamma, dz, None, 0.0,
                  None, dgamma, dbeta, dg0, db0, beta_acc, conv_dbias, B, HW, C, None, sums=sums)


def check_bn_stats(lp, name, launch, x, B, HW, C, stats):
    launch(x, B, HW, C, stats)
    xx = x.reshape(B, HW, -1)[..., :C].double()
    ref = torch.stack([xx.sum(1), (xx * xx).sum(1)], -1)
    rabs = torch.stack([xx.abs().sum(1), (xx * xx).sum(1)], -1)
    lp.add(name, "C%d HW%d B%d" % (C, HW, B), "stats", red_err(_acc(stats, B, C), ref, rabs), 1e-6)


def check_bn_finalize_grouped(lp, name, launch, stats, mean_rstd, run_mean, run_var, B, C, HW, group, eps, momentum):
    rm0, rv0 = _clone(run_mean, run_var)
    launch(stats, mean_rstd, run_mean, run_var, B, C, HW, group, eps, momentum)
    _check_finalize(lp, name, "C%d HW%d B%d grp%d" % (C, HW, B, group), stats, mean_rstd, rm0, rv0, run_mean, run_var,
                    B, C, HW, eps, momentum, group=group)


def check_bn_backward_grouped(lp, name, launch, dy, z, mean_rstd, gamma, dz, dgamma, dbeta, B, HW, C, group,
                              dz_beta=0.0, y_relu=None):
    dz_old = dz.clone() if dz_beta else None
    dyr, zr = _keep_inputs(dz, dy, z)
    (yr,) = _keep_inputs(dz, y_relu)
    launch(dy, z, mean_rstd, gamma, dz, dgamma, dbeta, B, HW, C, group, dz_beta=dz_beta, y_relu=y_relu)
    mask = (yr.reshape(B, HW, C).float() > 0) if yr is not None else None
    _check_bn_bwd(lp, name, "C%d HW%d B%d grp%d" % (C, HW, B, group), dyr, zr, mean_rstd, gamma, dz, dz_old, dz_beta,
                  None, dgamma, dbeta, None, None, 0.0, None, B, HW, C, mask, group=group)


# ================================================================================================
# pooling / resampling / elementwise
# ================================================================================================
def _pool3_ref(a):
    """ZeroPadding2D(1) + MaxPool 3x3/2 (first maximum in window order) of a [B,H,W,C] -> (y, arg)."""
    B, H, W, C = a.shape
    Ho, Wo = (H + 2 - 3) // 2 + 1, (W + 2 - 3) // 2 + 1
    ap = F.pad(a.permute(0, 3, 1, 2).float(), (1, 1, 1, 1))
    win = F.unfold(ap, 3, stride=2).view(B, C, 9, Ho * Wo)           # taps t = ky*3 + kx in window order
    best, arg = win.max(2)                                            # ties: torch's max returns the first?
    first = (win == best.unsqueeze(2)).float().argmax(2)              # explicit first maximum
    return best.view(B, C, Ho, Wo).permute(0, 2, 3, 1), first.view(B, C, Ho, Wo).permute(0, 2, 3, 1)


def _pool3_bwd_ref(dy, arg, H, W):
    B, Ho, Wo, C = dy.shape
    oh = torch.nn.functional.one_hot(arg.long(), 9).double() * dy.double().unsqueeze(-1)   # [B,Ho,Wo,C,9]
    cols = oh.permute(0, 3, 4, 1, 2).reshape(B, C * 9, Ho * Wo)
    dxp = F.fold(cols, (2 * (Ho - 1) + 3, 2 * (Wo - 1) + 3), 3, stride=2)
    dxp = F.pad(dxp, (0, max(0, W + 1 - dxp.shape[3]), 0, max(0, H + 1 - dxp.shape[2])))
    return dxp[:, :, 1:1 + H, 1:1 + W].permute(0, 2, 3, 1)


def check_maxpool3x3s2(lp, name, launch, x, y, argmax):
    launch(x, y, argmax)
    ry, ra = _pool3_ref(x)
    d = "3x3/2 %dx%dx%d B%d" % (x.shape[1], x.shape[2], x.shape[3], x.shape[0])
    lp.exact(name, d, "y", y, ry.to(y.dtype))
    lp.exact(name, d, "argmax", argmax, ra.to(torch.uint8))


def check_bn_relu_maxpool(lp, name, launch, z, mean_rstd, gamma, beta, y, argmax):
    launch(z, mean_rstd, gamma, beta, y, argmax)
    B, H, W, C = z.shape
    m, rs = mean_rstd.view(B, C, 2)[..., 0], mean_rstd.view(B, C, 2)[..., 1]
    a, _ = bn_affine32(z.reshape(B, H * W, C), m[:, None], rs[:, None], gamma, beta)
    a = a.clamp_min(0).to(torch.bfloat16).view(B, H, W, C)
    ry, ra = _pool3_ref(a)
    d = "stem bn+relu+pool %dx%dx%d B%d" % (H, W, C, B)
    lp.exact(name, d, "y", y, ry.to(y.dtype), frac_tol=1e-5)
    lp.exact(name, d, "argmax", argmax, ra.to(torch.uint8), frac_tol=1e-5)


def check_maxpool3x3s2_backward(lp, name, launch, dy, argmax, dx):
    launch(dy, argmax, dx)
    B, H, W, C = dx.shape
    lp.cmp(name, "3x3/2 bwd %dx%dx%d B%d" % (H, W, C, B), "dx", dx, _pool3_bwd_ref(dy, argmax, H, W))


def check_maxpool3x3s2_backward_bn_relu(lp, name, launch, dp, argmax, z, mean_rstd, gamma, beta, dy, dz, dgamma, dbeta,
                                        beta_acc=0.0, conv_dbias=None):
    """The stem's fused pool1 / conv1_relu / conv1_bn backward: dy against the pool reference, then dz /
    dgamma / dbeta / conv_dbias as check_bn_backward_relu on that dy."""
    dg0, db0 = _clone(dgamma, dbeta)
    (zr,) = _keep_inputs(dz, z)
    launch(dp, argmax, z, mean_rstd, gamma, beta, dy, dz, dgamma, dbeta, beta_acc=beta_acc, conv_dbias=conv_dbias)
    B, H, W, C = z.shape
    HW = H * W
    lp.cmp(name, "3x3/2 bwd %dx%dx%d B%d" % (H, W, C, B), "dy", dy, _pool3_bwd_ref(dp, argmax, H, W))
    dyr = dy.clone()
    mask = _mask_relu_z(zr, mean_rstd, gamma, beta, B, HW, C)
    _check_bn_bwd(lp, name, "C%d HW%d B%d pool relu(z)" % (C, HW, B), dyr, zr, mean_rstd, gamma, dz, None, 0.0, None,
                  dgamma, dbeta, dg0, db0, beta_acc, conv_dbias, B, HW, C, mask)


def _up2(b):
    return b.repeat_interleave(2, 1).repeat_interleave(2, 2)


def check_upsample2x_add(lp, name, launch, a, b, out, B, H, W, C):
    a0, b0 = a.clone(), b.clone()
    launch(a, b, out, B, H, W, C)
    ref = a0.reshape(B, H, W, C).double() + _up2(b0.reshape(B, H // 2, W // 2, C).double())
    lp.cmp(name, "nearest up2 add %dx%dx%d B%d" % (H, W, C, B), "out", out.reshape(B, H, W, C), ref)


def check_upsample2x_backward(lp, name, launch, dout, db, B, H, W, C, beta=0.0):
    old = db.clone() if beta else None
    launch(dout, db, B, H, W, C, beta)
    d = dout.reshape(B, H // 2, 2, W // 2, 2, C).double().sum((2, 4))
    if beta:
        d = d + beta * old.reshape(d.shape).double()
    lp.cmp(name, "nearest up2 bwd %dx%dx%d B%d" % (H, W, C, B), "db", db.reshape(d.shape), d)


def check_relu_backward(lp, name, launch, dy, y, dx, beta=0.0):
    old = dx.clone() if beta else None
    dy0, y0 = dy.clone(), y.clone()
    launch(dy, y, dx, beta)
    ref = dy0.reshape(-1).double() * (y0.reshape(-1).float() > 0).double()
    if beta:
        ref = ref + beta * old.reshape(-1).double()
    lp.cmp(name, "n%d" % dy.numel(), "dx", dx.reshape(-1), ref)


def check_add(lp, name, launch, a, b, out):
    a0, b0 = a.clone(), b.clone()          # out may alias an operand (in-place add)
    launch(a, b, out)
    lp.cmp(name, "n%d" % a.numel(), "out", out.reshape(-1), a0.reshape(-1).double() + b0.reshape(-1).double())


def _bias_ref(dy, ld, coff, ncol, base, img_stride, HW, B):
    rows = _rows(dy, ld)
    idx = _row_index(int(base), int(img_stride), list(range(B)), HW, dy.device)
    t = rows[idx, coff:coff + ncol].double()
    return t.sum(0), t.abs().sum(0)


def check_bias_grad(lp, name, launch, dy, ld, coff, ncol, base, img_stride, HW, B, db, beta=0.0):
    old = db.clone() if beta else None
    launch(dy, ld, coff, ncol, base, img_stride, HW, B, db, beta)
    r, ra = _bias_ref(dy, ld, coff, ncol, base, img_stride, HW, B)
    if beta:
        r, ra = r + beta * old.double(), ra + abs(beta) * old.double().abs()
    lp.add(name, "ncol%d HW%d B%d" % (ncol, HW, B), "db", red_err(db[:ncol], r, ra), TOL_F32)


def check_bias_grad_multi(lp, name, launch, items):
    olds = [it[8].clone() if it[9] else None for it in items]
    launch(items)
    for it, old in zip(items, olds):
        dy, ld, coff, ncol, base, img_stride, HW, B, db, beta = it
        r, ra = _bias_ref(dy, ld, coff, ncol, base, img_stride, HW, B)
        if beta:
            r, ra = r + beta * old.double(), ra + abs(beta) * old.double().abs()
        lp.add(name, "ncol%d HW%d B%d" % (ncol, HW, B), "db", red_err(db[:ncol], r, ra), TOL_F32)


# ================================================================================================
# optimizer / schedule / misc
# ================================================================================================
def _upd_err(w, w0, upd_ref):
    """max over elements of |w - (w0 + upd)| / (1e-4 |upd| + 2 ulp(w)): an fp32 weight update
    checked to the fp32 tolerance on the UPDATE (the rounding of w + update is an ulp of w)."""
    ref = w0.double() + upd_ref
    ulp = torch.finfo(torch.float32).eps * ref.abs().clamp_min(torch.finfo(torch.float32).tiny)
    return float(((w.double() - ref).abs() / (1e-4 * upd_ref.abs() + 2 * ulp)).max())


def check_sgd(lp, name, launch, w, g, v, lr_dev, momentum, inv_bs, clip, ws=None):
    w0, v0 = w.clone(), v.clone()
    launch(w, g, v, lr_dev, momentum, inv_bs, clip, ws=ws)
    gg = g.double() * inv_bs
    norm = float(gg.norm())
    scale = clip / max(norm, clip) if clip > 0 else 1.0
    rv = momentum * v0.double() - float(lr_dev.double().item()) * gg * scale
    d = "n%d clip%g |g|%.3g" % (w.numel(), clip, norm)
    lp.cmp(name, d, "v", v, rv, tol=TOL_F32)
    lp.add(name, d, "w", _upd_err(w, w0, v.double()), 1.0)


def check_adam(lp, name, launch, w, g, m, v, lr_dev, iterations, beta1, beta2, eps, inv_bs, clip, ws=None):
    w0, m0, v0 = w.clone(), m.clone(), v.clone()
    it0 = int(iterations.item())
    launch(w, g, m, v, lr_dev, iterations, beta1, beta2, eps, inv_bs, clip, ws=ws)
    gg = g.double() * inv_bs
    norm = float(gg.norm())
    gg = gg * (clip / max(norm, clip) if clip > 0 else 1.0)
    t = it0 + 1
    lr = float(lr_dev.double().item())
    rm = beta1 * m0.double() + (1 - beta1) * gg
    rv = beta2 * v0.double() + (1 - beta2) * gg * gg
    lr_t = lr * math.sqrt(1 - beta2 ** t) / (1 - beta1 ** t)
    d = "n%d t%d |g|%.3g" % (w.numel(), t, norm)
    lp.cmp(name, d, "m", m, rm, tol=TOL_F32)
    lp.cmp(name, d, "v", v, rv, tol=TOL_F32)
    # the step from the kernel's own moments (teacher-forced): w = w0 - lr_t m / (sqrt(v) + eps)
    lp.add(name, d, "w", _upd_err(w, w0, -lr_t * m.double() / (torch.sqrt(v.double()) + eps)), 1.0)


def check_lr_schedule(lp, name, launch, step_dev, lr_dev, init_lr, min_lr, decay_rate, decay_step, max_decays=None):
    s0 = int(step_dev.item())
    launch(step_dev, lr_dev, init_lr, min_lr, decay_rate, decay_step, max_decays=max_decays)
    k = s0 // decay_step
    if max_decays is not None:
        k = min(k, max_decays)
    ref = max(init_lr * decay_rate ** k, min_lr)
    lp.add(name, "step %d" % s0, "lr", abs(float(lr_dev.item()) - ref) / ref, 1e-6)


def check_l2reg(lp, name, launch, obj):
    launch()
    st = obj.store
    ref = sum(math.sqrt(float((st.p(n).double() ** 2).sum()) / 2.0) for n in st.offsets)
    lp.add("L2Reg.run", "%d tensors" % len(st.offsets), "l2", abs(float(obj.out.item()) - ref) / max(ref, 1e-30), 1e-5)


def check_passthrough(lp, name, launch, *a, **k):
    """Launches checked by a dedicated test rather than here (recorded for the coverage list)."""
    out = launch(*a, **k)
    lp.add(name, "covered by " + PASSTHROUGH_TESTS.get(name, "?"), "-", 0.0, 0.0)
    return out


# ---- depthwise / separable / bilinear (CenterNet hourglass) --------------------------------------
def _dw_weight(w, k, C):
    return w.reshape(k, k, C).permute(2, 0, 1).unsqueeze(1).double()      # [C,1,k,k]


def check_depthwise_fwd(lp, name, launch, x, w, y, k, stride, pad_t, pad_l):
    launch(x, w, y, k, stride, pad_t, pad_l)
    B, H, W, C = x.shape
    Ho, Wo = y.shape[1], y.shape[2]
    xp = _pad_crop(x.double().permute(0, 3, 1, 2), k, k, stride, pad_t, pad_l, Ho, Wo)
    ref = F.conv2d(xp.cpu(), _dw_weight(w, k, C).cpu(), stride=stride, groups=C).to(x.device).permute(0, 2, 3, 1)
    lp.cmp(name, "dw%d/%d %dx%dx%d B%d" % (k, stride, H, W, C, B), "y", y, ref)


def check_depthwise_dgrad(lp, name, launch, dy, w, dx, k, stride, pad_t, pad_l, beta=0.0):
    old = dx.clone() if beta else None
    launch(dy, w, dx, k, stride, pad_t, pad_l, beta=beta)
    B, H, W, C = dx.shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    x = torch.zeros((B, C, H, W), dtype=F64, requires_grad=True)
    xp = _pad_crop(x, k, k, stride, pad_t, pad_l, Ho, Wo)
    yy = F.conv2d(xp, _dw_weight(w, k, C).cpu(), stride=stride, groups=C)
    (gx,) = torch.autograd.grad(yy, x, dy.double().permute(0, 3, 1, 2).cpu())
    ref = gx.permute(0, 2, 3, 1).to(dx.device)
    if beta:
        ref = ref + beta * old.double()
    lp.cmp(name, "dw%d/%d bwd %dx%dx%d B%d" % (k, stride, H, W, C, B), "dx", dx, ref)


def check_depthwise_wgrad(lp, name, launch, x, dy, dw, k, stride, pad_t, pad_l, beta=0.0):
    old = dw.clone() if beta else None
    launch(x, dy, dw, k, stride, pad_t, pad_l, beta=beta)
    B, H, W, C = x.shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    xp = _pad_crop(x.double().permute(0, 3, 1, 2), k, k, stride, pad_t, pad_l, Ho, Wo)
    cols = F.unfold(xp, k, stride=stride).view(B, C, k * k, Ho * Wo)
    g = dy.double().permute(0, 3, 1, 2).reshape(B, C, 1, Ho * Wo)
    r = (cols * g).sum((0, 3))                                            # [C, k*k]
    ra = (cols * g).abs().sum((0, 3))
    r, ra = r.t().reshape(-1), ra.t().reshape(-1)                         # [k*k][C] (HWC(1))
    if beta:
        r, ra = r + beta * old.reshape(-1).double(), ra + abs(beta) * old.reshape(-1).double().abs()
    lp.add(name, "dw%d/%d wgrad %dx%dx%d B%d" % (k, stride, H, W, C, B), "dW", red_err(dw.reshape(-1), r, ra), TOL_F32)


def check_maxpool2x2(lp, name, launch, x, y, argmax):
    launch(x, y, argmax)
    B, H, W, C = x.shape
    Ho, Wo = y.shape[1], y.shape[2]
    xp = F.pad(x.permute(0, 3, 1, 2).float(), (0, 2 * Wo - W, 0, 2 * Ho - H), value=float("-inf"))
    win = F.unfold(xp, 2, stride=2).view(B, C, 4, Ho * Wo)
    best = win.max(2).values
    first = (win == best.unsqueeze(2)).float().argmax(2)
    d = "2x2/2 %dx%dx%d B%d" % (H, W, C, B)
    lp.exact(name, d, "y", y, best.view(B, C, Ho, Wo).permute(0, 2, 3, 1).to(y.dtype))
    lp.exact(name, d, "argmax", argmax, first.view(B, C, Ho, Wo).permute(0, 2, 3, 1).to(torch.uint8))


def check_maxpool2x2_backward(lp, name, launch, dy, argmax, dx):
    launch(dy, argmax, dx)
    B, H, W, C = dx.shape
    Ho, Wo = dy.shape[1], dy.shape[2]
    oh = torch.nn.functional.one_hot(argmax.long(), 4).double() * dy.double().unsqueeze(-1)
    cols = oh.permute(0, 3, 4, 1, 2).reshape(B, C * 4, Ho * Wo)
    ref = F.fold(cols, (2 * Ho, 2 * Wo), 2, stride=2)[:, :, :H, :W].permute(0, 2, 3, 1)
    lp.cmp(name, "2x2/2 bwd %dx%dx%d B%d" % (H, W, C, B), "dx", dx, ref)


def _bilinear_up2(a):
    """Keras UpSampling2D(interpolation='bilinear') x2 = half-pixel bilinear (align_corners=False)."""
    return F.interpolate(a.double().permute(0, 3, 1, 2), scale_factor=2, mode="bilinear",
                         align_corners=False).permute(0, 2, 3, 1)


def check_upsample_bilinear2x_add(lp, name, launch, prev, other, out):
    launch(prev, other, out)
    ref = _bilinear_up2(prev) + other.double()
    lp.cmp(name, "bilinear up2 add %s" % (tuple(out.shape),), "out", out, ref)


def check_upsample_bilinear2x_sum(lp, name, launch, a, b, out):
    launch(a, b, out)
    s = a.double() if b is None else a.double() + b.double()
    lp.cmp(name, "bilinear up2 sum %s" % (tuple(out.shape),), "out", out, _bilinear_up2(s))


def check_upsample_bilinear2x_backward(lp, name, launch, dout, dprev, beta=0.0):
    old = dprev.clone() if beta else None
    launch(dout, dprev, beta=beta)
    p = torch.zeros(dprev.shape, dtype=F64, device=dprev.device, requires_grad=True)
    (g,) = torch.autograd.grad(_bilinear_up2(p), p, dout.double())
    if beta:
        g = g + beta * old.double()
    lp.cmp(name, "bilinear up2 bwd %s" % (tuple(dprev.shape),), "dprev", dprev, g)


def check_sep_fold(lp, name, launch, plan):
    launch()
    for dw, pw, weff, gweff, gdw, gpw in plan._keep:
        kh, kw, cin, _ = dw.shape
        cout = pw.shape[3]
        ref = dw.double().reshape(kh, kw, cin, 1) * pw.double().reshape(1, 1, cin, cout)
        lp.cmp("SepPlan.fold", "sep %dx%d %d->%d" % (kh, kw, cin, cout), "W", weff[:, :, :cin, :cout], ref, tol=1e-6)


def check_sep_unfold(lp, name, launch, plan):
    launch()
    for dw, pw, weff, gweff, gdw, gpw in plan._keep:
        kh, kw, cin, _ = dw.shape
        cout = pw.shape[3]
        G = gweff[:, :, :cin, :cout].double()
        rdw = (G * pw.double().reshape(1, 1, cin, cout)).sum(3).reshape(gdw.shape)
        rpw = (G * dw.double().reshape(kh, kw, cin, 1)).sum((0, 1)).reshape(gpw.shape)
        d = "sep %dx%d %d->%d" % (kh, kw, cin, cout)
        lp.add("SepPlan.unfold", d, "g_dw", red_err(gdw, rdw, (G * pw.double().reshape(1, 1, cin, cout)).abs()
                                                    .sum(3).reshape(gdw.shape)), TOL_F32)
        lp.add("SepPlan.unfold", d, "g_pw", red_err(gpw, rpw, (G * dw.double().reshape(kh, kw, cin, 1)).abs()
                                                    .sum((0, 1)).reshape(gpw.shape)), TOL_F32)


PASSTHROUGH_TESTS = {
    # fused target / loss kernels: bit-exact / 2e-5 vs the reference goldens and float64 autograd
    "fcos_assign": "test_gpu_fullsize + test_gpu_targets_loss (bit-exact)",
    "fcos_center_assign": "test_gpu_fcos_center (bit-exact)",
    "fcos_center_v1_assign": "test_gpu_fcos_center (bit-exact)",
    "retina_assign": "test_gpu_fullsize + test_gpu_retina_centernet (bit-exact)",
    "centernet_assign": "test_gpu_fullsize + test_gpu_retina_centernet (bit-exact)",
    "retina_loss": "test_gpu_fullsize (fp64 autograd at 640/C80)",
    "centernet_loss": "test_gpu_fullsize + test_gpu_hourglass (fp64 autograd)",
    "select_first_nonzero": "test_gpu_retina_model",
    "gather_rows": "test_gpu_retina_model",
    "bias_scalar_fold": "test_gpu_hourglass", "bias_scalar_unfold": "test_gpu_hourglass",
    "bias_scalar_fold_periodic": "test_gpu_hourglass_v2", "bias_scalar_unfold_periodic": "test_gpu_hourglass_v2",
    "reshape_concat": "test_gpu_hourglass_v2", "reshape_concat_backward": "test_gpu_hourglass_v2",
}


def check_fcos_loss(lp, name, launch, reg_pred, cls_pred, targets, num_classes, reg_type="l1", grad_scale=1.0,
                    with_grad=True, grad_dtype=torch.float32, d_reg=None, d_cls=None, cen_type="l1",
                    reg_sigmoid=False, cen_in_cls=False, losses=None):
    out = launch(reg_pred, cls_pred, targets, num_classes, reg_type=reg_type, grad_scale=grad_scale,
                 with_grad=with_grad, grad_dtype=grad_dtype, d_reg=d_reg, d_cls=d_cls, cen_type=cen_type,
                 reg_sigmoid=reg_sigmoid, cen_in_cls=cen_in_cls, losses=losses)
    losses, gr, gc = out
    if cen_type != "l1" or reg_sigmoid or cen_in_cls or not isinstance(reg_type, str):
        lp.add(name, "centre variant: test_gpu_fcos_center", "-", 0.0, 0.0)
        return out
    from oracle import fcos_torch
    C = num_classes
    B = targets.shape[0]
    errs = collections.defaultdict(list)
    for b in lp.img_set(B):
        tr = reg_pred[b].double().cpu().requires_grad_()
        tc = cls_pred[b].double().cpu().requires_grad_()
        lc, lr, le = fcos_torch.packed_loss(tr, tc, targets[b].double().cpu(), C, reg_type)
        (grad_scale * (lc + lr + le)).backward()
        ref = torch.stack([lc, lr, le]).detach()
        errs["losses"].append(float(((losses[b].double().cpu() - ref).abs() / ref.abs().clamp_min(1e-3)).max()))
        if with_grad:
            errs["d_reg"].append(rel_l2(gr[b, :, :5].cpu(), tr.grad[:, :5]))
            errs["d_cls"].append(rel_l2(gc[b, :, :C].cpu(), tc.grad[:, :C]))
    d = "B%d P%d C%d %s" % (B, targets.shape[1], C, reg_type)
    lp.add(name, d, "losses", max(errs["losses"]), 2e-5)
    if with_grad:
        tol = TOL_F32 if gr.dtype == torch.float32 else TOL_BF16
        lp.add(name, d, "d_reg", max(errs["d_reg"]), tol)
        lp.add(name, d, "d_cls", max(errs["d_cls"]), tol)
    return out


CHECKS = {
    "conv_igemm": check_conv_igemm,
    "conv_igemm_relu_mask": check_conv_igemm_relu_mask,
    "conv_wgrad": check_conv_wgrad,
    "conv_wgrad_grouped": check_conv_wgrad_grouped,
    "conv_wgrad_batch": check_conv_wgrad_batch,
    "conv_igemm_dgrad_bnsum": check_dgrad_bnsum,
    "conv_igemm_dgrad_bnsum_res": check_dgrad_bnsum_res,
    "pack_conv_weights": check_pack_conv_weights,
    "im2col": check_im2col,
    "stem_conv7x7s2": check_stem_conv,
    "stem_wgrad": check_stem_wgrad,
    "bn_finalize": check_bn_finalize,
    "bn_apply": check_bn_apply,
    "bn_finalize_apply": check_bn_finalize_apply,
    "bn_finalize_apply_bnres": check_bn_finalize_apply_bnres,
    "bn_backward": check_bn_backward,
    "bn_backward_relu": check_bn_backward_relu,
    "bn_backward_relu6": check_bn_backward_relu6,
    "bn_backward_relu_sums": check_bn_backward_relu_sums,
    "bn_backward_res_sums": check_bn_backward_res_sums,
    "bn_backward_res_sums_sc": check_bn_backward_res_sums_sc,
    "bn_backward_sums": check_bn_backward_sums,
    "bn_backward_sc": check_bn_backward_sc,
    "bn_relu_maxpool3x3s2": check_bn_relu_maxpool,
    "maxpool3x3s2": check_maxpool3x3s2,
    "maxpool3x3s2_backward": check_maxpool3x3s2_backward,
    "maxpool3x3s2_backward_bn_relu": check_maxpool3x3s2_backward_bn_relu,
    "upsample2x_add": check_upsample2x_add,
    "upsample2x_backward": check_upsample2x_backward,
    "relu_backward": check_relu_backward,
    "add": check_add,
    "bias_grad": check_bias_grad,
    "bias_grad_multi": check_bias_grad_multi,
    "sgd_clip_update": check_sgd,
    "adam_clip_update": check_adam,
    "lr_schedule": check_lr_schedule,
    "bn_stats": check_bn_stats,
    "bn_finalize_grouped": check_bn_finalize_grouped,
    "bn_backward_grouped": check_bn_backward_grouped,
    "depthwise_fwd": check_depthwise_fwd,
    "depthwise_dgrad": check_depthwise_dgrad,
    "depthwise_wgrad": check_depthwise_wgrad,
    "maxpool2x2": check_maxpool2x2,
    "maxpool2x2_backward": check_maxpool2x2_backward,
    "upsample_bilinear2x_add": check_upsample_bilinear2x_add,
    "upsample_bilinear2x_sum": check_upsample_bilinear2x_sum,
    "upsample_bilinear2x_backward": check_upsample_bilinear2x_backward,
}
for _n in ("select_first_nonzero", "gather_rows", "bias_scalar_fold", "bias_scalar_unfold",
           "bias_scalar_fold_periodic", "bias_scalar_unfold_periodic", "reshape_concat", "reshape_concat_backward"):
    CHECKS[_n] = check_passthrough

TARGET_CHECKS = {
    "fcos_loss": check_fcos_loss,
    "fcos_assign": check_passthrough,
    "fcos_center_assign": check_passthrough,
    "fcos_center_v1_assign": check_passthrough,
    "retina_assign": check_passthrough,
    "retina_loss": check_passthrough,
    "centernet_assign": check_passthrough,
    "centernet_loss": check_passthrough,
}
