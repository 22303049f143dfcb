"""Weight interchange with the reference's Keras models.

The reference saves `tf.train.Checkpoint(step, model, optimizer)` (FCOS/train_fcos.py:289-310,
RetinaNet/train_retinanet_coco.py:372-392).  TensorFlow is not part of this image, so the
interchange format here is the one a Keras user gets from `{v.name: v.numpy() for v in
model.variables}`: a flat .npz keyed by Keras variable names (`<layer>/<var>:0`), kernels in
Keras HWIO layout.  cvlite's parameter store already uses the Keras layer names
(`conv{2..5}_block{i}_{0..3}_{conv,bn}`, `c{3..7}_{1x1,3x3}`, `cls_layer_k`, `reg_layer_k`,
`logits_output_l`, `reg_output_l`, ...), so export/import is a renaming, except for:
  * BatchNormalization `moving_mean` / `moving_variance` (cvlite keeps them beside the store);
  * RetinaNet's per-(level, anchor) heads `cls_output_{l}_anchor_{a}` / `reg_output_{l}_anchor_{a}`
    (retinanet_module.py:115-148, Q28), which cvlite fuses into one conv per level: they are split
    / re-assembled along the output-channel axis (RetinaNetNet.keras_names).
Files are written with numpy (no pickle) and read with allow_pickle=False.
"""
import numpy as np
import torch


def model_bns(net):
    """Every BatchNorm layer (with moving statistics) of a cvlite network."""
    if hasattr(net, "bns"):
        return list(net.bns())
    bb = getattr(net, "backbone", None)
    return list(bb.bns()) if bb is not None and hasattr(bb, "bns") else []


_bns = model_bns


def _split_map(net):
    """{store name: [(keras var name, output-channel slice)]} for fused parameters."""
    out = {}
    if hasattr(net, "keras_names"):
        for kname, sname, sl in net.keras_names():
            out.setdefault(sname, []).append((kname, sl))
    return out


def keras_weights(net):
    """net (FCOSNet / RetinaNetNet) -> {Keras variable name: float32 ndarray}."""
    st = net.store
    split = _split_map(net)
    w = {}
    for name in st.offsets:
        a = st.p(name).detach().float().cpu().numpy()
        if name in split:
            for kname, sl in split[name]:
                w[kname + ":0"] = np.ascontiguousarray(a[..., sl])
        else:
            w[name + ":0"] = a
    for bn in _bns(net):
        w[bn.name + "/moving_mean:0"] = bn.run_mean.detach().cpu().numpy()
        w[bn.name + "/moving_variance:0"] = bn.run_var.detach().cpu().numpy()
    return w


def export_keras_weights(net, path):
    np.savez(path, **keras_weights(net))


def load_keras_weights(net, weights, strict=True):
    """Inverse of keras_weights: copy a {Keras variable name: array} dict into net (then re-pack
    the MFMA weight tiles).  strict: every store parameter and BN statistic must be present with
    its exact shape."""
    st = net.store
    split = _split_map(net)
    seen = set()

    def take(key, shape):
        if key not in weights:
            if strict:
                raise KeyError("missing Keras variable %s" % key)
            return None
        a = np.asarray(weights[key], dtype=np.float32)
        if tuple(a.shape) != tuple(shape):
            raise ValueError("%s: shape %s, expected %s" % (key, tuple(a.shape), tuple(shape)))
        seen.add(key)
        return a

    for name in st.offsets:
        dst = st.p(name)
        if name in split:
            full = dst.detach().float().cpu().numpy().copy()
            for kname, sl in split[name]:
                a = take(kname + ":0", full[..., sl].shape)
                if a is not None:
                    full[..., sl] = a
            dst.copy_(torch.from_numpy(full).to(dst.device, dst.dtype))
        else:
            a = take(name + ":0", tuple(dst.shape))
            if a is not None:
                dst.copy_(torch.from_numpy(a).to(dst.device, dst.dtype))
    for bn in _bns(net):
        for attr, var in (("run_mean", "moving_mean"), ("run_var", "moving_variance")):
            t = getattr(bn, attr)
            a = take("%s/%s:0" % (bn.name, var), tuple(t.shape))
            if a is not None:
                t.copy_(torch.from_numpy(a).to(t.device))
    if strict:
        extra = sorted(set(weights) - seen)
        if extra:
            raise KeyError("unused Keras variables: %s" % extra[:5])
    net.pack()
    return net


def import_keras_weights(net, path, strict=True):
    with np.load(path, allow_pickle=False) as z:
        return load_keras_weights(net, {k: z[k] for k in z.files}, strict=strict)


# -------------------------------------------------------------------------------------------------
# Training-state checkpoints: the tf.train.Checkpoint / tf.train.CheckpointManager pair the
# reference loops use for resume (FCOS/train_fcos.py:289-310, RetinaNet/train_retinanet_coco.py,
# CenterNet/train_hourglass_voc.py).  A checkpoint holds the step counter, every parameter, the
# optimizer slots (SGD momentum lives in the store, Adam m / v / iterations in the optimizer) and
# the BatchNorm moving statistics; the parameter names are checked against the current layout on
# restore.  Files are torch archives of plain tensors (read back with weights_only=True).
# -------------------------------------------------------------------------------------------------
def _net_of(obj):
    """The cvlite network behind a model object (FCOSModel.net, RetinaNet.model, or the net)."""
    for attr in ("net", "model"):
        inner = getattr(obj, attr, None)
        if inner is not None and hasattr(inner, "store"):
            return inner
    return obj if hasattr(obj, "store") else None


def net_state(net):
    st = net.store
    return {"params": st.flat.detach().cpu().clone(), "momentum": st.mom.detach().cpu().clone(),
            "names": [[k, int(o), int(n)] for k, (o, n, _) in st.offsets.items()],
            "bn": {bn.name: (bn.run_mean.detach().cpu().clone(), bn.run_var.detach().cpu().clone())
                   for bn in model_bns(net)}}


def load_net_state(net, s):
    st = net.store
    names = [[k, int(o), int(n)] for k, (o, n, _) in st.offsets.items()]
    if [list(x) for x in s["names"]] != names:
        raise ValueError("checkpoint parameter layout does not match this model")
    st.flat.copy_(s["params"].to(st.flat.device))
    st.mom.copy_(s["momentum"].to(st.flat.device))
    for bn in model_bns(net):
        m, v = s["bn"][bn.name]
        bn.run_mean.copy_(m)
        bn.run_var.copy_(v)
    net.pack()


def _opt_state(opt):
    if getattr(opt, "m", None) is not None:            # train_centernet.Adam once bound
        return {"m": opt.m.detach().cpu().clone(), "v": opt.v.detach().cpu().clone(),
                "iterations": opt.iterations.detach().cpu().clone()}
    return {}


def _load_opt_state(opt, s):
    """Adam slots into a bound optimizer, or kept on it until bind() (a restore before the trainer
    exists must not silently restart Adam at m = v = iterations = 0)."""
    if not s:
        return
    if getattr(opt, "m", None) is not None:
        opt.load_state(s)
    elif hasattr(opt, "pending_state"):
        opt.pending_state = s
    else:
        raise ValueError("checkpoint holds optimizer slots this optimizer object cannot take")


class Variable(object):
    """tf.Variable stand-in for the integer step counter (`ckpt.step.assign_add(1)`)."""

    def __init__(self, value=0):
        self.value = int(value)

    def assign_add(self, n):
        self.value += int(n)
        return self

    def assign(self, v):
        self.value = int(v)
        return self

    def numpy(self):
        return np.int64(self.value)


class Checkpoint(object):
    """tf.train.Checkpoint(step=tf.Variable(0), <model>=..., <optimizer>=...)."""

    def __init__(self, step=None, **objects):
        self.step = step if isinstance(step, Variable) else Variable(0 if step is None else step)
        self.objects = objects

    def state(self):
        out = {"step": self.step.value, "objects": {}}
        for name, obj in self.objects.items():
            net = _net_of(obj)
            out["objects"][name] = net_state(net) if net is not None else _opt_state(obj)
        return out

    def write(self, path):
        torch.save(self.state(), path)
        return path

    def restore(self, path):
        if path is None:
            return self
        s = torch.load(path, weights_only=True)
        self.step.assign(int(s["step"]))
        for name, obj in self.objects.items():
            if name not in s["objects"]:
                raise KeyError("checkpoint has no object %r" % name)
            net = _net_of(obj)
            if net is not None:
                load_net_state(net, s["objects"][name])
            else:
                _load_opt_state(obj, s["objects"][name])
        return self


class CheckpointManager(object):
    """tf.train.CheckpointManager(checkpoint, directory, max_to_keep): save() writes
    `<directory>/ckpt-<n>.pt` and keeps the newest max_to_keep; latest_checkpoint is the newest."""

    def __init__(self, checkpoint, directory, max_to_keep=1):
        import os
        self.checkpoint, self.directory, self.max_to_keep = checkpoint, directory, int(max_to_keep)
        os.makedirs(directory, exist_ok=True)
        self._counter = max([n for n, _ in self._existing()] or [0])

    def _existing(self):
        import os
        import re
        out = []
        for f in os.listdir(self.directory):
            m = re.match(r"ckpt-(\d+)\.pt$", f)
            if m:
                out.append((int(m.group(1)), os.path.join(self.directory, f)))
        return sorted(out)

    @property
    def checkpoints(self):
        return [p for _, p in self._existing()]

    @property
    def latest_checkpoint(self):
        ex = self._existing()
        return ex[-1][1] if ex else None

    def save(self):
        import os
        self._counter += 1
        path = os.path.join(self.directory, "ckpt-%d.pt" % self._counter)
        self.checkpoint.write(path)
        ex = self._existing()
        for _, p in ex[:max(0, len(ex) - self.max_to_keep)]:
            os.remove(p)
        return path
