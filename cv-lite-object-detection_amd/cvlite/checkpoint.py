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


def _bns(net):
    bb = getattr(net, "backbone", None)
    return list(bb.bns()) if bb is not None and hasattr(bb, "bns") else []


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
