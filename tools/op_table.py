"""Per-shape table of every NON-conv launch of one FCOS training step (configs[1]: 512x512, bs 16):
BN, pooling, up-sampling, ReLU/add, bias-grad, targets, loss, optimizer.  The calls are recorded
during one eager step (every public function of ops_nn / ops_targets except the conv entry points),
then each distinct call is replayed alone with HIP events on its stream.

Bytes per call = the sum of nbytes of the call's tensor arguments of >= 64 KiB (each operand read
or written once: the algorithmic traffic of these one-pass kernels; small per-channel vectors and
workspaces ignored).  GB/s = those bytes / the measured launch time, against the 8 TB/s HBM peak
(MI355X_MICROARCH.md).  Prints a markdown table sorted by time per step.
usage: op_table.py [--bs 16] [--size 512] [--iters 10] [--out file.md]"""
import argparse
import collections
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite import ops_nn as nn, ops_targets as ot  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402
from cvlite.train_fcos import FCOSTrainer, synthetic_batch  # noqa: E402

PEAK_GBS = 8000.0
SKIP = {"seg", "make_desc", "conv_igemm", "conv_wgrad", "conv_wgrad_grouped", "desc_ptr"}
MIN_BYTES = 64 * 1024


def big_tensors(args, kwargs):
    out = []
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, torch.Tensor) and a.is_cuda and a.numel() * a.element_size() >= MIN_BYTES:
            out.append(a)
    return out


def shape_key(name, args, kwargs):
    parts = [name]
    for a in list(args) + list(kwargs.values()):
        if isinstance(a, torch.Tensor):
            parts.append(("T", tuple(a.shape), str(a.dtype)))
        elif isinstance(a, (int, float, bool, str, type(None))):
            parts.append(a)
        else:
            parts.append(type(a).__name__)
    return tuple(parts)


def describe(name, args, kwargs):
    ts = big_tensors(args, kwargs)
    shp = "x".join(str(s) for s in ts[0].shape) if ts else "-"
    return "%s %s" % (name, shp)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bs", type=int, default=16)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    args = ap.parse_args()
    B, H = args.bs, args.size
    net = FCOSNet(20, device=torch.device("cuda"), seed=0)
    tr = FCOSTrainer(net, B, (H, H), use_graph=False)
    tr.load_batch(*synthetic_batch(B, H, H, 20, seed=1234, device="cuda"))
    tr.step()
    torch.cuda.synchronize()
    calls = collections.OrderedDict()
    counts = collections.Counter()
    saved = []
    for mod in (nn, ot):
        for name in dir(mod):
            fn = getattr(mod, name)
            if name.startswith("_") or name in SKIP or not callable(fn) or getattr(fn, "__module__", "") != mod.__name__:
                continue
            if isinstance(fn, type):
                continue

            def wrap(*a, _fn=fn, _name=name, **k):
                key = shape_key(_name, a, k)
                counts[key] += 1
                if key not in calls:
                    calls[key] = (lambda: _fn(*a, **k), describe(_name, a, k),
                                  sum(t.numel() * t.element_size() for t in big_tensors(a, k)))
                return _fn(*a, **k)
            saved.append((mod, name, fn))
            setattr(mod, name, wrap)
    tr.load_batch(*synthetic_batch(B, H, H, 20, seed=77, device="cuda"))
    tr.step()
    torch.cuda.synchronize()
    for mod, name, fn in saved:
        setattr(mod, name, fn)
    rows = []
    s = torch.cuda.current_stream()
    for key, (replay, desc, nbytes) in calls.items():
        try:
            replay()
        except Exception as e:            # host-side helpers (no launch) or non-replayable calls
            print("skip", desc, type(e).__name__, e, file=sys.stderr)
            continue
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.iters):
            replay()
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) / args.iters * 1e3
        n = counts[key]
        gbs = nbytes / us / 1e3 if us > 0 else 0.0
        rows.append((us * n / 1e3, desc, n, us, nbytes / 1e6, gbs))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    by = collections.defaultdict(float)
    for r in rows:
        by[r[1].split()[0]] += r[0]
    lines = ["# Non-conv launches of one FCOS step (bs %d, %dx%d), replayed alone" % (B, H, H), "",
             "Total %.3f ms per step over %d calls.  By op: %s." % (
                 tot, sum(counts.values()),
                 ", ".join("%s %.3f" % kv for kv in sorted(by.items(), key=lambda kv: -kv[1]))), "",
             "Bytes = tensor operands >= 64 KiB, each once (algorithmic); frac = GB/s / 8000.", "",
             "| ms/step | call (first big operand) | per step | us/call | MB/call | GB/s | frac of 8 TB/s |",
             "|---|---|---|---|---|---|---|"]
    for ms, desc, n, us, mb, gbs in rows:
        lines.append("| %.3f | %s | %d | %.1f | %.1f | %.0f | %.3f |" % (ms, desc, n, us, mb, gbs, gbs / PEAK_GBS))
    text = "\n".join(lines) + "\n"
    print(text, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
