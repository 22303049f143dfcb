"""Per-shape table of every conv launch of one FCOS training step (configs[1]: 512x512, bs 16):
the launches are recorded during one eager step (ops_nn.conv_igemm / conv_wgrad /
conv_wgrad_grouped / conv_wgrad_batch -- a batched call is one row: the problems it launched
together, with their summed FLOPs), then each distinct launch is replayed alone with HIP events on
its stream.
Prints a markdown table (kernel chosen, us per launch, TFLOP/s, fraction of the 2.5 PF bf16 dense
peak, ms per step) sorted by time per step.
usage: conv_table.py [--bs 16] [--size 512] [--iters 10] [--out file.md]"""
import argparse
import collections
import ctypes
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite import _lib, ops_nn as nn  # noqa: E402
from cvlite.fcos_net import FCOSNet  # noqa: E402
from cvlite.train_fcos import FCOSTrainer, synthetic_batch  # noqa: E402

PEAK = 2500.0


def desc_key(kind, d):
    segs = tuple((d.seg[i].Hr, d.seg[i].Wr, d.seg[i].Hs, d.seg[i].Ws) for i in range(d.nseg))
    return (kind, d.mode, d.B, d.Cin, d.KH, d.KW, d.stride, d.Npad, d.n_store, d.dst_f32, d.relu_in, segs)


def describe(kind, d, ngroups=1):
    s0 = d.seg[0]
    mode = {0: "fwd", 1: "dgrad"}[d.mode] if kind == "igemm" else "wgrad"
    geo = "%dx%d" % (d.KH, d.KW) + (" s%d" % d.stride if d.stride > 1 else "")
    chans = "%d->%d" % (d.Cin, d.n_store)
    lv = "%dx%d" % (s0.Hr, s0.Wr) + (" +%d seg" % (d.nseg - 1) if d.nseg > 1 else "")
    g = " (%d groups)" % ngroups if ngroups > 1 else ""
    return "%s %s %s @ %s%s" % (mode, geo, chans, lv, g)


def flops(kind, d):
    """Algorithmic FLOPs: 2 x (forward output pixels) x KH*KW*Cin_fwd x Cout_fwd for all three
    passes.  A data-gradient descriptor's result map (Hr, Wr) is the forward INPUT and its source
    (Hs, Ws) the forward output (dY), so its rows are B*Hs*Ws -- for stride s the dX map has s^2 as
    many pixels, and counting those would over-state a strided dgrad's work s^2-fold."""
    dgrad = kind == "igemm" and d.mode == 1
    rows = sum(d.B * (d.seg[i].Hs * d.seg[i].Ws if dgrad else d.seg[i].Hr * d.seg[i].Wr) for i in range(d.nseg))
    K = d.KH * d.KW * d.Cin
    return 2.0 * rows * K * d.n_store


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--bs", type=int, default=16)
    ap.add_argument("--size", type=int, default=512)
    ap.add_argument("--iters", type=int, default=10)
    ap.add_argument("--out", default=None)
    ap.add_argument("--model", default="fcos", choices=["fcos", "retinanet", "centernet"])
    args = ap.parse_args()
    B, H = args.bs, args.size
    dev = torch.device("cuda")
    if args.model == "retinanet":              # configs[4]: 640, bs 8, C = 80
        from cvlite.retinanet import RetinaNet
        from cvlite.train_retinanet import RetinaTrainer, synthetic_coco_batch
        rn = RetinaNet(80, {}, anchor_sizes=[20.0, 40.0, 80.0, 160.0, 320.0])
        tr = RetinaTrainer(rn.model, rn, B, H, n_max=50, use_graph=False)
        tr.load_candidates(*synthetic_coco_batch(3 * B, H, 80, n_max=50, seed=4321, device=dev))
    elif args.model == "centernet":            # configs[3]: 512, bs 8, BN sub-batch 2
        from cvlite.hourglass_net import HourglassNet
        from cvlite.train_centernet import CenterNetTrainer, synthetic_batch as cn_batch
        net = HourglassNet(20, device=dev, seed=0)
        tr = CenterNetTrainer(net, B, (H, H), sub_batch_sz=2, n_max=16, use_graph=False)
        tr.load_batch(*cn_batch(B, H, H, 20, n_max=16, seed=777, device=dev))
    else:
        net = FCOSNet(20, device=dev, seed=0)
        tr = FCOSTrainer(net, B, (H, H), use_graph=False)
        tr.load_batch(*synthetic_batch(B, H, H, 20, seed=1234, device="cuda"))
    tr.step()                      # warm-up (allocations, first-touch)
    torch.cuda.synchronize()
    calls = collections.OrderedDict()
    counts = collections.Counter()
    orig = (nn.conv_igemm, nn.conv_wgrad, nn.conv_wgrad_grouped, nn.conv_wgrad_batch)

    def rec(key, replay, d, kind, ng=1):
        counts[key] += 1
        if key not in calls:
            calls[key] = (replay, d, kind, ng)

    def igemm(desc, src, dst, stats=None):
        rec(desc_key("igemm", desc), lambda: orig[0](desc, src, dst, stats), desc, "igemm")
        return orig[0](desc, src, dst, stats)

    def wgrad(desc, x, dy, dw, beta=0.0):
        rec(desc_key("wgrad", desc), lambda: orig[1](desc, x, dy, dw, beta), desc, "wgrad")
        return orig[1](desc, x, dy, dw, beta)

    def wgrad_g(desc, x, dy, dws, beta=0.0):
        rec(desc_key("wgrad_g", desc), lambda: orig[2](desc, x, dy, dws, beta), desc, "wgrad", len(dws))
        return orig[2](desc, x, dy, dws, beta)

    def wgrad_b(descs, xs, dys, dws, beta=0.0):
        key = ("wgrad_b",) + tuple(desc_key("wgrad", d) for d in descs)
        rec(key, lambda: orig[3](descs, xs, dys, dws, beta), list(descs), "wgrad_b", len(descs))
        return orig[3](descs, xs, dys, dws, beta)

    nn.conv_igemm, nn.conv_wgrad, nn.conv_wgrad_grouped, nn.conv_wgrad_batch = igemm, wgrad, wgrad_g, wgrad_b
    if args.model == "fcos":
        tr.load_batch(*synthetic_batch(B, H, H, 20, seed=77, device="cuda"))
    tr.step()
    torch.cuda.synchronize()
    nn.conv_igemm, nn.conv_wgrad, nn.conv_wgrad_grouped, nn.conv_wgrad_batch = orig
    lib = _lib.load()
    rows = []
    s = torch.cuda.current_stream()
    for key, (replay, d, kind, ng) in calls.items():
        replay()
        code = lib.cvl_conv_igemm_last_kernel()
        kname = lib.cvl_conv_kernel_name(code).decode().split(" (")[0]
        replay()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        for _ in range(args.iters):
            replay()
        e1.record(s)
        e1.synchronize()
        us = e0.elapsed_time(e1) / args.iters * 1e3
        n = counts[key]
        if kind == "wgrad_b":      # one batched call: its problems' summed FLOPs, shapes listed
            fl = sum(flops("wgrad", q) for q in d)
            shapes = collections.Counter(describe("wgrad", q)[6:] for q in d)
            label = "wgrad batch of %d: %s" % (ng, ", ".join("%s%s" % ("%dx " % c if c > 1 else "", sh)
                                                              for sh, c in shapes.items()))
            rows.append((us * n / 1e3, label, kname + " (batched)", n, us, fl / us / 1e6))
            continue
        fl = flops(kind, d)
        rows.append((us * n / 1e3, describe(kind, d, ng), kname, n, us, fl / us / 1e6))
    rows.sort(key=lambda r: -r[0])
    tot = sum(r[0] for r in rows)
    by_mode = collections.defaultdict(float)
    for r in rows:
        by_mode[r[1].split()[0]] += r[0]
    lines = ["# Conv launches of one %s step (bs %d, %dx%d), replayed alone" % (args.model, B, H, H), "",
             "Total %.3f ms per step over %d launches (%s)." % (
                 tot, sum(counts.values()), ", ".join("%s %.3f ms" % kv for kv in sorted(by_mode.items()))), "",
             "| ms/step | launch | kernel | per step | us/launch | TFLOP/s | frac of 2.5 PF |",
             "|---|---|---|---|---|---|---|"]
    for ms, desc, kname, n, us, tf in rows:
        lines.append("| %.3f | %s | %s | %d | %.1f | %.0f | %.3f |" % (ms, desc, kname, n, us, tf, tf / PEAK))
    text = "\n".join(lines) + "\n"
    print(text, flush=True)
    if args.out:
        with open(args.out, "w") as f:
            f.write(text)


if __name__ == "__main__":
    main()
