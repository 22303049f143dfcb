"""Do two independent conv launches overlap (a) eagerly on two HIP streams and (b) as parallel
branches of one captured HIP graph (fork/join via events)?  Pairs a backbone-layer dgrad with its
wgrad (independent: both read dz) at bs 16, the shapes whose single launch leaves most CUs idle.
usage: overlap_probe.py [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite.layers import Conv, ParamStore  # noqa: E402

BF = torch.bfloat16


def timed(fn, iters):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters * 1e3


def probe(B, H, W, cin, cout, k, iters):
    st = ParamStore()
    c = Conv(st, "c", k, cin, cout)
    st.finalize("cuda", 0)
    c.pack()
    x = torch.randn((B, H, W, cin), device="cuda").to(BF)
    dz = torch.randn((B, H, W, cout), device="cuda").to(BF)
    dx = torch.empty((B, H, W, cin), dtype=BF, device="cuda")
    side = torch.cuda.Stream()

    def dgrad():
        c.dgrad(dz, B, H, W, out=dx)

    def wgrad():
        c.wgrad(x, dz, B, H, W, bias=False)

    def serial():
        dgrad()
        wgrad()

    def forked():
        main = torch.cuda.current_stream()
        side.wait_stream(main)
        dgrad()
        with torch.cuda.stream(side):
            wgrad()
        main.wait_stream(side)

    t_d, t_w, t_s, t_f = timed(dgrad, iters), timed(wgrad, iters), timed(serial, iters), timed(forked, iters)
    graphs = {}
    for name, fn in (("serial", serial), ("forked", forked)):
        cap = torch.cuda.Stream()
        cap.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(cap):
            fn()
            torch.cuda.synchronize()
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=cap):
                for _ in range(8):
                    fn()
        torch.cuda.current_stream().wait_stream(cap)
        graphs[name] = timed(g.replay, max(1, iters // 8)) / 8
    print("%dx%dx%d %d->%d k%d: dgrad %.1f us, wgrad %.1f us, sum %.1f | eager serial %.1f, eager 2-stream %.1f | "
          "graph serial %.1f, graph forked %.1f" % (B, H, W, cin, cout, k, t_d, t_w, t_d + t_w, t_s, t_f,
                                                     graphs["serial"], graphs["forked"]), flush=True)


def main():
    iters = int(sys.argv[1]) if len(sys.argv) > 1 else 40
    probe(16, 32, 32, 256, 256, 3, iters)
    probe(16, 16, 16, 512, 512, 3, iters)
    probe(16, 64, 64, 128, 128, 3, iters)
    probe(16, 32, 32, 1024, 256, 1, iters)


if __name__ == "__main__":
    main()
