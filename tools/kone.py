"""Run one conv launch shape repeatedly (for rocprofv3 --pmc / kernel-trace of a single kernel).
usage: kone.py <fwd|dgrad|wgrad> B H W Cin Cout k stride [iters]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "cv-lite-object-detection_amd")]
import torch  # noqa: E402

from cvlite.layers import Conv, ParamStore  # noqa: E402

BF = torch.bfloat16


def main():
    mode = sys.argv[1]
    B, H, W, cin, cout, k, s = (int(v) for v in sys.argv[2:9])
    iters = int(sys.argv[9]) if len(sys.argv) > 9 else 20
    st = ParamStore()
    c = Conv(st, "c", k, cin, cout, stride=s)
    st.finalize("cuda", 0)
    c.pack()
    Ho, Wo, _, _ = c.out_hw(H, W)
    x = torch.randn((B, H, W, cin), device="cuda").to(BF)
    dy = torch.randn((B, Ho, Wo, cout), device="cuda").to(BF)
    out = torch.empty((B, Ho, Wo, cout), dtype=BF, device="cuda")
    dx = torch.empty((B, H, W, cin), dtype=BF, device="cuda")
    fn = {"fwd": lambda: c.fwd(x, B, H, W, out=out),
          "dgrad": lambda: c.dgrad(dy, B, H, W, out=dx),
          "wgrad": lambda: c.wgrad(x, dy, B, H, W, bias=False)}[mode]
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    print("done", mode, B, H, W, cin, cout, k, s)


if __name__ == "__main__":
    main()
