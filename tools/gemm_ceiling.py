"""What hipBLASLt (torch.matmul, bf16) reaches on the tower conv's GEMM shape (im2col'd: M=87,296,
N=256, K=2,304) and neighbours -- the practical ceiling our implicit-GEMM conv is compared with."""
import torch


def t(fn, iters=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        fn()
    e1.record()
    e1.synchronize()
    return e0.elapsed_time(e1) / iters


for (M, N, K) in [(8192, 8192, 8192), (87296, 256, 2304), (87296, 512, 2304), (87296, 2304, 256),
                  (2304, 256, 87296), (65536, 256, 2304), (262144, 64, 576)]:
    a = torch.randn(M, K, device="cuda").to(torch.bfloat16)
    b = torch.randn(K, N, device="cuda").to(torch.bfloat16)
    ms = t(lambda: a @ b)
    print("M %6d N %5d K %6d: %.3f ms  %.0f TF/s" % (M, N, K, ms, 2.0 * M * N * K / ms / 1e9), flush=True)
