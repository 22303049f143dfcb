"""Probe: do timing events recorded inside a captured HIP graph (external=True) give elapsed times?"""
import torch
a = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
b = torch.randn(4096, 4096, device="cuda", dtype=torch.bfloat16)
c = a @ b
evs = [(torch.cuda.Event(enable_timing=True, external=True), torch.cuda.Event(enable_timing=True, external=True))
       for _ in range(3)]
torch.cuda.synchronize()
g = torch.cuda.CUDAGraph()
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    g.capture_begin()
    for e0, e1 in evs:
        e0.record()
        torch.matmul(a, b, out=c)
        e1.record()
    g.capture_end()
torch.cuda.synchronize()
for it in range(3):
    g.replay()
    torch.cuda.synchronize()
    print("replay", it, [round(e0.elapsed_time(e1), 4) for e0, e1 in evs])
x0, x1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
x0.record()
for _ in range(10):
    torch.matmul(a, b, out=c)
x1.record()
torch.cuda.synchronize()
print("eager avg", x0.elapsed_time(x1) / 10)
