"""Per-kernel cost of dependent launches inside a hipGraph (no profiler): N tiny kernels
captured back to back, replayed; prints us per kernel for a few kernel shapes."""
import time
import torch

def bench(fn, n=200, reps=20):
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            for _ in range(n):
                fn()
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps / n * 1e6

a = torch.zeros(16, device="cuda")
b = torch.zeros(1 << 20, device="cuda")
c = torch.zeros(8 << 20, device="cuda")
print("fill 16 floats      : %.2f us/kernel" % bench(lambda: a.fill_(1.0)))
print("fill 1M floats (4MB): %.2f us/kernel" % bench(lambda: b.fill_(1.0)))
print("add_ 1M floats      : %.2f us/kernel" % bench(lambda: b.add_(1.0)))
print("fill 8M floats(32MB): %.2f us/kernel" % bench(lambda: c.fill_(1.0)))
