"""Do parallel branches of a captured hipGraph run concurrently on ROCm?  Two side streams each
run a single-wave spin kernel (torch.cuda._sleep); concurrent execution replays in ~1x the spin
time, serialized execution in ~2x. Also checks eager multi-stream and a 4-branch graph."""
import time
import torch

CYC = 2_000_000   # ~1 ms at 2 GHz


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def branches(k):
    ss = [torch.cuda.Stream() for _ in range(k)]
    def run():
        main = torch.cuda.current_stream()
        for s in ss:
            s.wait_stream(main)
            with torch.cuda.stream(s):
                torch.cuda._sleep(CYC)
        for s in ss:
            main.wait_stream(s)
    return run


one = timed(lambda: torch.cuda._sleep(CYC))
print(f"single spin: {one:.3f} ms")
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    torch.cuda._sleep(CYC)
    torch.cuda._sleep(CYC)
print(f"graph 2 serial spins: {timed(g.replay):.3f} ms")
for k in (2, 4):
    run = branches(k)
    print(f"eager {k} streams: {timed(run):.3f} ms")
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        run()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        run()
    print(f"graph {k} branches: {timed(g.replay):.3f} ms")
