"""Do hipGraph replays run independent branches concurrently?  Two spin
kernels (torch.cuda._sleep, one workgroup each) on two streams: eager and
captured, timed against the same two spins on one stream."""
import time
import torch

def run(fn, n=20):
    fn(); torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / n * 1e3

CYC = 1 << 22
main = torch.cuda.current_stream()
side = torch.cuda.Stream()

def serial():
    torch.cuda._sleep(CYC); torch.cuda._sleep(CYC)

def forked():
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        torch.cuda._sleep(CYC)
    torch.cuda._sleep(CYC)
    torch.cuda.current_stream().wait_stream(side)

print("eager serial ms", run(serial))
print("eager forked ms", run(forked))
for name, f in (("serial", serial), ("forked", forked)):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        f()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        f()
    print("graph", name, "ms", run(g.replay))

# real GEMM-sized work: two bf16 matmuls that each fill ~half the chip
a = torch.randn(8192, 512, device="cuda", dtype=torch.bfloat16)
b = torch.randn(512, 512, device="cuda", dtype=torch.bfloat16)
c = torch.randn(512, 8192, device="cuda", dtype=torch.bfloat16)
d = torch.randn(8192, 512, device="cuda", dtype=torch.bfloat16)
def mm_serial():
    for _ in range(4):
        a @ b; c @ d
def mm_forked():
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(4):
            c @ d
    for _ in range(4):
        a @ b
    torch.cuda.current_stream().wait_stream(side)
print("eager mm serial ms", run(mm_serial))
print("eager mm forked ms", run(mm_forked))
for name, f in (("serial", mm_serial), ("forked", mm_forked)):
    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        f()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        f()
    print("graph mm", name, "ms", run(g.replay))
