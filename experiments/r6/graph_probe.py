"""Per-launch device cost of back-to-back dependent small kernels: eager stream launches vs one
hipGraph replay (torch.cuda.CUDAGraph on ROCm), to see whether graphs would shorten L=64 steps."""
import time
import torch

x = torch.rand(64 ** 3 * 2, device="cuda")
N = 2000


def body():
    y = x
    for _ in range(N):
        y = y.mul_(1.0000001)  # dependent, ~1 us kernels
    return y


for _ in range(3):
    body()
torch.cuda.synchronize()
t0 = time.perf_counter()
body()
torch.cuda.synchronize()
eager = (time.perf_counter() - t0) / N * 1e6
s = torch.cuda.Stream()
s.wait_stream(torch.cuda.current_stream())
with torch.cuda.stream(s):
    body()
torch.cuda.current_stream().wait_stream(s)
g = torch.cuda.CUDAGraph()
with torch.cuda.graph(g):
    body()
g.replay()
torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(3):
    g.replay()
torch.cuda.synchronize()
graph = (time.perf_counter() - t0) / (3 * N) * 1e6
print(f"eager {eager:.2f} us/launch, graph replay {graph:.2f} us/launch")
