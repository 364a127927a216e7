"""CPU cost of HIP kernel launches: eager torch ops vs a replayed hipGraph of
the same ops (used to size how many launches a pipeline step can afford)."""
import time

import torch

x = torch.zeros(1024, device="cuda")
N = 100


def body():
    for _ in range(N):
        x.add_(1)


for _ in range(3):
    body()
torch.cuda.synchronize()
t = time.perf_counter()
for _ in range(20):
    body()
t_eager = (time.perf_counter() - t) / (20 * N) * 1e6
torch.cuda.synchronize()
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
t = time.perf_counter()
for _ in range(20):
    g.replay()
t_launch = (time.perf_counter() - t) / 20 * 1e6
torch.cuda.synchronize()
t_all = (time.perf_counter() - t) / 20 * 1e6
print(f"eager launch {t_eager:.1f} us/op; graph replay CPU {t_launch:.1f} us per {N}-node graph "
      f"({t_launch / N:.1f} us/node), incl. execution {t_all:.1f} us")
