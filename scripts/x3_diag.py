import os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
import nnstreamer_amd  # noqa
torch.ops.nnsx.set_f32_math("x3")
M, K, N = 256, 32, 64
torch.manual_seed(0)
x = torch.randn(M, K, device="cuda")
wt = torch.randn(N, K, device="cuda")
b = torch.zeros(N, device="cuda")
torch.ops.nnsx.x3_weight_cache(False)
y0 = torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, None, N, 0, 64064)
torch.ops.nnsx.x3_weight_cache(True)
y1 = torch.ops.nnsx.pw_conv_f32_tile(x, wt, b, None, N, 0, 64064)
d = (y1 - y0).abs() > 1e-4
print("bad", d.sum().item(), "of", d.numel())
rows = d.any(1).nonzero().flatten().tolist(); cols = d.any(0).nonzero().flatten().tolist()
print("rows", rows[:80]); print("cols", cols)
# probe with one-hot weights: which weight element lands where
for part_test in range(3):
    pass
wt2 = torch.zeros(N, K, device="cuda"); wt2[5, 3] = 1.0
x2 = torch.zeros(M, K, device="cuda"); x2[:, 3] = 1.0
y2 = torch.ops.nnsx.pw_conv_f32_tile(x2, wt2, b, None, N, 0, 64064)
print("one-hot w[5,3]: nonzero cols", (y2.abs() > 0).any(0).nonzero().flatten().tolist(), "rows", (y2.abs() > 0).any(1).sum().item())
for n in [0, 1, 16, 17, 31, 32, 63]:
    for k in [0, 7, 8, 15, 16, 31]:
        w3 = torch.zeros(N, K, device="cuda"); w3[n, k] = 1.0
        x3 = torch.zeros(M, K, device="cuda"); x3[:, k] = 1.0
        y3 = torch.ops.nnsx.pw_conv_f32_tile(x3, w3, b, None, N, 0, 64064)
        nz = (y3.abs() > 0).any(0).nonzero().flatten().tolist()
        if nz != [n]:
            print(f"w[{n},{k}] -> cols {nz}")
