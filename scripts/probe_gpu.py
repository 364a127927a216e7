"""One-off GPU probe: HIP runtime mix check + PyTorch/MIOpen MobileNetV2 timings."""
import ctypes
import os
import sys
import time

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from nnstreamer_amd.models.mobilenet_v2 import mobilenet_v2  # noqa: E402

print("torch", torch.__version__, "hip", torch.version.hip, "dev", torch.cuda.get_device_name(0), flush=True)
lib = ctypes.CDLL(os.path.join(os.path.dirname(os.path.abspath(__file__)), "probe_kernel.so"))
x = torch.zeros(1000, device="cuda")
rc = lib.probe_add_one(ctypes.c_void_p(x.data_ptr()), 1000, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
torch.cuda.synchronize()
print("probe kernel rc", rc, "sum", x.sum().item(), flush=True)


def bench(fn, iters=50, warm=10):
    for _ in range(warm):
        fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / iters * 1e3


m = mobilenet_v2().cuda()
for dtype in (torch.float32, torch.bfloat16):
    for cl in (False, True):
        mm = m.to(dtype)
        if cl:
            mm = mm.to(memory_format=torch.channels_last)
        for bs in (1, 32, 128):
            inp = torch.randn(bs, 3, 224, 224, device="cuda", dtype=dtype)
            if cl:
                inp = inp.contiguous(memory_format=torch.channels_last)
            with torch.no_grad():
                ms = bench(lambda: mm(inp))
                g = torch.cuda.CUDAGraph()
                s = torch.cuda.Stream()
                s.wait_stream(torch.cuda.current_stream())
                with torch.cuda.stream(s):
                    for _ in range(3):
                        mm(inp)
                torch.cuda.current_stream().wait_stream(s)
                with torch.cuda.graph(g):
                    out = mm(inp)
                gms = bench(lambda: g.replay())
            print(f"mbv2 {str(dtype):15s} cl={cl} bs={bs:4d} eager {ms:8.3f} ms ({bs/ms*1e3:9.0f} img/s)  graph {gms:8.3f} ms ({bs/gms*1e3:9.0f} img/s)", flush=True)
