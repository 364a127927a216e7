"""A/B of the fp32 engine's product method: native v_mfma_f32_16x16x4_f32
(`fp32`) vs split-bf16 MFMAs (`x3`), on the GEMM shapes of the benched models
and on the whole MobileNetV2 forward.  Interleaved rounds in one process
(median of R rounds); per shape also the error of each method against an fp64
oracle (max and mean of |err| / max(1, max|ref|)).

    python scripts/x3_ab.py [--rounds 5] [--model-batch 512]
"""
import argparse
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

SHAPES = [  # (label, M, K, N, act)
    ("mbv2 head b512 (pool)", 512 * 49, 320, 1280, -1),
    ("mbv2 7x7 960->320 b512", 512 * 49, 960, 320, 0),
    ("mbv2 classifier b512", 512, 1280, 1000, 0),
    ("posenet 65x65 64->128 b64", 64 * 65 * 65, 64, 128, 1),
    ("posenet 65x65 128->128 b64", 64 * 65 * 65, 128, 128, 1),
    ("posenet 33x33 128->256 b64", 64 * 33 * 33, 128, 256, 1),
    ("posenet 33x33 256->256 b64", 64 * 33 * 33, 256, 256, 1),
    ("posenet 17x17 256->512 b64", 64 * 17 * 17, 256, 512, 1),
    ("posenet 17x17 512->512 b64", 64 * 17 * 17, 512, 512, 1),
    ("posenet 17x17 512->1024 b64", 64 * 17 * 17, 512, 1024, 1),
    ("posenet 17x17 1024->1024 b64", 64 * 17 * 17, 1024, 1024, 1),
]


def timeit(fn, n=20):
    for _ in range(2):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(n):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / n * 1e3


def errs(y, ref):
    d = (y.double().cpu() - ref).abs()
    sc = max(1.0, ref.abs().max().item())
    return d.max().item() / sc, d.mean().item() / sc


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--model-batch", type=int, default=512)
    ap.add_argument("--skip-gemm", action="store_true")
    a = ap.parse_args()
    methods = ["fp32", "x3"]
    print(f"# fp32 product method A/B, {torch.cuda.get_device_name(0)}; median of {a.rounds} interleaved rounds")
    if not a.skip_gemm:
        print(f"{'shape':32s} {'M':>7s} {'K':>5s} {'N':>5s} | {'fp32 us':>8s} {'TF/s':>6s} | {'x3 us':>8s} {'TF/s':>6s} "
              f"| {'speedup':>7s} | {'fp32 max/mean err':>20s} | {'x3 max/mean err':>20s}")
        for label, M, K, N, act in SHAPES:
            torch.manual_seed(M + K + N)
            if act == -1:
                x = (torch.randn(M // 49, 7, 7, K, device="cuda") * 2).clamp(0, 6)
            else:
                x = (torch.randn(M, K, device="cuda") * 2).clamp(0, 6)
            npad, kpad = (N + 15) // 16 * 16, (K + 7) // 8 * 8
            wt = torch.zeros(npad, kpad, device="cuda")
            wt[:N, :K] = torch.randn(N, K, device="cuda") / K ** 0.5
            bias = torch.zeros(npad, device="cuda")
            bias[:N] = torch.randn(N, device="cuda") * 0.1
            if act == -1:
                fn = lambda: torch.ops.nnsx.pw_conv_pool(x, wt, bias, N, 1)  # noqa: E731
            else:
                fn = lambda: torch.ops.nnsx.pw_conv(x, wt, bias, None, N, act, True)  # noqa: E731
            t = {m: [] for m in methods}
            out = {}
            for _ in range(a.rounds):
                for m in methods:
                    torch.ops.nnsx.set_f32_math(m)
                    t[m].append(timeit(fn))
                    out[m] = fn()
            # fp64 oracle on a row subset (the whole product for the pooled head)
            if act == -1:
                ref = (x.double().cpu() @ wt[:N, :K].double().cpu().t() + bias[:N].double().cpu()).clamp(0, 6).mean((1, 2))
                ys = {m: out[m] for m in methods}
            else:
                rows = torch.arange(0, M, max(1, M // 2048))
                ref = x[rows].double().cpu() @ wt[:N, :K].double().cpu().t() + bias[:N].double().cpu()
                if act == 1:
                    ref = ref.clamp(0, 6)
                ys = {m: out[m][rows] for m in methods}
            e = {m: errs(ys[m], ref) for m in methods}
            med = {m: sorted(t[m])[len(t[m]) // 2] for m in methods}
            fl = 2.0 * M * K * N
            print(f"{label:32s} {M:7d} {K:5d} {N:5d} | {med['fp32']:8.1f} {fl / med['fp32'] / 1e6:6.1f} | "
                  f"{med['x3']:8.1f} {fl / med['x3'] / 1e6:6.1f} | {med['fp32'] / med['x3']:6.2f}x | "
                  f"{e['fp32'][0]:9.2e}/{e['fp32'][1]:9.2e} | {e['x3'][0]:9.2e}/{e['x3'][1]:9.2e}", flush=True)

    # whole model, batch B, one hipGraph per method (captured under that method)
    from nnstreamer_amd.models.fused import FusedMobileNetV2
    from nnstreamer_amd.models.mobilenet_v2 import mobilenet_v2

    B = a.model_batch
    m_ref = mobilenet_v2(seed=2).cuda().eval()
    f = torch.jit.script(FusedMobileNetV2.from_reference(mobilenet_v2(seed=2), "fp32").cuda().eval())
    g = torch.Generator().manual_seed(2)
    x = torch.randint(0, 256, (B, 224, 224, 3), generator=g, dtype=torch.uint8).cuda()
    with torch.no_grad():
        ref = m_ref(((x.float() - 127.5) / 127.5).permute(0, 3, 1, 2))
        # fp64 oracle on the host for the first 64 images
        m64 = mobilenet_v2(seed=2).double().eval()
        ref64 = m64(((x[:64].cpu().double() - 127.5) / 127.5).permute(0, 3, 1, 2))
    graphs, outs = {}, {}
    for meth in methods:
        torch.ops.nnsx.set_f32_math(meth)
        with torch.no_grad():
            for _ in range(2):
                f(x)
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr):
                outs[meth] = f(x)
        graphs[meth] = gr
    t = {m: [] for m in methods}
    for _ in range(a.rounds):
        for meth in methods:
            t[meth].append(timeit(graphs[meth].replay, n=20))
    print(f"\n# MobileNetV2 fused fp32 forward, batch {B}, one hipGraph per method")
    for meth in methods:
        o = outs[meth]
        med = sorted(t[meth])[len(t[meth]) // 2]
        top1 = (o.argmax(1) == ref.argmax(1)).float().mean().item()
        rel_t = ((o - ref).abs().max() / ref.abs().max()).item()
        o64 = o[:64].double().cpu()
        rel64 = ((o64 - ref64).abs().max() / ref64.abs().max()).item()
        mean64 = ((o64 - ref64).abs().mean() / ref64.abs().max()).item()
        print(f"{meth:5s} {med:8.1f} us/forward  {B / med * 1e6:9.0f} frames/s  top-1 vs torch fp32 {top1 * 100:6.2f} %  "
              f"max rel logit err vs torch fp32 {rel_t:.2e}  vs fp64 (64 images) max {rel64:.2e} mean {mean64:.2e}", flush=True)
    r64 = ref[:64].double().cpu()
    ref_t64 = ((r64 - ref64).abs().max() / ref64.abs().max()).item()
    print(f"torch fp32 (MIOpen) itself vs fp64: max rel logit err {ref_t64:.2e}")


if __name__ == "__main__":
    main()
