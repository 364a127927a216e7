#!/usr/bin/env python3
"""Padded-frame upload micro-bench (round-3 verdict item 2): videotestsrc
(pinned ring of pre-rendered RGB frames whose rows are padded to 4 bytes, as
GStreamer lays out 513- and 257-wide RGB) -> tensor_converter
frames-per-tensor=B device=0 -> tensor_sink sync-device.  Reports the packed
bytes per second that reach HBM (a queue before the sink: the sink's device
sync does not stall the converter).

    python scripts/upload_bench.py [width] [batch] [batches]
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


def main():
    w = int(sys.argv[1]) if len(sys.argv) > 1 else 513
    B = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 200
    import torch

    import nnstreamer_amd as nns

    frame = w * w * 3
    pool = max(2 * B, -(-512 * 2**20 // frame))  # 512 MiB ring: larger than the last-level cache
    host = os.environ.get("UPLOAD_BENCH_HOST") == "1"  # reference: the same pipeline without the upload
    dev = "" if host else " device=0"
    for rep in range(2):  # first pass warms the pools / code objects
        desc = (f"videotestsrc num-buffers={n * B} pattern=snow pool-size={min(pool, n * B)} "
                f"! video/x-raw,format=RGB,width={w},height={w},framerate=0/1 "
                f"! tensor_converter frames-per-tensor={B}{dev} ! queue max-size-buffers=4 "
                f"! tensor_sink name=sink sync-device=true")
        p = nns.parse_launch(desc)
        torch.cuda.synchronize()
        t = time.perf_counter()
        p.run(timeout=600)
        torch.cuda.synchronize()
        el = time.perf_counter() - t
        p.stop()
    mode = "padded DMA + unpad_rows"
    if host:
        mode = "host only, no upload"
    print(f"width {w} batch {B} ({mode}): {n} batches in {el * 1e3:.1f} ms, {el / n * 1e6:.1f} us per batch, "
          f"{n * B * frame / el / 1e9:.2f} GB/s packed frames to HBM")


if __name__ == "__main__":
    main()
