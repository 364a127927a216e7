#!/usr/bin/env python3
"""Config-4 ingest ceiling on one GPU: the rank-0 half of bench.py's
deeplab_fan (BASELINE.json config 4) without the DeepLab branches -- N
cameras (videotestsrc, 513 x 513 RGB, pinned frame rings) -> per-camera
tensor_converter device=0 (padded-row DMA + unpad) -> tensor_mux -> tensor_demux
-> N device-resident tensor_sink sync-device=true.  Reports frames/s and the
packed bytes per second that reach HBM, at each batch, over the steady state:
sink arrival stamps from the 4th batch to the last (pipeline start-up -- pinned
rings, pools, threads -- outside).  Reference elements:
gsttensor_converter.c:1062-1107 (stride strip), gsttensor_demux.c:469-556
(hand-out by reference, no copy).

    python scripts/fan_ingest.py [cameras] [batches...]     (default 8 cameras, batches 8 32)
"""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))


W = 4  # warm-up batches per camera outside the timed window


def run(nns, torch, cams, B, n, S=513):
    frame = S * S * 3
    pool = max(2 * B, min(n * B, -(-64 * 2**20 // frame)))  # 64 MiB ring per camera (512 MiB for 8)
    desc = ("".join(f"videotestsrc num-buffers={n * B} pattern=snow pool-size={pool} "
                    f"! video/x-raw,format=RGB,width={S},height={S},framerate=0/1 "
                    f"! tensor_converter frames-per-tensor={B} device=0 ! queue max-size-buffers=2 ! mux.sink_{r} "
                    for r in range(cams))
            + "tensor_mux name=mux sync-mode=nosync ! tensor_demux name=d "
            + " ".join(f"d.src_{r} ! queue max-size-buffers=2 ! tensor_sink name=s{r} sync-device=true"
                       for r in range(cams)))
    p = nns.parse_launch(desc)
    for r in range(cams):  # native arrival stamps (sync-device: the batch is in HBM when it arrives)
        p.get_by_name(f"s{r}").set_property("emit-signal", "false")
        p.get_by_name(f"s{r}").set_property("stats-every", "1")
    torch.cuda.synchronize()
    t = time.perf_counter()
    p.run(timeout=900)
    torch.cuda.synchronize()
    wall = time.perf_counter() - t
    arr = []
    for r in range(cams):
        st = p.get_by_name(f"s{r}").get_property("stats")
        arr.append([int(e.split(":")[0]) / 1e9 for e in st.split(",") if e])
    p.stop()
    # steady state: from the W-th batch's arrival (the earliest camera) to the last one (the latest);
    # the pipeline start (pinned rings, pools, threads) stays outside
    t0 = min(a[W - 1] for a in arr)
    t1 = max(a[-1] for a in arr)
    return t1 - t0, [len(a) for a in arr], frame, wall


def main():
    cams = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    batches = [int(x) for x in sys.argv[2:]] or [8, 32]
    import torch

    import nnstreamer_amd as nns

    print(f"# {cams} cameras 513x513 RGB -> tensor_converter device=0 -> tensor_mux -> tensor_demux -> "
          f"{cams} tensor_sink sync-device (1 x {torch.cuda.get_device_name(0)})")
    for B in batches:
        n = max(40, 1920 // B)  # batches per camera
        run(nns, torch, cams, B, W + 1)  # warm-up: code objects
        el, got, frame, wall = run(nns, torch, cams, B, n)
        frames = cams * (n - W) * B
        print(f"batch {B:3d}: {frames} frames in {el * 1e3:8.1f} ms  {frames / el:9.0f} frames/s  "
              f"{frames * frame / el / 1e9:6.2f} GB/s into HBM  (sink buffers per camera {sorted(set(got))}; "
              f"whole run incl. start-up {wall * 1e3:.0f} ms)", flush=True)


if __name__ == "__main__":
    main()
