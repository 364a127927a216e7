#!/usr/bin/env python3
"""BASELINE.json config 1: the CPU plumbing pipeline, no GPU --

    videotestsrc ! tensor_converter ! tensor_transform mode=arithmetic ! (sink)

frames/s over the timed frames and p50 / p99 per-frame latency (source PTS ->
sink arrival, live source) on the host.  Prints one JSON line.

    python scripts/bench_plumbing.py [--size 224] [--frames 20000] [--warmup 500] [--live-fps 0]
"""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def run(nns, size, frames, warmup, live_fps, fpt):
    live = "is-live=true " if live_fps > 0 else ""
    desc = (f"videotestsrc num-buffers={frames} pattern=snow pool-size=64 {live}"
            f"! video/x-raw,format=RGB,width={size},height={size},framerate={live_fps}/1 "
            f"! tensor_converter frames-per-tensor={fpt} "
            f"! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 "
            f"! tensor_sink name=sink")
    p = nns.parse_launch(desc)
    sink = p.get_by_name("sink")
    sink.set_property("emit-signal", "false")
    sink.set_property("stats-every", "1")
    t0 = time.perf_counter()
    p.run(timeout=3600)
    wall = time.perf_counter() - t0
    recs = [tuple(int(v) for v in e.split(":")) for e in sink.get_property("stats").split(",") if e]
    p.stop()
    arr = [t / 1e9 for t, _ in recs]
    lat = sorted(l / 1e6 for _, l in recs[warmup:] if l >= 0)
    n = len(arr) - warmup
    fps = (n - 1) * fpt / (arr[-1] - arr[warmup]) if n > 1 else 0.0
    pct = (lambda q: lat[min(len(lat) - 1, int(q * len(lat)))] if lat else 0.0)
    return dict(desc=desc, frames_per_s=round(fps, 1), p50_latency_ms=round(pct(0.5), 4),
                p99_latency_ms=round(pct(0.99), 4), wall_s=round(wall, 3), buffers=len(arr))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--size", type=int, default=224)
    ap.add_argument("--frames", type=int, default=20000)
    ap.add_argument("--warmup", type=int, default=500)
    ap.add_argument("--live-fps", type=int, default=0)
    a = ap.parse_args()
    import nnstreamer_amd as nns

    thr = run(nns, a.size, a.frames, a.warmup, 0, 1)
    lat = run(nns, a.size, min(a.frames, 3000), min(a.warmup, 200), a.live_fps or 500, 1)
    print(json.dumps({
        "metric": "frames/sec + p50 per-frame latency, videotestsrc ! tensor_converter ! tensor_transform "
                  "arithmetic ! sink (CPU plumbing, no GPU)",
        "value": thr["frames_per_s"], "unit": "frames/s", "n_gpus": 0, "higher_is_better": True,
        "p50_latency_ms": lat["p50_latency_ms"], "p99_latency_ms": lat["p99_latency_ms"],
        "latency_source": f"live source at {a.live_fps or 500} frames/s",
        "free_running_p50_latency_ms": thr["p50_latency_ms"], "cpus": os.cpu_count(),
        "data": "synthetic video frames (videotestsrc pattern=snow)",
        "config": {"frame": f"{a.size}x{a.size} RGB", "pipeline": thr["desc"]}}))


if __name__ == "__main__":
    main()
