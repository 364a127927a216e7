#!/usr/bin/env python3
"""Headline benchmark: end-to-end frames/sec + p50 per-frame latency of the
MobileNetV2 224x224 image-classification pipeline (BASELINE.json config 2),
one pipeline per GPU (weak scaling: per-GPU work fixed as N grows).

    python bench.py --gpus N --steps K --warmup W

Pipeline (one per rank, pinned to GPU LOCAL_RANK):

  videotestsrc pattern=snow ! video/x-raw,format=RGB,width=224,height=224
    ! tensor_converter frames-per-tensor=B device=<gpu>     # H2D into HBM, B frames per tensor
    ! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5   # HIP kernel
    ! tensor_filter framework=pytorch model=mbv2.pt accelerator=true:gpu custom=hipgraph:true
    ! tensor_decoder mode=image_labeling option1=labels.txt # HIP argmax, labels D2H
    ! tensor_sink

A "step" is one batch of B frames reaching the sink.  W batches warm up
(graph capture, allocator), then the wall time of exactly K batches is
measured at the sink; ranks are bracketed by barrier + device synchronize,
the max over ranks is reported.  Latency = sink arrival - frame capture time
(the PTS of the oldest frame in the batch).  Data: synthetic video frames,
random-init weights.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse_args():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("NNSX_BENCH_BATCH", "128")))
    ap.add_argument("--model", default=os.environ.get("NNSX_BENCH_MODEL", "mobilenet_v2_fused"),
                    help="mobilenet_v2 (plain torch) | mobilenet_v2_fused (nnsx CDNA4 kernels)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--cpu", action="store_true", help="CPU reference path (device=-1, torch CPU)")
    ap.add_argument("--queue", type=int, default=4, help="queue depth between filter and decoder")
    return ap.parse_args()


def main():
    a = parse_args()
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist

        backend = "nccl" if (torch.cuda.is_available() and not a.cpu) else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend=backend)

    import nnstreamer_amd as nns
    from nnstreamer_amd.models.export import export, write_labels

    use_gpu = (not a.cpu) and torch.cuda.is_available() and nns.gpu_count() > 0
    dev = local_rank if use_gpu else -1
    workdir = os.path.join(tempfile.gettempdir(), f"nnsx_bench_{os.getuid()}_{rank}")
    os.makedirs(workdir, exist_ok=True)
    model_path = os.path.join(workdir, f"{a.model}.pt")
    layout = "nhwc"
    export(a.model, model_path, layout=layout)
    labels = write_labels(os.path.join(workdir, "labels.txt"))

    B = a.batch
    total = a.warmup + a.steps
    frames = total * B
    graph = "true" if (use_gpu and not a.no_graph) else "false"
    accel = "true:gpu" if use_gpu else "false"
    desc = (
        f"videotestsrc num-buffers={frames} pattern=snow pool-size=16 "
        f"! video/x-raw,format=RGB,width=224,height=224,framerate=0/1 "
        f"! tensor_converter frames-per-tensor={B} device={dev} "
        f"! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 "
        f"! tensor_filter framework=pytorch model={model_path} input=3:224:224:{B} inputtype=float32 "
        f"accelerator={accel} device={dev} custom=hipgraph:{graph} "
        f"! queue max-size-buffers={a.queue} "
        f"! tensor_decoder mode=image_labeling option1={labels} "
        f"! tensor_sink name=sink"
    )
    pipe = nns.parse_launch(desc)
    sink = pipe.get_by_name("sink")
    arrivals = []
    latencies = []

    def on_data(buf):
        now = pipe.running_time()
        arrivals.append(time.perf_counter())
        if buf.pts >= 0:
            latencies.append((now - buf.pts) / 1e6)

    sink.connect("new-data", on_data)

    if dist is not None:
        dist.barrier()
    if use_gpu:
        torch.cuda.synchronize()
    t_start = time.perf_counter()
    pipe.run(timeout=3600)
    if use_gpu:
        torch.cuda.synchronize()
    t_end = time.perf_counter()
    if dist is not None:
        dist.barrier()
    pipe.stop()

    n = len(arrivals)
    if n < total:
        raise SystemExit(f"rank {rank}: only {n}/{total} batches reached the sink")
    # timed region: exactly K steps after W warmup steps
    t0 = arrivals[a.warmup - 1] if a.warmup > 0 else t_start
    t1 = arrivals[a.warmup + a.steps - 1]
    elapsed = t1 - t0
    lat = np.array(latencies[a.warmup:a.warmup + a.steps]) if latencies else np.array([0.0])
    stats = torch.tensor([elapsed, float(np.percentile(lat, 50)), float(np.percentile(lat, 99))], dtype=torch.float64)
    if dist is not None:
        if dist.get_backend() == "nccl":
            stats = stats.cuda()
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        stats = stats.cpu()
    elapsed, p50, p99 = stats.tolist()
    ms_per_step = elapsed / a.steps * 1e3
    fps_total = world * a.steps * B / elapsed
    if rank == 0:
        out = {
            "metric": "end-to-end frames/sec + p50 per-frame latency, MobileNetV2 224x224 pipeline",
            "value": round(fps_total, 2),
            "unit": "frames/s",
            "n_gpus": world if use_gpu else 0,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "bf16" if "fused" in a.model else "fp32",
            "data": "synthetic video frames (videotestsrc pattern=snow), random-init weights",
            "p50_latency_ms": round(p50, 3),
            "p99_latency_ms": round(p99, 3),
            "frames_per_step_per_gpu": B,
            "wall_s": round(t_end - t_start, 3),
            "config": {
                "model": "MobileNetV2 224x224 (tensor_filter + image_labeling decoder)",
                "global_batch": B * world,
                "seq_len": 1,
                "parallelism": f"branch-dp{world}",
                "pipeline": desc,
            },
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
