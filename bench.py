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
    ap.add_argument("--no-fuse-norm", action="store_true",
                    help="keep the normalisation as a separate tensor_transform element")
    ap.add_argument("--cpu", action="store_true", help="CPU reference path (device=-1, torch CPU)")
    ap.add_argument("--queue", type=int, default=4, help="queue depth between filter and decoder")
    ap.add_argument("--comm-backend", default="auto", choices=["auto", "rccl", "tcp"],
                    help="posenet_multi: tensor_allgather data plane")
    ap.add_argument("--config", default=os.environ.get("NNSX_BENCH_CONFIG", "mbv2"),
                    choices=sorted(CONFIGS), help="BASELINE.json config (default: the headline MobileNetV2 pipeline)")
    return ap.parse_args()


# best CPU reference path for the MobileNetV2 pipeline
# (identical pipeline, host elements + fp32 PyTorch CPU, 8 vCPU).
CPU_BASELINE_FPS = 254.1

# BASELINE.json configs that run on one GPU per rank.  Each: input size, model,
# normalisation, decoder string and whether the decoder emits one buffer per frame.
CONFIGS = {
    "mbv2": dict(size=224, model="mobilenet_v2_fused", norm="typecast:float32,add:-127.5,div:127.5",
                 decoder="tensor_decoder mode=image_labeling option1={labels}", per_frame=False,
                 metric="end-to-end frames/sec + p50 per-frame latency, MobileNetV2 224x224 pipeline",
                 desc="MobileNetV2 224x224 (tensor_filter + image_labeling decoder)"),
    "ssd": dict(size=300, model="ssd_fused", norm="typecast:float32,add:-127.5,div:127.5",
                decoder="tensor_decoder mode=bounding_boxes option1=mobilenet-ssd option2={coco} option3={priors} "
                        "option4=300:300 option5=300:300", per_frame=True,
                metric="end-to-end frames/sec + p50 per-frame latency, SSD-MobileNet 300x300 + bounding_boxes + HIP NMS",
                desc="SSDLite-MobileNetV2 300x300 (tensor_filter + bounding_boxes decoder, HIP NMS)"),
    "deeplab": dict(size=513, model="deeplab_fused", norm="typecast:float32,div:255.0",
                    decoder="tensor_decoder mode=image_segment option1=tflite-deeplab", per_frame=True,
                    metric="end-to-end frames/sec + p50 per-frame latency, DeepLabV3 513x513 segmentation pipeline",
                    desc="DeepLabV3-MobileNetV2 513x513 (tensor_filter + image_segment decoder)"),
    # BASELINE.json config 4: one camera rank fans its batches out to the other ranks
    # (edgesink connect-type=RCCL rccl-mode=scatter -> ncclSend/ncclRecv over xGMI);
    # every other rank runs DeepLabV3 + image_segment on what it receives
    "deeplab_fan": dict(size=513, model="deeplab_fused", norm="typecast:float32,div:255.0",
                        decoder="tensor_decoder mode=image_segment option1=tflite-deeplab", per_frame=True, fan=True,
                        metric="end-to-end frames/sec, DeepLabV3 513x513 segmentation, branches fanned over RCCL",
                        desc="DeepLabV3-MobileNetV2 513x513 on N-1 ranks fed by a camera rank (RCCL scatter)"),
    # BASELINE.json config 5: PoseNet multi-source, outputs all-gathered across ranks
    "posenet_multi": dict(size=257, model="posenet_fused", norm="typecast:float32,add:-127.5,div:127.5",
                          decoder="tensor_decoder mode=pose_estimation option1=640:480 option2=257:257 "
                                  "option3={pose} option4=heatmap-offset", per_frame=True, gather=True,
                          metric="end-to-end frames/sec + p50 per-frame latency, PoseNet multi-source "
                                 "pipeline with RCCL all-gather",
                          desc="PoseNet-MobileNetV1 257x257 per rank + tensor_allgather of the pose tensors"),
    "posenet": dict(size=257, model="posenet_fused", norm="typecast:float32,add:-127.5,div:127.5",
                    decoder="tensor_decoder mode=pose_estimation option1=640:480 option2=257:257 option3={pose} "
                            "option4=heatmap-offset", per_frame=True,
                    metric="end-to-end frames/sec + p50 per-frame latency, PoseNet 257x257 pipeline",
                    desc="PoseNet-MobileNetV1 257x257 (tensor_filter + pose_estimation decoder)"),
}


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
    numa = "off"
    if use_gpu and os.environ.get("NNSX_BENCH_NUMA", "1") != "0":
        # each rank's streaming threads and its pinned frame ring on the GPU's own
        # NUMA node: with 8 ranks the host-to-device uploads never cross sockets
        numa = nns.bind_numa(dev)
        print(f"rank {rank}: GPU {dev} NUMA binding: {numa}", file=sys.stderr, flush=True)
    workdir = os.path.join(tempfile.gettempdir(), f"nnsx_bench_{os.getuid()}_{rank}")
    os.makedirs(workdir, exist_ok=True)
    cfg = CONFIGS[a.config]
    model_name = a.model if a.config == "mbv2" else cfg["model"]
    model_path = os.path.join(workdir, f"{model_name}.pt")
    layout = "nhwc"
    export(model_name, model_path, layout=layout)
    from nnstreamer_amd.models.posenet import write_pose_labels
    from nnstreamer_amd.models.ssd import write_box_priors, write_coco_labels

    files = dict(labels=write_labels(os.path.join(workdir, "labels.txt")),
                 coco=write_coco_labels(os.path.join(workdir, "coco.txt")),
                 priors=write_box_priors(os.path.join(workdir, "priors.txt")),
                 pose=write_pose_labels(os.path.join(workdir, "pose17.txt")))
    S = cfg["size"]

    B = a.batch
    total = a.warmup + a.steps
    frames = total * B
    graph = "true" if (use_gpu and not a.no_graph) else "false"
    # fused models take the raw uint8 frame and apply the tensor_transform normalisation
    # ((x + add) / div, bit-identical) inside their first kernel; plain models keep the element
    fuse_norm = "fused" in model_name and not a.no_fuse_norm
    accel = "true:gpu" if use_gpu else "false"
    # The source cycles through a ring of distinct pre-rendered frames (a camera ring
    # buffer).  The ring is sized to 512 MiB, twice the MI355X's 256 MiB last-level
    # cache, so every batch's H2D upload really crosses the host link.
    frame_bytes = S * S * 3
    pool = max(64, -(-512 * 2**20 // frame_bytes)) if use_gpu else 16
    desc = (
        f"videotestsrc num-buffers={frames} pattern=snow pool-size={pool} "
        f"! video/x-raw,format=RGB,width={S},height={S},framerate=0/1 "
        f"! tensor_converter frames-per-tensor={B} device={dev} "
        # thread boundary: the next batch's upload is issued while the filter thread
        # is still submitting this batch's kernels
        f"! queue max-size-buffers=2 "
        + (f"! tensor_transform mode=arithmetic option={cfg['norm']} " if not fuse_norm else "")
        + f"! tensor_filter framework=pytorch model={model_path} input=3:{S}:{S}:{B} "
        f"inputtype={'uint8' if fuse_norm else 'float32'} "
        f"accelerator={accel} device={dev} custom=hipgraph:{graph} "
        + (f"! tee name=t t. ! queue max-size-buffers={a.queue} " if cfg.get("gather") else
           f"! queue max-size-buffers={a.queue} ")
        + f"! {cfg['decoder'].format(**files)} "
        f"! tensor_sink name=sink"
        # multi-source: every rank's PoseNet outputs are all-gathered (RCCL over xGMI
        # between GPUs, the TCP store on CPU) so each rank holds the synchronised
        # multi-camera set -- one collective per batch, beside the local decoder
        + (f" t. ! queue max-size-buffers={a.queue} ! tensor_allgather name=ag channel=posenet mode=concat "
           f"rank={rank} world-size={world} device={dev} comm-backend={a.comm_backend} ! fakesink" if cfg.get("gather") else "")
    )
    fan = bool(cfg.get("fan")) and world > 1
    workers = world - 1 if fan else world
    if fan:
        link = f"connect-type=RCCL rccl-mode=scatter topic=fan rank={rank} world-size={world} device={dev}"
        if rank == 0:  # the camera rank: upload batches, scatter them round-robin to the workers
            desc = (f"videotestsrc num-buffers={frames * workers} pattern=snow pool-size={pool} "
                    f"! video/x-raw,format=RGB,width={S},height={S},framerate=0/1 "
                    f"! tensor_converter frames-per-tensor={B} device={dev} ! queue max-size-buffers=4 "
                    f"! edgesink {link}")
        else:
            desc = (f"edgesrc {link} peer-rank=0 ! queue max-size-buffers=2 "
                    f"! tensor_filter framework=pytorch model={model_path} input=3:{S}:{S}:{B} "
                    f"inputtype={'uint8' if fuse_norm else 'float32'} accelerator={accel} device={dev} "
                    f"custom=hipgraph:{graph} ! queue max-size-buffers={a.queue} "
                    f"! {cfg['decoder'].format(**files)} ! tensor_sink name=sink")
    per_step = B if cfg["per_frame"] else 1  # sink buffers per batch
    pipe = nns.parse_launch(desc)
    sink = pipe.get_by_name("sink")
    # native per-buffer arrival stats (no Python callback per frame); sync-device
    # makes an arrival mean "the GPU has produced this frame", not "it was queued"
    if sink is not None:  # (the fan-out camera rank has no sink: it only produces)
        sink.set_property("emit-signal", "false")
        sink.set_property("sync-device", "true")
        sink.set_property("stats-every", "1")

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
    gathered = pipe.get_by_name("ag").get_property("comm-bytes") if cfg.get("gather") else None
    pipe.stop()

    recs = [tuple(int(v) for v in e.split(":")) for e in sink.get_property("stats").split(",") if e] if sink else []
    arrivals = [t / 1e9 for i, (t, _) in enumerate(recs) if (i + 1) % per_step == 0]  # last frame of each batch
    step_lat = [[lat / 1e6 for _, lat in recs[k * per_step:(k + 1) * per_step] if lat >= 0]
                for k in range(len(arrivals))]
    n = len(arrivals)
    if sink is None:
        stats = torch.zeros(3, dtype=torch.float64)  # the workers' clocks decide
    else:
        if n < total:
            raise SystemExit(f"rank {rank}: only {n}/{total} batches reached the sink")
        # timed region: exactly K steps after W warmup steps
        t0 = arrivals[a.warmup - 1] if a.warmup > 0 else t_start
        t1 = arrivals[a.warmup + a.steps - 1]
        elapsed = t1 - t0
        timed = [x for k in range(a.warmup, a.warmup + a.steps) for x in step_lat[k]]
        lat = np.array(timed) if timed else np.array([0.0])
        if fan:  # PTS were stamped on the camera rank's clock: no per-frame latency here
            lat = np.array([0.0])
        stats = torch.tensor([elapsed, float(np.percentile(lat, 50)), float(np.percentile(lat, 99))],
                             dtype=torch.float64)
    if dist is not None:
        if dist.get_backend() == "nccl":
            stats = stats.cuda()
        dist.all_reduce(stats, op=dist.ReduceOp.MAX)
        stats = stats.cpu()
    elapsed, p50, p99 = stats.tolist()
    ms_per_step = elapsed / a.steps * 1e3
    fps_total = workers * a.steps * B / elapsed
    if rank == 0:
        out = {
            "metric": cfg["metric"],
            "value": round(fps_total, 2),
            "unit": "frames/s",
            "n_gpus": world if use_gpu else 0,
            "steps": a.steps,
            "warmup": a.warmup,
            "ms_per_step": round(ms_per_step, 4),
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": (round(fps_total / CPU_BASELINE_FPS, 2) if a.config == "mbv2" else None),
            "dtype": "bf16" if "fused" in a.model else "fp32",
            "data": "synthetic video frames (videotestsrc pattern=snow), random-init weights",
            "p50_latency_ms": None if fan else round(p50, 3),
            "p99_latency_ms": None if fan else round(p99, 3),
            "frames_per_step_per_gpu": B,
            "preprocess": ("tensor_transform normalisation fused into the model's stem kernel (uint8 input)"
                           if fuse_norm else "tensor_transform element"),
            "wall_s": round(t_end - t_start, 3),
            "numa_binding": numa,
            **({"allgather_bytes_sent_received_rank0": gathered} if gathered is not None else {}),
            "config": {
                "model": cfg["desc"],
                "global_batch": B * world,
                "seq_len": 1,
                "parallelism": f"fan-out 1->{workers} (RCCL scatter)" if fan else f"branch-dp{world}",
                "pipeline": desc,
            },
        }
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
