#!/usr/bin/env python3
"""Headline benchmark: end-to-end frames/sec + p50 per-frame latency of the
MobileNetV2 224x224 image-classification pipeline (BASELINE.json config 2),
one pipeline per GPU (weak scaling: per-GPU work fixed as N grows).

    python bench.py --gpus N --steps K --warmup W

`--gpus N` without a launcher: this process spawns N rank processes itself
(RANK/LOCAL_RANK/WORLD_SIZE/MASTER_* set, one GPU each) BEFORE anything here
touches the GPU, waits for them and exits with the first failure's code.
Under torch.distributed.run the ranks come from the environment and
WORLD_SIZE must equal N.

Pipeline (one per rank, pinned to GPU LOCAL_RANK):

  videotestsrc pattern=snow ! video/x-raw,format=RGB,width=224,height=224
    ! tensor_converter frames-per-tensor=B device=<gpu>     # H2D into HBM, B frames per tensor
    ! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5   # the reference string
    ! queue
    ! tensor_filter framework=pytorch model=mbv2.pt accelerator=true:gpu custom=hipgraph:true
    ! tensor_decoder mode=image_labeling option1=labels.txt # HIP argmax, labels D2H
    ! tensor_sink

The tensor_transform is the reference's own normalisation element
(gsttensor_transform.c:1241-1412).  At caps negotiation tensor_filter absorbs
it (runtime/fusion.h): the model's uint8 input table takes the transform's exact
fp32 arithmetic and the transform passes the uint8 frames through, so the
first kernel reads 1 byte per channel instead of 4.  `--no-absorb` keeps the
transform's own kernel (float32 frames into the model) for comparison.

Precision: the reference runs the model in float32 (tensor_filter_pytorch.cc
:517-536), so the headline `value` is the fp32 engine (fp32 activations,
weights and accumulation: v_mfma_f32_16x16x4_f32 GEMMs, fp32 depthwise).
`--precision bf16|both` also measures the bf16 engine (`value_bf16`).
After the headline run a short sweep over smaller batches (`--sweep`,
default 8,32,128) reports throughput and p50 latency per batch size
(`sweep`), and a live batch-1 run reports the pipeline's per-frame latency.

A "step" is one batch of B frames reaching the sink.  W batches warm up
(graph capture, allocator), then the wall time of exactly K batches is
measured at the sink; ranks are bracketed by barrier + device synchronize,
the max over ranks is reported.  The filter's HIP events give the
device-clock time of the same K batches (`gpu_event_fps`); `value` uses the
slower of the two windows (`sink_fps` is the sink-only figure).  Latency =
sink arrival - frame capture time (the PTS of the oldest frame in the batch);
`p50_latency_ms_b1` is a separate batch-1 run of the same pipeline fed by
a live camera (`--latency-fps`, frames released at their PTS), so it measures
the pipeline's latency, not queueing behind a free-running source.
Data: synthetic video frames, random-init weights.
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--batch", type=int, default=int(os.environ.get("NNSX_BENCH_BATCH", "512")))
    ap.add_argument("--batch-bf16", type=int, default=int(os.environ.get("NNSX_BENCH_BATCH_BF16", "128")),
                    help="batch of the secondary bf16 run (its kernels were tuned at 128; at 512 they "
                         "measured 71-125k frames/s from run to run, at 128 117-125k)")
    ap.add_argument("--precision", default=os.environ.get("NNSX_BENCH_PRECISION", "fp32"),
                    choices=["fp32", "bf16", "both"],
                    help="fp32 = reference precision (headline); bf16 = secondary; both = fp32 headline + bf16")
    ap.add_argument("--engine", default=os.environ.get("NNSX_BENCH_ENGINE", "fused"),
                    choices=["fused", "lowered", "torch"],
                    help="fused = nnsx's exported model on the CDNA4 kernels; lowered = the plain TorchScript model, "
                         "lowered onto the same kernels by tensor_filter at load (custom=lower:auto); torch = the "
                         "plain model on PyTorch/MIOpen (custom=lower:off)")
    ap.add_argument("--latency-frames", type=int, default=int(os.environ.get("NNSX_BENCH_LAT_FRAMES", "300")),
                    help="frames of the batch-1 latency run (0 = skip)")
    ap.add_argument("--latency-fps", type=int, default=int(os.environ.get("NNSX_BENCH_LAT_FPS", "0")),
                    help="frame rate of the live camera in the batch-1 latency run (0: the config's, "
                         "500 unless the model needs longer per frame)")
    ap.add_argument("--no-graph", action="store_true")
    ap.add_argument("--no-absorb", "--no-fuse-norm", dest="no_absorb", action="store_true",
                    help="tensor_filter absorb-transform=false: the tensor_transform runs its own kernel and the "
                         "model reads float32 frames")
    ap.add_argument("--sweep", default=os.environ.get("NNSX_BENCH_SWEEP", "8,32,128"),
                    help="comma-separated batch sizes of the throughput / latency sweep ('' = skip)")
    ap.add_argument("--sweep-steps", type=int, default=100, help="timed steps per sweep point")
    ap.add_argument("--sweep-warmup", type=int, default=20,
                    help="warm-up steps per sweep point (replay lanes reach steady state)")
    ap.add_argument("--extra-configs", default=os.environ.get("NNSX_BENCH_EXTRA", "deeplab_fan,posenet_multi"),
                    help="WORLD_SIZE > 1: short passes of these multi-rank configs after the headline "
                         "(their frames/s and RCCL world as extra keys; '' = skip)")
    ap.add_argument("--extra-steps", type=int, default=20, help="timed steps of each extra config pass")
    ap.add_argument("--no-selfcheck", action="store_true",
                    help="WORLD_SIZE > 1: skip the rank-group data-plane self-check (run after the headline)")
    ap.add_argument("--selfcheck-timeout-ms", type=int, default=60000,
                    help="group timeout of the self-check (a missing member fails an operation after this)")
    ap.add_argument("--aux-timeout", type=float, default=float(os.environ.get("NNSX_BENCH_AUX_TIMEOUT", "300")),
                    help="seconds for the whole self-check + extra-config phase; on expiry the headline is "
                         "printed with aux_timeout and every rank exits 0")
    ap.add_argument("--cpu", action="store_true", help="CPU reference path (device=-1, torch CPU)")
    # (depth 1 / 1: same frames/s as 4 / 2 at batch 512, p50 23 vs 37 ms: profiles/r4_mbv2_ab_b512.txt q11)
    ap.add_argument("--queue", type=int, default=int(os.environ.get("NNSX_BENCH_QUEUE", "1")),
                    help="queue depth between filter and decoder")
    ap.add_argument("--queue-in", type=int, default=int(os.environ.get("NNSX_BENCH_QUEUE_IN", "1")),
                    help="queue depth between converter and filter")
    ap.add_argument("--model-broadcast", default=os.environ.get("NNSX_BENCH_BCAST", "auto"),
                    choices=["off", "tcp", "rccl", "auto"],
                    help="N > 1: rank 0 broadcasts the model bytes to every rank at load over this data plane")
    ap.add_argument("--comm-backend", default="auto", choices=["auto", "rccl", "tcp"],
                    help="posenet_multi: tensor_allgather data plane")
    ap.add_argument("--fan-transport", default=os.environ.get("NNSX_BENCH_FAN", "shm"), choices=["shm", "rccl"],
                    help="deeplab_fan: shm = rank 0's cameras render into shared rings and every worker's "
                         "tensor_converter DMAs its own camera over its own GPU's link (edgesink/edgesrc "
                         "connect-type=SHM); rccl = rank 0 uploads all cameras, tensor_demux + RCCL scatter")
    ap.add_argument("--config", default=os.environ.get("NNSX_BENCH_CONFIG", "mbv2"),
                    choices=sorted(CONFIGS), help="BASELINE.json config (default: the headline MobileNetV2 pipeline)")
    return ap.parse_args(argv)


# best CPU reference path for the MobileNetV2 pipeline
# (identical pipeline, host elements + fp32 PyTorch CPU, 8 vCPU).
CPU_BASELINE_FPS = 254.1

_FAN_RUN = 0  # deeplab_fan passes so far (each gets fresh shared-ring names and ports)

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
    "deeplab": dict(size=513, model="deeplab_fused_lowres", norm="typecast:float32,div:255.0",
                    decoder="tensor_decoder mode=image_segment option1=tflite-deeplab option3=513:513", per_frame=True,
                    metric="end-to-end frames/sec + p50 per-frame latency, DeepLabV3 513x513 segmentation pipeline",
                    desc="DeepLabV3-MobileNetV2 513x513 (tensor_filter + image_segment decoder)"),
    # (DeepLab: the model ships its 33x33 logits; the decoder's option3 resizes
    # them bilinearly per label inside the argmax pass -- same frames as a
    # 513x513x21 model output, without the 22 MB-per-frame score map)
    # BASELINE.json config 4: "8 parallel video branches fanned via tensor_demux + RCCL".
    # Rank 0 holds the N cameras: tensor_converter per camera -> tensor_mux -> tensor_demux;
    # demux pad 0 feeds rank 0's own DeepLab branch, pad r goes to rank r through
    # edgesink connect-type=RCCL (a two-member group {0, r}: ncclSend / ncclRecv over
    # xGMI on a per-direction link).  Every rank runs DeepLabV3 + image_segment.
    "deeplab_fan": dict(size=513, model="deeplab_fused_lowres", norm="typecast:float32,div:255.0",
                        decoder="tensor_decoder mode=image_segment option1=tflite-deeplab option3=513:513", per_frame=True, fan=True,
                        metric="end-to-end frames/sec, DeepLabV3 513x513 segmentation, N video branches fanned "
                               "via tensor_demux + RCCL",
                        desc="DeepLabV3-MobileNetV2 513x513, N camera branches on rank 0 demuxed to N GPUs over RCCL"),
    # BASELINE.json config 5: "PoseNet multi-source pipeline with tensor_mux sync +
    # nnstreamer-edge RCCL all-gather".  Every rank: camera -> PoseNet -> pose decoder,
    # and its pose tensors published with edgesink connect-type=RCCL rccl-mode=allgather
    # (one ncclAllGather per round over all cameras); one edgesrc per other camera feeds
    # tensor_mux sync-mode=slowest next to the rank's own stream: every rank holds the
    # synchronised N-camera pose set.
    "posenet_multi": dict(size=257, model="posenet_fused", norm="typecast:float32,add:-127.5,div:127.5",
                          decoder="tensor_decoder mode=pose_estimation option1=640:480 option2=257:257 "
                                  "option3={pose} option4=heatmap-offset", per_frame=True, gather=True,
                          metric="end-to-end frames/sec, PoseNet multi-source pipeline with tensor_mux sync "
                                 "+ edge RCCL all-gather",
                          desc="PoseNet-MobileNetV1 257x257 per rank, pose tensors all-gathered (edgesink/edgesrc "
                               "rccl-mode=allgather) into tensor_mux sync-mode=slowest"),
    "posenet": dict(size=257, model="posenet_fused", norm="typecast:float32,add:-127.5,div:127.5",
                    decoder="tensor_decoder mode=pose_estimation option1=640:480 option2=257:257 option3={pose} "
                            "option4=heatmap-offset", per_frame=True,
                    metric="end-to-end frames/sec + p50 per-frame latency, PoseNet 257x257 pipeline",
                    desc="PoseNet-MobileNetV1 257x257 (tensor_filter + pose_estimation decoder)"),
}


# ----------------------------------------------------------------- launcher ----
def _free_port() -> int:
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def spawn_ranks(n: int, argv) -> int:
    """Start n rank processes of this script (one per GPU) and wait for them.

    Runs before anything in this process touches the GPU (no torch.cuda call,
    no HIP runtime), and starts children instead of exec'ing.  Every rank
    reads its GPU from LOCAL_RANK; rank 0 prints the JSON line."""
    port = _free_port()
    procs = []
    for r in range(n):
        env = dict(os.environ)
        env.update(RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n), GROUP_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), NNSX_BENCH_SPAWNED="1")
        procs.append(subprocess.Popen([sys.executable, "-u", os.path.abspath(__file__), *argv], env=env))
    rc = 0
    alive = set(range(n))
    while alive:
        for r in sorted(alive):
            code = procs[r].poll()
            if code is None:
                continue
            alive.discard(r)
            if code != 0 and rc == 0:
                rc = code if code > 0 else 1
                print(f"bench: rank {r} exited with {code}; stopping the other ranks", file=sys.stderr, flush=True)
                for q in alive:
                    procs[q].terminate()
        time.sleep(0.05)
    for p in procs:
        p.wait()
    return rc


# ---------------------------------------------------------------- one run ----
def run_pipeline(a, nns, cfg, model_name, model_path, files, B, steps, warmup, rank, world, dev, use_gpu, dist,
                 live_fps=0):
    """Build and run one pipeline to EOS; return this rank's timing record.

    live_fps > 0: the source is a live camera at that frame rate (frames are
    released at their PTS), so per-frame latency is the pipeline's own latency
    rather than time spent queued behind a source that runs ahead."""
    S = cfg["size"]
    total = warmup + steps
    frames = total * B
    graph = "true" if (use_gpu and not a.no_graph) else "false"
    # the reference string always carries the tensor_transform; tensor_filter absorbs it
    # into fused models (uint8 input table) unless --no-absorb
    absorb = "false" if a.no_absorb else "true"
    accel = "true:gpu" if use_gpu else "false"
    # The source cycles through a ring of distinct pre-rendered frames (a camera ring
    # buffer).  The ring is sized to 512 MiB, twice the MI355X's 256 MiB last-level
    # cache, so every batch's H2D upload really crosses the host link.
    frame_bytes = S * S * 3
    pool = max(64, -(-512 * 2**20 // frame_bytes)) if use_gpu else 16
    pool = min(pool, max(frames, 16))
    # with several ranks the model is loaded once: rank 0 reads the file and
    # broadcasts its bytes to every rank at filter start (custom=broadcast:0;
    # --model-broadcast selects the data plane, TCP store by default)
    bcast = ""
    if world > 1 and a.model_broadcast != "off" and not cfg.get("fan"):  # (fan-out: rank 0 runs no filter)
        bcast = f",broadcast:0,broadcast-backend:{a.model_broadcast},broadcast-name:{model_name}-b{B}"
    lower = ",lower:off" if a.engine == "torch" else ""
    filt = (f"tensor_filter name=filt framework=pytorch model={model_path} input=3:{S}:{S}:{B} "
            f"inputtype=float32 absorb-transform={absorb} accelerator={accel} device={dev} "
            f"custom=hipgraph:{graph}{bcast}{lower} device-stats={'true' if use_gpu else 'false'} ")
    live = f"is-live=true " if live_fps > 0 else ""
    gather = bool(cfg.get("gather"))
    # multi-source sync: the cameras of every rank stamp the same frame clock (frame k
    # at k ms) so tensor_mux sync-mode=slowest pairs round k of every camera
    fr = live_fps if live_fps > 0 else (1000 if gather else 0)
    # throughput runs: queues are thread boundaries, so the next batch's upload
    # is issued while the filter thread still submits this batch's kernels, and
    # the decoder's read-back overlaps the next forward.  The live batch-1
    # latency run keeps the whole chain in the source's streaming thread: no
    # queue hand-off on the path of a frame.
    q1 = f"! queue max-size-buffers={a.queue_in} " if live_fps <= 0 else ""
    q2 = f"! queue max-size-buffers={a.queue} " if live_fps <= 0 else ""
    desc = (
        f"videotestsrc num-buffers={frames} pattern=snow pool-size={pool} {live}"
        f"! video/x-raw,format=RGB,width={S},height={S},framerate={fr}/1 "
        f"! tensor_converter frames-per-tensor={B} device={dev} "
        + f"! tensor_transform name=norm mode=arithmetic option={cfg['norm']} "
        + q1
        + f"! {filt}"
        + (f"! tee name=t t. ! queue max-size-buffers={a.queue} " if gather else q2)
        + f"! {cfg['decoder'].format(**files)} "
        f"! tensor_sink name=sink"
    )
    if gather:
        # this camera's pose tensors go out on the topic (one all-gather round per
        # batch); every other camera comes back through its own edgesrc, and
        # tensor_mux pairs the N streams by timestamp (slowest policy)
        edge = (f"connect-type=RCCL rccl-mode=allgather topic=posenet-b{B} rank={rank} world-size={world} "
                f"comm-backend={a.comm_backend}")
        desc += (f" t. ! queue max-size-buffers={a.queue} ! edgesink name=ag {edge} device={dev}"
                 f" t. ! queue max-size-buffers={a.queue} ! mux.sink_{rank}"
                 + "".join(f" edgesrc name=sub{r} {edge} peer-rank={r} device={dev} ! queue max-size-buffers="
                           f"{a.queue} ! mux.sink_{r}" for r in range(world) if r != rank)
                 + " tensor_mux name=mux sync-mode=slowest ! tensor_sink name=msink")
    fan = bool(cfg.get("fan")) and world > 1
    workers = world
    if fan:
        def link(r):  # the two-member group of demux branch r: rank 0 -> rank r
            return (f"connect-type=RCCL rccl-mode=scatter topic=fan{r}-b{B} group-ranks=0,{r} rank={rank} "
                    f"world-size={world} device={dev} comm-backend={a.comm_backend}")
        branch = (f"! tensor_transform name=norm mode=arithmetic option={cfg['norm']} ! {filt}"
                  f"! queue max-size-buffers={a.queue} ! {cfg['decoder'].format(**files)} ! tensor_sink name=sink")
        cam_pool = max(2 * B, min(pool, -(-128 * 2**20 // frame_bytes)))
        if a.fan_transport == "shm":
            # same host: camera r's ring lives in a named shared segment on rank 0
            # (videotestsrc pool-shm); rank r subscribes (edgesrc connect-type=SHM),
            # gets its frames as references into its hipHostRegister'ed mapping and
            # its own tensor_converter DMAs them over ITS GPU's host link -- the
            # ingest scales with the ranks instead of funnelling through GPU 0
            # (profiles/r6_shared_ring_ingest.txt); rank 0 runs camera 0's branch
            global _FAN_RUN
            _FAN_RUN += 1
            mport = int(os.environ.get("MASTER_PORT", "29500"))
            port = lambda r: 20000 + (mport * 37 + _FAN_RUN * 16 + r) % 40000  # noqa: E731
            tag = f"{mport}-{_FAN_RUN}"
            conv = f"! tensor_converter frames-per-tensor={B} device={dev} ! queue max-size-buffers=2 "
            shm_pool = max(2 * B, min(cam_pool, -(-64 * 2**20 // frame_bytes)))  # (64 MiB of /dev/shm per camera)
            cam = (f"videotestsrc num-buffers={frames} pattern=snow pool-size={shm_pool} {{shm}}"
                   f"! video/x-raw,format=RGB,width={S},height={S},framerate=0/1 ")
            if rank == 0:
                desc = (cam.format(shm="") + conv + branch + " "
                        + " ".join(cam.format(shm=f"pool-shm=nnsx-fan-{tag}-{r} ")
                                   + f"! edgesink name=fan{r} port={port(r)} connect-type=SHM wait-connection=1"
                                   for r in range(1, world)))
            else:
                desc = (f"edgesrc name=fan dest-host=127.0.0.1 dest-port={port(rank)} connect-type=SHM "
                        + conv + branch)
        elif rank == 0:  # the N cameras: upload, mux, demux -> own branch + one RCCL edge per other rank
            desc = ("".join(f"videotestsrc num-buffers={frames} pattern=snow pool-size={cam_pool} "
                            f"! video/x-raw,format=RGB,width={S},height={S},framerate=0/1 "
                            f"! tensor_converter frames-per-tensor={B} device={dev} ! queue max-size-buffers=2 "
                            f"! mux.sink_{r} " for r in range(world))
                    + "tensor_mux name=mux sync-mode=nosync ! tensor_demux name=d "
                    + f"d.src_0 ! queue max-size-buffers=2 {branch} "
                    + " ".join(f"d.src_{r} ! queue max-size-buffers=2 ! edgesink name=fan{r} {link(r)}"
                               for r in range(1, world)))
        else:
            desc = f"edgesrc name=fan {link(rank)} peer-rank=0 ! queue max-size-buffers=2 {branch}"
    per_step = B if cfg["per_frame"] else 1  # sink buffers per batch
    pipe = nns.parse_launch(desc)
    sink = pipe.get_by_name("sink")
    filt_el = pipe.get_by_name("filt")
    # native per-buffer arrival stats (no Python callback per frame); sync-device
    # makes an arrival mean "the GPU has produced this frame", not "it was queued"
    if sink is not None:  # (the fan-out camera rank has no sink: it only produces)
        sink.set_property("emit-signal", "false")
        sink.set_property("sync-device", "true")
        sink.set_property("stats-every", "1")
        # roctx marks at the timed window's ends (the arrivals of batch W and W + K):
        # scripts/kstats.py --window keeps only the kernels that ran between them
        sink.set_property("roctx-marks", f"{warmup * per_step},{(warmup + steps) * per_step}")

    import torch

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
    gathered = pipe.get_by_name("ag").get_property("comm-bytes") if gather else None
    mux_sets = None
    if gather:
        ms = pipe.get_by_name("msink")
        mux_sets = int(ms.get_property("frames")) if ms is not None else None
    dev_stamps = filt_el.get_property("device-stamps") if (filt_el is not None and use_gpu) else ""
    absorbed = filt_el.get_property("absorbed") if filt_el is not None else ""
    lowered = filt_el.get_property("lowered") if filt_el is not None else ""
    absorbed_dec = filt_el.get_property("absorbed-decoder") if filt_el is not None else ""
    # the nnsx rank groups this rank actually used (data plane : members)
    groups = {}
    if filt_el is not None and filt_el.get_property("model-broadcast"):
        groups["model_broadcast"] = filt_el.get_property("model-broadcast")
    for el in ["ag"] + [f"fan{r}" for r in range(1, world)] + ["fan"]:
        e = pipe.get_by_name(el)
        if e is not None and e.get_property("comm-group"):
            groups["edge_allgather" if el == "ag" else f"edge_{el}"] = e.get_property("comm-group")
    pipe.stop()

    import numpy as np

    rec = dict(elapsed=0.0, p50=0.0, p99=0.0, gpu_elapsed=0.0, gpu_busy_ms=0.0, wall=t_end - t_start,
               desc=desc, fan=fan, workers=workers, absorbed=absorbed, absorbed_dec=absorbed_dec, gathered=gathered,
               lowered=lowered,
               groups=groups, mux_sets=mux_sets)
    recs = [tuple(int(v) for v in e.split(":")) for e in sink.get_property("stats").split(",") if e]
    arrivals = [t / 1e9 for i, (t, _) in enumerate(recs) if (i + 1) % per_step == 0]  # last frame of each batch
    step_lat = [[lat / 1e6 for _, lat in recs[k * per_step:(k + 1) * per_step] if lat >= 0]
                for k in range(len(arrivals))]
    if len(arrivals) < total:
        raise SystemExit(f"rank {rank}: only {len(arrivals)}/{total} batches reached the sink")
    # timed region: exactly K steps after W warmup steps
    t0 = arrivals[warmup - 1] if warmup > 0 else t_start
    t1 = arrivals[warmup + steps - 1]
    rec["elapsed"] = t1 - t0
    timed = [x for k in range(warmup, warmup + steps) for x in step_lat[k]]
    # (multi-source: the cameras stamp a shared synthetic frame clock, so sink-side
    # latency is not a pipeline latency there)
    lat = np.array(timed) if (timed and not fan and not gather) else np.array([0.0])
    rec["p50"] = float(np.percentile(lat, 50))
    rec["p99"] = float(np.percentile(lat, 99))
    # device-clock cross-check: the filter's end-of-invoke events of the same K batches
    ds = [tuple(int(v) for v in e.split(":")) for e in dev_stamps.split(",") if e]
    if len(ds) >= total and warmup > 0:
        # (replay lanes: invokes may end out of order; the window runs from the
        # last warmup end to the last timed end)
        rec["gpu_elapsed"] = (max(d[0] for d in ds[:warmup + steps]) - max(d[0] for d in ds[:warmup])) / 1e9
        rec["gpu_busy_ms"] = float(np.median([d[1] for d in ds[warmup:warmup + steps]])) / 1e6
        if os.environ.get("NNSX_BENCH_SERIES") == "1":  # (diagnostics: every invoke's device ms, warm-up included)
            print(f"rank {rank}: device ms per invoke " + " ".join(f"{d[1] / 1e6:.3f}" for d in ds[:warmup + steps]),
                  file=sys.stderr, flush=True)
    return rec


def main():
    a = parse_args()
    if "WORLD_SIZE" not in os.environ and a.gpus > 1:
        # launcher mode: N fresh rank processes, nothing here touches the GPU
        sys.exit(spawn_ranks(a.gpus, sys.argv[1:]))

    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != a.gpus:
        raise SystemExit(f"bench: --gpus {a.gpus} but WORLD_SIZE={world}: refusing to report a mismatched run")
    dist = None
    if world > 1:
        import torch.distributed as dist

        backend = "nccl" if (torch.cuda.is_available() and not a.cpu) else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local_rank)
        dist.init_process_group(backend=backend)
        if dist.get_world_size() != a.gpus:
            raise SystemExit(f"bench: process group has {dist.get_world_size()} ranks, expected {a.gpus}")

    import nnstreamer_amd as nns
    from nnstreamer_amd.models.export import export, write_labels

    use_gpu = (not a.cpu) and torch.cuda.is_available() and nns.gpu_count() > 0
    if use_gpu and world > nns.gpu_count():
        raise SystemExit(f"bench: {world} ranks but only {nns.gpu_count()} GPUs visible")
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
    from nnstreamer_amd.models.posenet import write_pose_labels
    from nnstreamer_amd.models.ssd import write_box_priors, write_coco_labels

    files = dict(labels=write_labels(os.path.join(workdir, "labels.txt")),
                 coco=write_coco_labels(os.path.join(workdir, "coco.txt")),
                 priors=write_box_priors(os.path.join(workdir, "priors.txt")),
                 pose=write_pose_labels(os.path.join(workdir, "pose17.txt")))

    # which engines to run: (label, model name, dtype)
    base = cfg["model"]
    if a.engine in ("torch", "lowered") or not use_gpu:
        plain = base.replace("_fused", "").replace("_lowres", "")  # the plain oracle emits full-size maps
        runs = [("fp32", plain, "fp32")]
    else:
        runs = []
        if a.precision in ("fp32", "both"):
            runs.append(("fp32", base + "_fp32", "fp32"))
        if a.precision in ("bf16", "both"):
            runs.append(("bf16", base, "bf16"))

    results = {}
    for label, model_name, dtype in runs:
        model_path = os.path.join(workdir, f"{model_name}.pt")
        export(model_name, model_path, layout="nhwc")
        eb = a.batch_bf16 if (label == "bf16" and a.precision == "both") else a.batch
        rec = run_pipeline(a, nns, cfg, model_name, model_path, files, eb, a.steps, a.warmup, rank, world, dev,
                           use_gpu, dist)
        rec["dtype"] = dtype
        rec["batch"] = eb
        results[label] = rec

    # batch-1 latency of the headline engine (the "p50 per-frame latency" half of the metric)
    lat_b1 = None
    if a.latency_frames > 0 and not cfg.get("fan") and not cfg.get("gather"):
        label, model_name, _ = runs[0]
        model_path = os.path.join(workdir, f"{model_name}.pt")
        w1 = max(10, a.latency_frames // 5)
        lat_b1 = run_pipeline(a, nns, cfg, model_name, model_path, files, 1, a.latency_frames, w1, rank, world, dev,
                              use_gpu, dist, live_fps=a.latency_fps or cfg.get("lat_fps", 500))

    # throughput / latency trade-off at smaller batches (same engine, same pipeline)
    sweep = []
    if a.sweep and use_gpu and not cfg.get("fan"):
        label, model_name, _ = runs[0]
        model_path = os.path.join(workdir, f"{model_name}.pt")
        for sb in [int(x) for x in a.sweep.split(",") if x.strip()]:
            if sb == a.batch:
                continue
            r = run_pipeline(a, nns, cfg, model_name, model_path, files, sb, a.sweep_steps, a.sweep_warmup, rank,
                             world, dev, use_gpu, dist)
            sweep.append((sb, r))

    # per-rank records, all-gathered over the job's process group (RCCL on GPUs):
    # [elapsed, p50, p99, gpu_elapsed, gpu_busy] per engine + batch-1 p50/p99
    # + [max(sink, device) elapsed, p50] per sweep batch
    vec = []
    for label, _, _ in runs:
        r = results[label]
        vec += [r["elapsed"], r["p50"], r["p99"], r["gpu_elapsed"], r["gpu_busy_ms"]]
    vec += [lat_b1["p50"], lat_b1["p99"]] if lat_b1 else [0.0, 0.0]
    for _, r in sweep:
        vec += [max(r["elapsed"], r["gpu_elapsed"]), r["p50"]]
    per_rank, pg_world, pg_backend = gather_rows(vec, world, dist, torch)
    out = None
    if rank == 0:
        out = headline_record(a, cfg, runs, results, lat_b1, sweep, per_rank, world, use_gpu, numa,
                              pg_world, pg_backend, torch)

    # WORLD_SIZE > 1, AFTER the headline is recorded: the rank-group data-plane
    # self-check (every comm::Group operation on frame-sized payloads) and short
    # passes of the multi-rank configs (config 4's demux fan-out over RCCL p2p,
    # config 5's edge all-gather).  Each is guarded on its own (an exception is
    # recorded, not raised) and a watchdog bounds the whole auxiliary phase: if
    # it expires, rank 0 prints the headline with `aux_timeout` and every rank
    # exits 0, so no auxiliary pass can cost the headline record.
    if world > 1 and (not a.no_selfcheck or a.extra_configs):
        run_aux(a, nns, cfg, files, rank, world, dev, use_gpu, dist, workdir, out, torch, np)
    if rank == 0:
        print(json.dumps(out), flush=True)
    if dist is not None:
        dist.destroy_process_group()


SC_KEYS = ["allgather", "allgather_ragged", "broadcast", "scatter", "p2p_ring", "p2p_exchange"]


def gather_rows(vec, world, dist, torch):
    """One all_gather of a per-rank float vector over the job's process group."""
    stats = torch.tensor(vec, dtype=torch.float64)
    if dist is None:
        return stats.view(1, -1), 1, None
    if dist.get_backend() == "nccl":
        stats = stats.cuda()
    gathered = [torch.zeros_like(stats) for _ in range(world)]
    dist.all_gather(gathered, stats)
    per_rank = torch.stack([g.cpu() for g in gathered])  # [world, len]
    return per_rank, len(gathered), ("rccl" if dist.get_backend() == "nccl" else dist.get_backend())


def headline_record(a, cfg, runs, results, lat_b1, sweep, per_rank, world, use_gpu, numa, pg_world, pg_backend,
                    torch):
    head_label = runs[0][0]
    head = results[head_label]
    workers = head["workers"]
    fan = head["fan"]
    B = a.batch

    def agg(i, B=B):
        cols = per_rank[:, i * 5:(i + 1) * 5]
        active = cols  # every rank runs a branch (config 4: rank 0's own demux pad too)
        sink_el = float(active[:, 0].max())
        gpu_el = float(active[:, 3].max())
        # the timed window on the slower of the two clocks: sink arrivals can
        # run ahead of the device when batches computed during warmup are
        # still queued at the window's start (up to queue-depth / K)
        eff = torch.maximum(active[:, 0], active[:, 3])
        elapsed = float(eff.max())
        per = [round(a.steps * B / float(e), 2) if e > 0 else None for e in eff.tolist()]
        return dict(
            fps=workers * a.steps * B / elapsed if elapsed > 0 else 0.0,
            sink_fps=workers * a.steps * B / sink_el if sink_el > 0 else 0.0,
            ms=elapsed / a.steps * 1e3,
            p50=float(active[:, 1].max()), p99=float(active[:, 2].max()),
            gpu_fps=(workers * a.steps * B / gpu_el) if gpu_el > 0 else None,
            gpu_busy=float(active[:, 4].max()), per_rank=per)

    h = agg(0)
    out = {
        "metric": cfg["metric"],
        "value": round(h["fps"], 2),
        "unit": "frames/s",
        "n_gpus": world if use_gpu else 0,
        "steps": a.steps,
        "warmup": a.warmup,
        "ms_per_step": round(h["ms"], 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": (round(h["fps"] / CPU_BASELINE_FPS, 2) if a.config == "mbv2" else None),
        "dtype": head["dtype"],
        "data": "synthetic video frames (videotestsrc pattern=snow), random-init weights",
        "p50_latency_ms": None if (fan or cfg.get("gather")) else round(h["p50"], 3),
        "p99_latency_ms": None if (fan or cfg.get("gather")) else round(h["p99"], 3),
        "gpu_event_fps": round(h["gpu_fps"], 2) if h["gpu_fps"] else None,
        "sink_fps": round(h["sink_fps"], 2),
        "timing": "value = frames / max(sink-arrival window, device-event window) of the same K batches",
        "gpu_invoke_ms_median": round(h["gpu_busy"], 4),
        "per_rank_fps": h["per_rank"],
        # the per-rank records above travelled through one all_gather on this process group
        "pg_world": pg_world,
        "pg_backend": pg_backend,
        "frames_per_step_per_gpu": B,
    }
    if "bf16" in results and head_label != "bf16":
        bb = results["bf16"]["batch"]
        b = agg(1, bb)
        out.update(value_bf16=round(b["fps"], 2), ms_per_step_bf16=round(b["ms"], 4), batch_bf16=bb,
                   p50_latency_ms_bf16=None if fan else round(b["p50"], 3),
                   gpu_event_fps_bf16=round(b["gpu_fps"], 2) if b["gpu_fps"] else None,
                   per_rank_fps_bf16=b["per_rank"])
    if lat_b1:
        n = len(runs)
        out.update(p50_latency_ms_b1=round(float(per_rank[:, n * 5].max()), 3),
                   p99_latency_ms_b1=round(float(per_rank[:, n * 5 + 1].max()), 3),
                   latency_b1_source=f"live camera, {a.latency_fps or cfg.get('lat_fps', 500)} frames/s, batch 1")
    if sweep:
        n = len(runs)
        base_i = n * 5 + 2
        pts = []
        for j, (sb, _) in enumerate(sweep):
            el = float(per_rank[:, base_i + 2 * j].max())
            pts.append({"batch": sb, "frames_per_s": round(workers * a.sweep_steps * sb / el, 1) if el > 0 else None,
                        "p50_latency_ms": round(float(per_rank[:, base_i + 2 * j + 1].max()), 3)})
        pts.append({"batch": B, "frames_per_s": round(h["fps"], 1), "p50_latency_ms": round(h["p50"], 3)})
        out["sweep"] = sorted(pts, key=lambda d: d["batch"])
    try:
        out["fp32_method"] = str(torch.ops.nnsx.f32_math())
    except Exception:  # noqa: BLE001
        out["fp32_method"] = None
    out.update({
        "preprocess": (f"tensor_transform (reference string) absorbed by tensor_filter into the model's uint8 "
                       f"input table ({head['absorbed']}: frames stay uint8)" if head["absorbed"]
                       else "tensor_transform element (own kernel, float32 frames into the model)"),
        "postprocess": (f"image_labeling argmax run by tensor_filter inside its hipGraph ({head['absorbed_dec']}: "
                        "int32 indices leave the model)" if head.get("absorbed_dec")
                        else "tensor_decoder's own argmax kernel"),
        "wall_s": round(sum(r["wall"] for r in results.values()), 3),
        "engine": a.engine,
        **({"lowered": head["lowered"]} if head.get("lowered") else {}),
        "numa_binding": numa,
        **({"allgather_bytes_published_rank0": head["gathered"]} if head["gathered"] is not None else {}),
        **({"mux_sets_rank0": head["mux_sets"]} if head.get("mux_sets") is not None else {}),
        # nnsx rank groups of rank 0 ("<data plane>:<members>[:bytes]") and the RCCL world they span
        "nnsx_groups_rank0": head["groups"],
        "rccl_world": max([int(v.split(":")[1]) for v in head["groups"].values() if v.startswith("rccl:")] or [0]),
        "config": {
            "model": cfg["desc"],
            "global_batch": B * world,
            "seq_len": 1,
            "parallelism": ((f"shared-ring fan-out 1->{world} (per-rank ingest)" if a.fan_transport == "shm" else
                             f"tensor_demux fan-out 1->{world} (RCCL p2p)") if fan else
                            f"branch-dp{world} + edge all-gather" if cfg.get("gather") else f"branch-dp{world}"),
            "pipeline": head["desc"],
        },
    })
    return out


def run_aux(a, nns, cfg, files, rank, world, dev, use_gpu, dist, workdir, out, torch, np):
    """Self-check + extra multi-rank configs after the headline (see main)."""
    import threading

    printed = threading.Lock()
    done = threading.Event()

    def expire():
        if done.is_set():
            return
        with printed:
            if rank == 0 and out is not None:
                out["aux_timeout"] = (f"the self-check / extra configs did not finish within {a.aux_timeout} s; "
                                      "the headline above is complete")
                print(json.dumps(out), flush=True)
            print(f"rank {rank}: auxiliary phase timed out after {a.aux_timeout} s", file=sys.stderr, flush=True)
            os._exit(0)

    watchdog = threading.Timer(a.aux_timeout, expire)
    watchdog.daemon = True
    watchdog.start()
    selfcheck, sc_error = None, None
    if not a.no_selfcheck:
        from nnstreamer_amd.parallel import selfcheck as sc

        if use_gpu:
            def arr(v, d=dev):
                return torch.as_tensor(v).cuda(d)
        else:
            def arr(v):
                return np.asarray(v)
        try:
            g = nns.Group("bench/selfcheck", rank, world, "", dev, a.comm_backend if use_gpu else "tcp",
                          a.selfcheck_timeout_ms)
            selfcheck = sc.run(g, rank, world, arr, scale=1.0 if use_gpu else 1.0 / 64,
                               recv_timeout_ms=a.selfcheck_timeout_ms)
            del g
        except Exception as e:  # noqa: BLE001
            sc_error = str(e)[:300]
        print(f"rank {rank}: rccl_selfcheck {selfcheck or sc_error}", file=sys.stderr, flush=True)
    extra = []
    if a.extra_configs and a.config == "mbv2":
        for name in [x for x in a.extra_configs.split(",") if x.strip()]:
            xb = (8 if name == "deeplab_fan" else 64) if use_gpu else 1
            xs_steps, xs_warm = (a.extra_steps, 5) if use_gpu else (2, 1)  # (CPU twin: plain models, short)
            try:
                xc = CONFIGS[name]
                xm = xc["model"] + "_fp32" if use_gpu else xc["model"].replace("_fused", "").replace("_lowres", "")
                xp = os.path.join(workdir, f"{xm}.pt")
                from nnstreamer_amd.models.export import export

                export(xm, xp, layout="nhwc")
                r = run_pipeline(a, nns, xc, xm, xp, files, xb, xs_steps, xs_warm, rank, world, dev, use_gpu, dist)
                r["steps"] = xs_steps
                extra.append((name, xb, r, None))
            except BaseException as e:  # noqa: BLE001 -- (SystemExit from run_pipeline included)
                extra.append((name, xb, None, str(e)[:300]))
    # [self-check flags, seconds, ok] + [elapsed or -1] per extra config
    vec = ([1.0 if (selfcheck or {}).get(k) else 0.0 for k in SC_KEYS]
           + [float((selfcheck or {}).get("seconds", 0.0)), 1.0 if selfcheck is not None else 0.0])
    vec += [max(r["elapsed"], r["gpu_elapsed"]) if r is not None else -1.0 for _, _, r, _ in extra]
    try:
        per_rank, _, _ = gather_rows(vec, world, dist, torch)
    except Exception as e:  # noqa: BLE001
        per_rank = None
        if out is not None:
            out["aux_error"] = f"gathering the auxiliary records failed: {str(e)[:200]}"
    done.set()
    watchdog.cancel()
    if rank != 0 or out is None or per_rank is None:
        return
    nk = len(SC_KEYS)
    if not a.no_selfcheck:
        ran = bool(float(per_rank[:, nk + 1].min()) > 0.5)
        flags = per_rank[:, :nk].min(0).values.tolist()
        rec = {**{k: bool(f > 0.5) for k, f in zip(SC_KEYS, flags)},
               "backend": (selfcheck or {}).get("backend"), "members": (selfcheck or {}).get("size"),
               "seconds_max": round(float(per_rank[:, nk].max()), 3),
               "payloads": ("64 MB all-gather / broadcast / scatter, 3-70 MB ragged all-gather, 48 MB p2p ring, "
                            "32 MB all-to-all" if use_gpu else "1/64 scale (CPU)")}
        rec["ok"] = ran and all(rec[k] for k in SC_KEYS)
        if selfcheck and selfcheck.get("errors"):
            rec["errors_rank0"] = selfcheck["errors"]
        if sc_error:
            rec["error_rank0"] = sc_error
        if not ran:
            rec["error"] = "the self-check did not run on every rank"
        out["rccl_selfcheck"] = rec
    if extra:
        xs = {}
        for j, (name, xb, r, e) in enumerate(extra):
            col = per_rank[:, nk + 2 + j]
            if float(col.min()) < 0 or r is None:
                xs[name] = {"frames_per_s": None, "batch": xb, "error_rank0": e or "failed on another rank"}
                continue
            el = float(col.max())
            xs[name] = {"frames_per_s": round(r["workers"] * r["steps"] * xb / el, 1) if el > 0 else None,
                        "batch": xb, "steps": r["steps"],
                        "rccl_world": max([int(v.split(":")[1]) for v in r["groups"].values()
                                           if v.startswith("rccl:")] or [0]),
                        "groups_rank0": r["groups"]}
            if name == "deeplab_fan":
                xs[name]["transport"] = a.fan_transport
        out["extra_configs"] = xs


if __name__ == "__main__":
    main()
