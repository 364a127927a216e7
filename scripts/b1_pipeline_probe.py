#!/usr/bin/env python3
"""Where does a batch-1 frame's latency go?  Builds bench.py's live-camera
batch-1 pipeline of a config and bisects it: the full chain, the chain without
the decoder, and source + converter alone, each reporting the sink's p50
arrival latency (frame PTS -> sink, device-synced) and the filter's device
time per invoke.

    python scripts/b1_pipeline_probe.py deeplab [fps] [frames]
"""
import os
import sys
import tempfile

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))

import numpy as np  # noqa: E402

import bench  # noqa: E402
import nnstreamer_amd as nns  # noqa: E402
from nnstreamer_amd.models.export import export, write_labels  # noqa: E402


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "deeplab"
    fps = int(sys.argv[2]) if len(sys.argv) > 2 else 100
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 120
    cfg = bench.CONFIGS[name]
    S = cfg["size"]
    work = tempfile.mkdtemp()
    model_name = cfg["model"] + "_fp32"
    path = export(model_name, os.path.join(work, f"{model_name}.pt"), layout="nhwc")
    from nnstreamer_amd.models.posenet import write_pose_labels
    from nnstreamer_amd.models.ssd import write_box_priors, write_coco_labels

    files = dict(labels=write_labels(os.path.join(work, "labels.txt")),
                 coco=write_coco_labels(os.path.join(work, "coco.txt")),
                 priors=write_box_priors(os.path.join(work, "priors.txt")),
                 pose=write_pose_labels(os.path.join(work, "pose17.txt")))
    src = (f"videotestsrc num-buffers={n} pattern=snow pool-size=16 is-live=true "
           f"! video/x-raw,format=RGB,width={S},height={S},framerate={fps}/1 ")
    conv = "! tensor_converter frames-per-tensor=1 device=0 "
    norm = f"! tensor_transform name=norm mode=arithmetic option={cfg['norm']} "
    filt = (f"! tensor_filter name=filt framework=pytorch model={path} input=3:{S}:{S}:1 inputtype=float32 "
            "absorb-transform=true accelerator=true:gpu device=0 custom=hipgraph:true latency=1 ")
    dec = "! " + cfg["decoder"].format(**files) + " "
    variants = {
        "full": src + conv + norm + filt + dec,
        "no-decoder": src + conv + norm + filt,
        "converter-only": src + conv,
    }
    for tag, desc in variants.items():
        p = nns.parse_launch(desc + "! tensor_sink name=sink")
        sink = p.get_by_name("sink")
        sink.set_property("emit-signal", "false")
        sink.set_property("sync-device", "true")
        sink.set_property("stats-every", "1")
        p.run(timeout=300)
        recs = [tuple(int(v) for v in e.split(":")) for e in sink.get_property("stats").split(",") if e]
        lat = np.array([r[1] / 1e6 for r in recs[n // 4:] if r[1] >= 0])
        f = p.get_by_name("filt")
        dev = f.get_property("latency") if f is not None else "-"
        p.stop()
        print(f"{name} {tag:15s} {fps} fps: sink p50 {np.median(lat):.3f} ms p99 {np.percentile(lat, 99):.3f} ms "
              f"({len(lat)} frames); filter device latency {dev} us")


if __name__ == "__main__":
    main()
