"""Batch-1 latency breakdown of the headline pipeline (fp32 fused MobileNetV2,
live 500 fps camera, whole chain in the source thread -- bench.py's
p50_latency_ms_b1 run) with the proctime / interlatency tracers on.

    python scripts/b1_latency_probe.py [frames] [fps]

Prints the sink latency percentiles (source PTS -> sink arrival) and each
element's processing time, so the device time of the model can be told apart
from the host path around it.
"""
import json
import os
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("NNSX_TRACERS", "proctime;interlatency")
import numpy as np  # noqa: E402

import nnstreamer_amd as nns  # noqa: E402
from nnstreamer_amd.models.export import export, write_labels  # noqa: E402

frames = int(sys.argv[1]) if len(sys.argv) > 1 else 300
fps = int(sys.argv[2]) if len(sys.argv) > 2 else 500
d = tempfile.mkdtemp(prefix="nnsx_b1_")
model = export("mobilenet_v2_fused_fp32", os.path.join(d, "m.pt"), layout="nhwc")
labels = write_labels(os.path.join(d, "labels.txt"))
desc = (f"videotestsrc num-buffers={frames} pattern=snow pool-size=64 is-live=true "
        f"! video/x-raw,format=RGB,width=224,height=224,framerate={fps}/1 "
        "! tensor_converter name=conv frames-per-tensor=1 device=0 "
        f"! tensor_filter name=filt framework=pytorch model={model} input=3:224:224:1 inputtype=uint8 "
        "accelerator=true:gpu device=0 custom=hipgraph:true device-stats=true "
        f"! tensor_decoder name=dec mode=image_labeling option1={labels} ! tensor_sink name=sink")
p = nns.parse_launch(desc)
sink = p.get_by_name("sink")
sink.set_property("emit-signal", "false")
sink.set_property("sync-device", "true")
sink.set_property("stats-every", "1")
nns.tracer_reset()
p.run(timeout=600)
recs = [tuple(int(v) for v in e.split(":")) for e in sink.get_property("stats").split(",") if e]
filt = p.get_by_name("filt")
ds = [tuple(int(v) for v in e.split(":")) for e in filt.get_property("device-stamps").split(",") if e]
p.stop()
w = max(10, frames // 5)
lat = np.array([r[1] for r in recs[w:] if r[1] >= 0]) / 1e3
dev = np.array([x[1] for x in ds[w:]]) / 1e3
out = {"frames": frames, "fps": fps, "latency_us": {"p50": float(np.percentile(lat, 50)),
                                                      "p99": float(np.percentile(lat, 99)),
                                                      "min": float(lat.min())},
       "filter_device_us_median": float(np.median(dev)) if dev.size else None,
       "tracer": json.loads(nns.tracer_report())}
print(json.dumps(out, indent=1))
