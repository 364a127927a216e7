#!/usr/bin/env python3
"""tensor_converter batch-1 latency probe: live camera -> converter (device=0)
-> sink (device-synced), p50 arrival latency per frame for several frame
widths (513 / 257: RGB rows padded to 4 bytes; 512 / 224: packed)."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

import nnstreamer_amd as nns  # noqa: E402

fps, n = 100, 150
for w in (513, 512, 257, 256, 224):
    desc = (f"videotestsrc num-buffers={n} pattern=snow pool-size=16 is-live=true "
            f"! video/x-raw,format=RGB,width={w},height={w},framerate={fps}/1 "
            "! tensor_converter frames-per-tensor=1 device=0 ! tensor_sink name=sink")
    p = nns.parse_launch(desc)
    s = p.get_by_name("sink")
    s.set_property("emit-signal", "false")
    s.set_property("sync-device", "true")
    s.set_property("stats-every", "1")
    p.run(timeout=120)
    lat = np.array([int(e.split(":")[1]) / 1e6 for e in s.get_property("stats").split(",") if e][n // 4:])
    p.stop()
    print(f"width {w}: p50 {np.median(lat):.3f} ms  p99 {np.percentile(lat, 99):.3f} ms "
          f"(padded rows: {(w * 3) % 4 != 0}) {os.environ.get('NNSX_CONVERTER_PADDED_DMA', '')}")
