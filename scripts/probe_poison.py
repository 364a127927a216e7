"""Which released block a stale read saw (NNSX_MEM_CHECK=1): host poison 0x7FBADBAD
vs released-device-block poison 0x7FDE7ADE, in tests/test_gpu_filter_graph.py's
static-outputs pipeline (appsrc).  Prints the frames whose output is not the
expected value, with the raw bits of their first element."""
import os
import sys
import tempfile
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import numpy as np  # noqa: E402
import torch  # noqa: E402

import nnstreamer_amd as nns  # noqa: E402


class _Scale(torch.nn.Module):
    def forward(self, x):
        return x * 2.0 + 1.0


def main():
    m = os.path.join(tempfile.mkdtemp(), "m.pt")
    torch.jit.script(_Scale()).save(m)
    n = 3 * 16 * 8
    frames = [np.full(n, i % 251, np.uint8) for i in range(40)]
    caps = "other/tensors,format=static,num_tensors=1,dimensions=3:16:8:1,types=uint8,framerate=0/1"
    p = nns.parse_launch(
        f"appsrc name=src caps={caps} ! tensor_transform mode=typecast option=float32 ! tensor_filter framework=pytorch "
        f"model={m} accelerator=true:gpu device=0 custom=hipgraph:true ! queue max-size-buffers=32 ! tensor_sink name=s")
    got = []

    def on_data(buf):
        if len(got) < 20:
            time.sleep(0.01)
        got.append(buf.memory(0).numpy("float32").copy())

    p.get_by_name("s").connect("new-data", on_data)
    p.set_state("playing")
    src = p.get_by_name("src")
    for i, f in enumerate(frames):
        src.push_buffer(f, pts=i)
    src.end_of_stream()
    p.wait(60)
    p.stop()
    bad = 0
    for i, g in enumerate(got):
        want = 2.0 * (i % 251) + 1.0
        if not np.all(g == want):
            bad += 1
            nanbits = {hex(int(v)) for v in g.view(np.uint32)[np.isnan(g)]}
            print(f"frame {i}: {np.isnan(g).sum()} NaN (bits {sorted(nanbits)}), first {g[0]}, want {want}")
    print(f"{bad} bad frames of {len(got)}")


if __name__ == "__main__":
    main()
