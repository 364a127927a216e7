"""Shared frame ring across processes on a GPU: a camera
process renders its ring into POSIX shared memory (videotestsrc pool-shm) and
publishes it with edgesink connect-type=SHM; this process maps the segment
(hipHostRegister'ed), receives the frames as references and its
tensor_converter device=0 DMAs the batches from the shared ring into HBM.
Bytes equal the camera's; every frame arrived by reference.  Rate:
scripts/shm_ingest.py -> profiles/r6_shared_ring_ingest.txt.  Reference:
gsttensor_demux.c:469-556 (hand-out by reference)."""
import os
import subprocess
import sys
import textwrap

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_shm_ring_to_hbm_in_second_process(nns, tmp_path):
    name = f"nnsx-gtest-{os.getpid()}"
    script = tmp_path / "cam.py"
    script.write_text(textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        import nnstreamer_amd as nns
        p = nns.parse_launch("videotestsrc num-buffers=32 pattern=snow pool-size=8 pool-shm={name} "
                             "! video/x-raw,format=RGB,width=513,height=513,framerate=0/1 "
                             "! edgesink name=es port=0 connect-type=SHM wait-connection=1")
        p.set_state("playing")
        while int(p.get_by_name("es").get_property("port")) == 0:
            time.sleep(0.01)
        print(p.get_by_name("es").get_property("port"), flush=True)
        msg = p.wait(120)
        print(msg[0] if msg else "timeout", flush=True)
        sys.stdin.readline()
        p.stop()
    """))
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")  # the camera process has no GPU
    proc = subprocess.Popen([sys.executable, str(script)], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                            env=env)
    out = []
    try:
        port = int(proc.stdout.readline())
        s = nns.parse_launch(f"edgesrc name=src dest-host=127.0.0.1 dest-port={port} connect-type=SHM "
                             "! tensor_converter frames-per-tensor=4 device=0 ! tensor_sink name=sink")
        s.get_by_name("sink").connect("new-data", lambda b: out.append(
            (b.memory(0).on_device, np.frombuffer(b.memory(0).bytes(), np.uint8).copy())))
        s.set_state("playing")
        msg = s.wait(120)
        assert msg and msg[0] == "eos", s.messages()
        refs = int(s.get_by_name("src").get_property("shm-blobs"))
        s.stop()
        assert proc.stdout.readline().strip() == "eos"
    finally:
        proc.stdin.write("\n")
        proc.stdin.flush()
        proc.wait(timeout=60)
    assert len(out) == 8 and refs == 32, (len(out), refs)
    assert all(dev for dev, _ in out)
    ref = nns.parse_launch("videotestsrc num-buffers=8 pattern=snow pool-size=8 "
                           "! video/x-raw,format=RGB,width=513,height=513,framerate=0/1 ! tensor_converter "
                           "! tensor_sink name=sink")
    want = []
    ref.get_by_name("sink").connect("new-data", lambda b: want.append(b.memory(0).numpy("uint8").copy()))
    ref.run(timeout=60)
    got = np.concatenate([a.reshape(4, -1) for _, a in out])
    for i in range(32):
        np.testing.assert_array_equal(got[i], want[i % 8].ravel())
