#!/usr/bin/env python3
"""Config-4 ingest through a shared frame ring: a camera
process renders N cameras' 513 x 513 RGB rings into named POSIX shared memory
(videotestsrc pool-shm) and publishes each camera with edgesink
connect-type=SHM; THIS process -- a second one, the way every rank of
bench.py's deeplab_fan is its own process -- subscribes (edgesrc
connect-type=SHM), receives frames as references into its hipHostRegister'ed
mapping of the same segments, and its tensor_converter device=0 DMAs each
batch straight from the shared ring into HBM (one DMA per run of adjacent ring
frames) -> tensor_sink sync-device=true.  Reported: frames/s and packed bytes/s
reaching HBM over the steady state (sink arrival stamps from the 4th batch to
the last).  Reference: gsttensor_demux.c:469-556 (hand-out by reference).

    python scripts/shm_ingest.py [cameras] [batches...]     (default 8 cameras, batches 8 32)
"""
import os
import subprocess
import sys
import textwrap
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

W = 4  # warm-up batches per camera outside the timed window


def producer(cams, B, n, S, tag):
    frame = S * S * 3
    pool = max(2 * B, min(n * B, -(-64 * 2**20 // frame)))  # 64 MiB ring per camera
    desc = " ".join(f"videotestsrc num-buffers={n * B} pattern=snow pool-size={pool} pool-shm=nnsx-ingest-{tag}-{r} "
                    f"! video/x-raw,format=RGB,width={S},height={S},framerate=0/1 "
                    f"! edgesink name=e{r} port=0 connect-type=SHM wait-connection=1" for r in range(cams))
    code = textwrap.dedent(f"""
        import sys, time
        sys.path.insert(0, {ROOT!r})
        import nnstreamer_amd as nns
        p = nns.parse_launch({desc!r})
        p.set_state("playing")
        ports = []
        for r in range({cams}):
            while int(p.get_by_name(f"e{{r}}").get_property("port")) == 0:
                time.sleep(0.01)
            ports.append(p.get_by_name(f"e{{r}}").get_property("port"))
        print(" ".join(str(x) for x in ports), flush=True)
        msg = p.wait(900)
        print(msg[0] if msg else "timeout", flush=True)
        sys.stdin.readline()
        p.stop()
    """)
    # the camera process never touches a GPU (its ring is plain shared memory)
    env = dict(os.environ, HIP_VISIBLE_DEVICES="")
    return subprocess.Popen([sys.executable, "-c", code], stdin=subprocess.PIPE, stdout=subprocess.PIPE, text=True,
                            env=env)


def run(nns, torch, cams, B, n, S=513):
    frame = S * S * 3
    proc = producer(cams, B, n, S, f"{os.getpid()}-{B}-{n}")
    try:
        ports = [int(x) for x in proc.stdout.readline().split()]
        assert len(ports) == cams, ports
        desc = " ".join(f"edgesrc name=src{r} dest-host=127.0.0.1 dest-port={ports[r]} connect-type=SHM "
                        f"! tensor_converter frames-per-tensor={B} device=0 ! queue max-size-buffers=2 "
                        f"! tensor_sink name=s{r} sync-device=true" for r in range(cams))
        p = nns.parse_launch(desc)
        for r in range(cams):
            p.get_by_name(f"s{r}").set_property("emit-signal", "false")
            p.get_by_name(f"s{r}").set_property("stats-every", "1")
        torch.cuda.synchronize()
        t = time.perf_counter()
        p.run(timeout=900)
        torch.cuda.synchronize()
        wall = time.perf_counter() - t
        arr, refs = [], 0
        for r in range(cams):
            st = p.get_by_name(f"s{r}").get_property("stats")
            arr.append([int(e.split(":")[0]) / 1e9 for e in st.split(",") if e])
            refs += int(p.get_by_name(f"src{r}").get_property("shm-blobs"))
        p.stop()
        status = proc.stdout.readline().split()
    finally:
        try:
            proc.stdin.write("\n")
            proc.stdin.flush()
        except BrokenPipeError:
            pass
        proc.wait(timeout=60)
    t0 = min(a[W - 1] for a in arr)
    t1 = max(a[-1] for a in arr)
    return t1 - t0, [len(a) for a in arr], frame, wall, refs, status


def main():
    cams = int(sys.argv[1]) if len(sys.argv) > 1 else 8
    batches = [int(x) for x in sys.argv[2:]] or [8, 32]
    import torch

    import nnstreamer_amd as nns

    print(f"# {cams} cameras 513x513 RGB in shared rings (camera process) -> edgesrc connect-type=SHM -> "
          f"tensor_converter device=0 -> tensor_sink sync-device in a second process (1 x "
          f"{torch.cuda.get_device_name(0)})")
    for B in batches:
        n = max(40, 1920 // B)  # batches per camera
        run(nns, torch, cams, B, W + 1)  # warm-up: code objects
        el, got, frame, wall, refs, status = run(nns, torch, cams, B, n)
        frames = cams * (n - W) * B
        print(f"batch {B:3d}: {frames} frames in {el * 1e3:8.1f} ms  {frames / el:9.0f} frames/s  "
              f"{frames * frame / el / 1e9:6.2f} GB/s into HBM  (sink buffers per camera {sorted(set(got))}; "
              f"frames received by reference {refs} of {cams * n * B}; camera process {' '.join(status)}; "
              f"whole run incl. start-up {wall * 1e3:.0f} ms)", flush=True)


if __name__ == "__main__":
    main()
