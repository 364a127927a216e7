"""RCCL data plane with one process per GPU (BASELINE.json configs 4 and 5):
every collective and p2p call of comm::Group over RCCL/xGMI between N =
min(#GPUs, 8) ranks, payload values checked on every member, plus the two
multi-rank bench configs (tensor_demux -> edgesink RCCL fan-out; edge all-gather -> tensor_mux).
Reference fan-out / fan-in points: tensor_query_client.c:657-746,
edge_sink.c:305-345, gsttensor_demux.c:469-556.  Skipped below 2 GPUs (the
1-GPU pool); the CPU twin is tests/test_rank_collectives.py."""
import json
import os
import subprocess
import sys

import pytest

from rank_util import ROOT, check, check_big, run_ranks

pytestmark = pytest.mark.gpu


def _ngpu():
    import torch

    return torch.cuda.device_count()


needs2 = pytest.mark.skipif(_ngpu() < 2, reason="needs >= 2 GPUs (one rank per GPU)")


@needs2
def test_group_collectives_rccl():
    world = min(_ngpu(), 8)
    res = run_ranks(world, list(range(world)), "rccl")
    check(res, world, "rccl")
    for x in res:  # payloads stayed in HBM: received blobs are device memories
        assert all(x["ag_on_device"]), x


@needs2
def test_group_collectives_rccl_frame_sized():
    """Frame-sized payloads over RCCL between GPUs (_rank_worker.py big): 64 MB
    and 3-70 MB ragged all-gathers, 64 MB broadcast / scatter, a send-first ring
    of 48 MB messages and an all-to-all 32 MB exchange -- the patterns that hang
    when every rank's sends and receives share one comm stream."""
    world = min(_ngpu(), 8)
    res = run_ranks(world, list(range(world)), "rccl", timeout=300, mode="big")
    check_big(res, world, "rccl")


@needs2
@pytest.mark.parametrize("cfg", ["posenet_multi", "deeplab_fan"])
def test_bench_multi_rank_configs(cfg):
    n = 2 if cfg == "posenet_multi" else 3
    if _ngpu() < n:
        pytest.skip(f"{cfg} needs {n} GPUs")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--config", cfg,
                        "--steps", "3", "--warmup", "1", "--batch", "4", "--latency-frames", "0", "--sweep", "",
                        "--comm-backend", "rccl"],
                       capture_output=True, text=True, timeout=600)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert rec["n_gpus"] == n and rec["value"] > 0, rec
    if cfg == "posenet_multi":
        assert int(rec.get("allgather_bytes_published_rank0", 0)) > 0, rec
        assert rec.get("mux_sets_rank0") == 4, rec  # every batch a full N-camera set
    else:
        assert "tensor_demux" in rec["config"]["pipeline"], rec


@needs2
def test_bench_headline_selfcheck_and_extra_configs():
    """The driver's scaling command shape at N = min(#GPUs, 8): bench.py's
    rccl_selfcheck (every comm::Group operation over RCCL on frame-sized
    payloads) and the config-4 / config-5 passes after the headline."""
    n = min(_ngpu(), 8)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n), "--steps", "5",
                        "--warmup", "2", "--latency-frames", "0", "--sweep", ""],
                       capture_output=True, text=True, timeout=900)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
    rec = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    sc = rec["rccl_selfcheck"]
    assert sc["backend"] == "rccl" and sc["members"] == n, sc
    assert all(sc[k] for k in ("allgather", "allgather_ragged", "broadcast", "scatter", "p2p_ring", "p2p_exchange"))
    xs = rec["extra_configs"]
    assert xs["deeplab_fan"]["rccl_world"] == 2 and xs["posenet_multi"]["rccl_world"] == n, xs
