"""bench.py launcher contract (CPU): `--gpus N` spawns N rank processes by
itself, all-gathers the per-rank records and reports the whole-job value."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, env=None, timeout=600):
    e = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        e.pop(k, None)
    e.update(env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *args], capture_output=True, text=True,
                          env=e, timeout=timeout, cwd=ROOT)


def test_bench_spawns_ranks_and_gathers():
    r = _run(["--cpu", "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "1", "--latency-frames", "0"])
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["pg_world"] == 2 and out["pg_backend"] == "gloo"
    assert len(out["per_rank_fps"]) == 2 and all(v > 0 for v in out["per_rank_fps"])
    assert out["config"]["global_batch"] == 2 and out["config"]["parallelism"] == "branch-dp2"
    assert out["steps"] == 2 and out["warmup"] == 1 and out["value"] > 0


def test_bench_refuses_world_mismatch():
    r = _run(["--cpu", "--gpus", "2", "--steps", "1", "--warmup", "1", "--batch", "1"],
             env={"WORLD_SIZE": "1", "RANK": "0", "LOCAL_RANK": "0"})
    assert r.returncode != 0
    assert "WORLD_SIZE=1" in (r.stderr + r.stdout)


@pytest.mark.parametrize("fan", ["shm", "rccl"])
def test_bench_three_ranks_selfcheck_and_extra_configs(fan):
    """WORLD_SIZE > 1 (the driver's scaling run): after the headline every
    comm::Group operation is checked on every rank (rccl_selfcheck; tcp data
    plane on CPU, RCCL on GPUs) and short passes of the multi-rank configs 4
    and 5 report their frames/s and groups -- all outside the timed region,
    well inside a minute.  Config 4 with both fan-out transports: shared frame
    rings (each worker ingests its own camera, the default) and tensor_demux +
    scatter over the rank group."""
    import time

    t0 = time.time()
    r = _run(["--cpu", "--gpus", "3", "--steps", "2", "--warmup", "1", "--batch", "1", "--latency-frames", "0",
              "--sweep", "", "--fan-transport", fan])
    assert r.returncode == 0, r.stderr[-3000:]
    assert time.time() - t0 < 120
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    sc = out["rccl_selfcheck"]
    for k in ("allgather", "allgather_ragged", "broadcast", "scatter", "p2p_ring", "p2p_exchange"):
        assert sc[k] is True, sc
    assert sc["ok"] is True
    assert sc["members"] == 3 and sc["backend"] == "tcp"
    xs = out["extra_configs"]
    assert set(xs) == {"deeplab_fan", "posenet_multi"}
    assert all(v["frames_per_s"] and v["frames_per_s"] > 0 for v in xs.values()), xs
    assert xs["deeplab_fan"]["transport"] == fan
    assert ("edge_fan1" in xs["deeplab_fan"]["groups_rank0"]) == (fan == "rccl")
    assert "edge_allgather" in xs["posenet_multi"]["groups_rank0"]
    assert out["fp32_method"] in ("x3", "fp32")
    assert out["value"] > 0 and out["n_gpus"] == 0


def test_bench_selfcheck_fault_never_blocks_headline():
    """One member skips the broadcast (NNSX_SELFCHECK_FAULT): the other members'
    broadcast fails within the self-check's deadline with an error naming the
    mismatch / the missing member, later collectives fail fast, p2p still
    checks out, and the headline JSON is printed with exit code 0."""
    import time

    t0 = time.time()
    r = _run(["--cpu", "--gpus", "3", "--steps", "2", "--warmup", "1", "--batch", "1", "--latency-frames", "0",
              "--sweep", "", "--extra-configs", "", "--selfcheck-timeout-ms", "10000"],
             env={"NNSX_SELFCHECK_FAULT": "1:broadcast"})
    assert r.returncode == 0, r.stderr[-3000:]
    assert time.time() - t0 < 150
    out = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert out["value"] > 0 and out["pg_world"] == 3
    sc = out["rccl_selfcheck"]
    assert sc["ok"] is False and sc["broadcast"] is False, sc
    assert sc["allgather"] is True and sc["allgather_ragged"] is True, sc
    assert sc["p2p_ring"] is True and sc["p2p_exchange"] is True, sc
    err = sc["errors_rank0"]["broadcast"]
    assert "member 1" in err or "member(s) 1" in err, err
    assert sc["seconds_max"] < 60


def test_bench_aux_watchdog_prints_headline(tmp_path):
    """A hung auxiliary phase (watchdog at 1 s while the extra configs run)
    still yields the headline line and exit code 0 on every rank."""
    r = _run(["--cpu", "--gpus", "2", "--steps", "2", "--warmup", "1", "--batch", "1", "--latency-frames", "0",
              "--sweep", "", "--aux-timeout", "1"])
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, r.stdout
    out = json.loads(lines[0])
    assert out["value"] > 0 and "aux_timeout" in out
