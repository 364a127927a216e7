"""Rank-group collectives and p2p across processes on CPU (tcp backend): the
same member logic the RCCL data plane runs on GPUs (tests/test_gpu_rccl_ranks.py):
uniform / ragged all-gather, broadcast, scatter, send/recv ring, byte counters."""
import pytest

from rank_util import check, check_big, run_ranks


@pytest.mark.parametrize("world", [2, 3])
def test_group_collectives_tcp(world):
    res = run_ranks(world, [-1] * world, "tcp")
    check(res, world, "tcp")


@pytest.mark.parametrize("world", [2, 3])
def test_group_collectives_tcp_frame_sized(world):
    """64 MB uniform / 3-70 MB ragged all-gather, 64 MB broadcast and scatter,
    a send-first ring of 48 MB messages and an all-to-all 32 MB exchange."""
    res = run_ranks(world, [-1] * world, "tcp", timeout=300, mode="big")
    check_big(res, world, "tcp")
