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


@pytest.mark.parametrize("mode", ["flush", "credit"])
def test_group_queued_sends_delivered(mode):
    """send() is asynchronous (the engine carries it in its next round).  A
    member queues 20 messages -- 2.5 credit windows -- for a member that only
    starts receiving a second later.  flush: the sender closes the group at
    once; the orderly close still delivers every message, in order (before the
    fix it dropped the queue -- under load test_group_collectives_tcp[3] lost
    its ring messages this way).  credit: the sender stays; once it has used a
    full window the receiver's consumption must trigger the round that grants
    it more (before the fix nothing did: a deadlock until the receive timed
    out)."""
    res = run_ranks(2, [-1, -1], "tcp", mode=mode)
    got = [r for r in res if r["rank"] == 0][0]["flush"]
    assert got == [[1, k, float(k)] for k in range(20)], got
    if mode == "credit":
        assert [r for r in res if r["rank"] == 1][0]["ack"] == 99
