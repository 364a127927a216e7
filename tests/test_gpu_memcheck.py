"""Device-memory lifetime: deterministic regression tests for the three
cross-stream races fixed in rounds 3-4, and the NNSX_MEM_CHECK debug mode.

Each native case (runtime/selftest.cc) holds a stream busy with a bounded spin
kernel so a copy or a read is still queued when the Memory owning its source is
released; the storage is then handed out again with other bytes.  An early
free shows every time:
  * pageable_h2d / pinned_h2d -- 7ba8684 (a pageable frame freed while its H2D
    copy was queued; the copy read the next frame);
  * mirror_other_stream -- ee80b24 (a replay lane read a recycled device mirror
    of a host frame);
  * device_reader -- a device block released while another stream reads it.
The ticket case pins 0e16787 (concurrent replays of a block shared the model's
ticket buffer): under a shared device scope -- what replay lanes set -- the
fused block must not use the ticket buffer at all, so poisoned tickets do not
change its result.  Reference analogue of the lifetime rules: the GLib lock /
condvar handoff of gst/nnstreamer/elements/gsttensor_repo.c:165-326."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("case", ["pageable_h2d", "pinned_h2d", "mirror_other_stream", "device_reader"])
def test_memory_lifetime_selftest(nns, case):
    from nnstreamer_amd import _C

    msg = _C.memory_selftest(case, 0)
    assert msg == "", msg


@pytest.mark.parametrize("case,mutation", [("pinned_h2d", 1), ("mirror_other_stream", 2)])
def test_memory_selftest_fails_without_its_fix(nns, case, mutation, monkeypatch):
    """each lifetime case must catch the bug its fix removed.
    The fix is undone at run time (Memory::set_test_mutation: 1 = a host
    source's H2D copy is not recorded as a use -- the rule 7ba8684 extended from
    pinned to pageable sources; 2 = a reader of a host memory does not hold its
    device mirror, before ee80b24) and the case must then fail; with the fix in
    place it passes again.  Output: profiles/r6_lifetime_fail_on_parent.txt."""
    from nnstreamer_amd import _C

    monkeypatch.setenv("NNSX_SELFTEST_VERBOSE", "1")  # (per size: how long map_device blocked)
    prev = _C.memory_test_mutation(mutation)
    try:
        broken = _C.memory_selftest(case, 0)
    finally:
        _C.memory_test_mutation(prev)
    torch.cuda.synchronize()
    print(f"{case} with fix undone ({mutation}): {broken!r}")
    assert broken != "", f"{case} did not notice the undone fix"
    assert _C.memory_selftest(case, 0) == ""


def test_pageable_h2d_without_its_fix_on_this_runtime(nns, monkeypatch, capfd):
    """The pageable half of 7ba8684 on this HIP runtime (ROCm 7.2): measured, a
    pageable H2D of <= 1 MB returns at once with the source already staged (the
    frame can be recycled without harm) and an 8 MB one blocks the host until
    the copy ran -- so with the fix undone the case still passes here.  The
    test pins that measurement (each size either intact with the host blocked
    for the spin, or intact after an immediate return) so that a runtime which
    starts reading pageable sources late shows up as a failure of
    pageable_h2d, where the fix then matters."""
    from nnstreamer_amd import _C

    monkeypatch.setenv("NNSX_SELFTEST_VERBOSE", "1")
    prev = _C.memory_test_mutation(1)
    try:
        broken = _C.memory_selftest("pageable_h2d", 0)
    finally:
        _C.memory_test_mutation(prev)
    err = capfd.readouterr().err
    print(err)
    lines = [x for x in err.splitlines() if x.startswith("pageable_h2d[")]
    assert len(lines) == 4, err
    assert broken == "" and all("bytes intact" in x for x in lines), err
    assert _C.memory_selftest("pageable_h2d", 0) == ""


@pytest.mark.parametrize("H,cin,hid,cout,stride,B", [(7, 160, 960, 160, 1, 8), (14, 96, 576, 160, 2, 2),
                                                     (14, 64, 384, 64, 1, 1)])
def test_shared_device_scope_ignores_tickets(nns, H, cin, hid, cout, stride, B):
    """0e16787: under a shared device scope (replay lanes, concurrent
    instances) the fused block adds its hidden parts without the ticket buffer:
    a garbage-filled buffer leaves the result bit for bit unchanged"""
    torch.manual_seed(H + cin + B)
    x = torch.randn(B, H, H, cin, device="cuda")
    we = torch.randn(hid, cin, device="cuda") / cin ** 0.5
    be = torch.randn(hid, device="cuda") * 0.1
    wd = torch.randn(9, hid, device="cuda") / 3
    bd = torch.randn(hid, device="cuda") * 0.1
    wp = torch.randn(cout, hid, device="cuda") / hid ** 0.5
    bp = torch.randn(cout, device="cuda") * 0.1
    res = stride == 1 and cin == cout
    ref = torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, res, 1, None)
    bad = torch.full((768,), 0x3A3A3A3A, dtype=torch.int32, device="cuda")  # no launch ever leaves this state
    prev = torch.ops.nnsx.set_device_shared(True)
    try:
        y = torch.ops.nnsx.ir_block(x, we, be, wd, bd, wp, bp, stride, cout, True, res, 1, bad)
        torch.cuda.synchronize()
    finally:
        torch.ops.nnsx.set_device_shared(prev)
    assert torch.equal(y, ref)
    assert int((bad != 0x3A3A3A3A).sum()) == 0  # untouched


def test_memcheck_mode_pipeline(nns, workdir, labels):
    """The benched pipeline shape in a child process with NNSX_MEM_CHECK=1:
    released device blocks are poisoned (NaN pattern), pooled blocks are checked
    for writes after release on every hand-out, maps of released memories
    throw.  Labels must equal the run without the checker."""
    import os
    import subprocess
    import sys

    here = os.path.dirname(os.path.abspath(__file__))
    code = f"""
import os, sys
sys.path.insert(0, {os.path.dirname(here)!r})
import nnstreamer_amd as nns
from nnstreamer_amd import _C
from nnstreamer_amd.models.export import export
model = export("mobilenet_v2_fused_fp32", os.path.join({workdir!r}, "mbv2_memcheck.pt"), layout="nhwc")
out = []
for B, lanes in ((8, 3), (16, 1)):
    p = nns.parse_launch(
        f"videotestsrc num-buffers={{B * 6}} pattern=snow pool-size=64 "
        "! video/x-raw,format=RGB,width=224,height=224,framerate=0/1 "
        f"! tensor_converter frames-per-tensor={{B}} device=0 ! queue max-size-buffers=2 "
        "! tensor_transform mode=arithmetic option=typecast:float32,add:-127.5,div:127.5 "
        f"! tensor_filter framework=pytorch model={{model}} input=3:224:224:{{B}} inputtype=float32 "
        f"accelerator=true:gpu device=0 custom=hipgraph:true,lanes:{{lanes}} ! queue max-size-buffers=2 "
        f"! tensor_decoder mode=image_labeling option1={labels!r} ! tensor_sink name=sink")
    p.get_by_name("sink").connect("new-data", lambda b: out.append(b.memory(0).bytes().decode()))
    p.run(timeout=240)
    p.stop()
_C.memory_drain_deferred()
print("CHECK", _C.memory_check_enabled())
print("LABELS", repr(out))
"""
    runs = {}
    for on in ("1", "0"):
        r = subprocess.run([sys.executable, "-c", code], env=dict(os.environ, NNSX_MEM_CHECK=on),
                           capture_output=True, text=True, timeout=400)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-3000:]
        assert f"CHECK {on == '1'}" in r.stdout
        runs[on] = [x for x in r.stdout.splitlines() if x.startswith("LABELS")][0]
    assert runs["1"] == runs["0"]
