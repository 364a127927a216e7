"""nnsx-launch: run a pipeline description like gst-launch-1.0.

    python -m nnstreamer_amd.tools.launch "videotestsrc num-buffers=10 ! \\
        tensor_converter ! tensor_sink"

Exit status 0 on EOS, 1 on an error message, 2 on a parse/state failure,
3 on timeout.  ``-v`` prints the negotiated caps of every pad, ``-m`` every
bus message, ``--dot FILE`` writes the graph (GST_DEBUG_DUMP_DOT_DIR style).
"""
from __future__ import annotations

import argparse
import sys
import time


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="nnsx-launch", description=__doc__,
                                 formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("pipeline", nargs="+", help="pipeline description (joined with spaces)")
    ap.add_argument("-v", "--verbose", action="store_true", help="print negotiated caps")
    ap.add_argument("-m", "--messages", action="store_true", help="print every bus message")
    ap.add_argument("-t", "--timeout", type=float, default=0.0, help="seconds before giving up (0 = none)")
    ap.add_argument("--dot", default="", help="write the pipeline graph (graphviz) here")
    ap.add_argument("--debug", default="", help="log threshold, e.g. 'warning' or '4'")
    a = ap.parse_args(argv)

    import nnstreamer_amd as nns

    if a.debug:
        nns.set_debug(a.debug)
    desc = " ".join(a.pipeline)
    try:
        p = nns.parse_launch(desc)
    except Exception as e:  # noqa: BLE001
        print(f"ERROR: pipeline could not be constructed: {e}", file=sys.stderr)
        return 2
    t0 = time.perf_counter()
    try:
        p.set_state("playing")
    except Exception as e:  # noqa: BLE001
        print(f"ERROR: pipeline doesn't want to play: {e}", file=sys.stderr)
        return 2
    print("Setting pipeline to PLAYING ...")
    msg = p.wait(a.timeout if a.timeout > 0 else 1e9)
    elapsed = time.perf_counter() - t0
    if a.verbose:
        for e in p.elements():
            for pad in e.pad_names():
                caps = e.pad_caps(pad)
                if caps is not None:
                    print(f"/{e.name}:{pad}: caps = {caps}")
    if a.messages:
        for m in p.messages():
            print(f"message: {m}")
    if a.dot:
        with open(a.dot, "w") as f:
            f.write(p.dot())
    p.stop()
    if msg is None:
        print(f"Timed out after {a.timeout:.1f} s", file=sys.stderr)
        return 3
    if msg[0] == "error":
        print(f"ERROR: {msg[1:]}", file=sys.stderr)
        return 1
    print(f"Got EOS from pipeline. Execution ended after {elapsed:.6f} s")
    return 0


if __name__ == "__main__":
    sys.exit(main())
