"""nnsx-pbtxt: gst-launch pipeline description <-> MediaPipe-style pbtxt.

    echo "videotestsrc ! tensor_converter ! tensor_sink" | nnsx-pbtxt
    nnsx-pbtxt --options "videotestsrc num-buffers=4 ! tensor_converter ! fakesink"
    nnsx-pbtxt --from-pbtxt < graph.pbtxt

Reference: tools/development/parser/toplevel.c (stdin in, pbtxt out; its
--from-pbtxt is "NYI" -- implemented here).
"""
from __future__ import annotations

import argparse
import sys


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="nnsx-pbtxt", description=__doc__.splitlines()[0])
    ap.add_argument("-p", "--from-pbtxt", action="store_true", help="from pbtxt to a launch description")
    ap.add_argument("-o", "--options", action="store_true",
                    help="emit node_options / stream_options with non-default properties (round-trippable)")
    ap.add_argument("-v", "--verbose", action="store_true")
    ap.add_argument("text", nargs="*", help="pipeline description (default: stdin)")
    a = ap.parse_args(argv)
    text = " ".join(a.text) if a.text else sys.stdin.read()
    import nnstreamer_amd as nns

    try:
        if a.from_pbtxt:
            print(nns.pbtxt_to_launch(text))
        else:
            print(nns.to_pbtxt(nns.parse_launch(text.strip()), a.options), end="")
    except Exception as e:  # noqa: BLE001
        print(f"nnsx-pbtxt: {e}", file=sys.stderr)
        return 1
    return 0


if __name__ == "__main__":
    sys.exit(main())
