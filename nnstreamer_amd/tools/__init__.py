"""Command-line tools (reference tools/development/confchk and gst-launch):

* ``python -m nnstreamer_amd.tools.check``  -- nnsx-check: version, config,
  registered elements / sub-plugins, GPUs (confchk.c:20-105).
* ``python -m nnstreamer_amd.tools.launch "<pipeline>"`` -- nnsx-launch: run a
  gst-launch style description to EOS (or a timeout) and print bus messages.

``bin/nnsx-check`` and ``bin/nnsx-launch`` are thin wrappers around these.
"""
