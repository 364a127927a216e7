"""nnsx-check: dump what this installation provides (reference
tools/development/confchk/confchk.c: version, configuration, sub-plugins)."""
from __future__ import annotations

import argparse
import json
import sys

KINDS = ("filter", "decoder", "converter", "trainer")


def report() -> dict:
    import nnstreamer_amd as nns

    gpus = []
    for d in range(nns.gpu_count()):
        gpus.append({"index": d, "arch": nns.gpu_arch(d)})
    return {
        "version": nns.version(),
        "gpus": gpus,
        "elements": sorted(e[0] for e in nns.list_elements()),
        "subplugins": {k: nns.subplugins(k) for k in KINDS},
        "config": nns.config_dump(),
    }


def main(argv=None) -> int:
    ap = argparse.ArgumentParser(prog="nnsx-check", description=__doc__)
    ap.add_argument("--json", action="store_true", help="machine-readable output")
    a = ap.parse_args(argv)
    r = report()
    if a.json:
        print(json.dumps(r, indent=2))
        return 0
    print(r["version"])
    print(f"GPUs: {len(r['gpus'])}" + "".join(f"\n  [{g['index']}] {g['arch']}" for g in r["gpus"]))
    print(f"Elements ({len(r['elements'])}):")
    for e in r["elements"]:
        print(f"  {e}")
    for k, v in r["subplugins"].items():
        print(f"{k} sub-plugins: {', '.join(v) if v else '(none)'}")
    print(r["config"])
    return 0


if __name__ == "__main__":
    sys.exit(main())
