#!/usr/bin/env python3
"""Static instruction mix of one kernel in a hipcc -S listing (gfx950): counts
per mnemonic, grouped (MFMA / VALU / packed VALU / LDS / VMEM / SALU / waits).

    python scripts/isa_mix.py listing.s <kernel-name-substring> [top]
"""
import collections
import re
import sys


def body_of(s, sub):
    for m in re.finditer(r"^([A-Za-z0-9_]+):\s*(?:;.*)?\n", s, re.M):
        name = m.group(1)
        if sub in name and not name.startswith(".L"):
            end = s.find("s_endpgm", m.end())
            return name, s[m.end():end]
    raise SystemExit(f"no kernel matching {sub}")


def main():
    s = open(sys.argv[1]).read()
    name, body = body_of(s, sys.argv[2])
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 30
    c = collections.Counter()
    for line in body.splitlines():
        t = line.strip().split()
        if not t or t[0].startswith((".", ";")) or t[0].endswith(":"):
            continue
        c[t[0]] += 1
    groups = collections.Counter()
    for k, v in c.items():
        if k.startswith("v_mfma"):
            g = "mfma"
        elif k.startswith("v_pk_"):
            g = "valu_packed"
        elif k.startswith("v_"):
            g = "valu"
        elif k.startswith("ds_"):
            g = "lds"
        elif k.startswith(("global_", "buffer_", "flat_")):
            g = "vmem"
        elif k.startswith("s_waitcnt"):
            g = "waitcnt"
        elif k.startswith("s_"):
            g = "salu"
        else:
            g = "other"
        groups[g] += v
    print(name)
    print("groups:", dict(groups))
    for k, v in c.most_common(top):
        print(f"  {k:30s} {v}")


if __name__ == "__main__":
    main()
