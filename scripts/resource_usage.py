#!/usr/bin/env python3
"""Per-kernel register / occupancy table of one HIP source for gfx950
(hipcc -Rpass-analysis=kernel-resource-usage), demangled and compact.

    python scripts/resource_usage.py csrc/kernels/mbv2_f32.hip [name-filter]
"""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/scripts/", 1)[0]


def main():
    src = sys.argv[1]
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    cmd = ["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", f"-I{ROOT}/csrc", f"-I{ROOT}/include", "-x", "hip",
           "--offload-arch=gfx950", "-munsafe-fp-atomics", "-ffp-contract=fast", "--cuda-device-only", "-c", src,
           "-o", "/dev/null", "-Rpass-analysis=kernel-resource-usage"]
    out = subprocess.run(cmd, capture_output=True, text=True).stderr
    rows, cur = [], None
    for line in out.splitlines():
        m = re.search(r"remark: (.*) \[-Rpass", line)
        if not m:
            continue
        t = m.group(1).strip()
        if t.startswith("Function Name:"):
            cur = {"name": t.split(":", 1)[1].strip()}
            rows.append(cur)
        elif cur is not None and ":" in t:
            k, v = t.split(":", 1)
            cur[k.strip()] = v.strip()
    names = subprocess.run(["c++filt"], input="\n".join(r["name"] for r in rows), capture_output=True,
                           text=True).stdout.splitlines()
    print(f"{'kernel':90s} {'VGPR':>5s} {'AGPR':>5s} {'spill':>5s} {'occ':>4s} {'SGPR':>5s}")
    for r, n in zip(rows, names):
        n = re.sub(r"\(anonymous namespace\)::|nnsx::kernels::|void ", "", n)
        n = re.sub(r"\(nnsx::kernels::[A-Za-z0-9]+\)$|\(.*\)$", "", n)
        if filt and filt not in n:
            continue
        print(f"{n[:90]:90s} {r.get('VGPRs', '?'):>5s} {r.get('AGPRs', '?'):>5s} {r.get('VGPRs Spill', '?'):>5s} "
              f"{r.get('Occupancy [waves/SIMD]', '?'):>4s} {r.get('SGPRs', '?'):>5s}")


if __name__ == "__main__":
    main()
