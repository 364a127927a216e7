"""Per-kernel PMC report from rocprofv3 --pmc counter CSVs (one directory per
pass, as scripts/pmc_f32.sh writes them): raw counters per dispatch averaged
over the kernel's dispatches, plus derived ratios.

    python scripts/pmc_report.py gpurun_out/pmc_f32 [name-substring]
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def short(name):
    m = re.search(r"(\w+_kernel)(<[^()]*>)?", name)
    if m:
        return m.group(1) + (m.group(2) or "")
    return name[:60]


def main():
    root = sys.argv[1]
    pat = sys.argv[2] if len(sys.argv) > 2 else ""
    tot = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(lambda: defaultdict(set))
    for f in glob.glob(os.path.join(root, "**", "*counter_collection.csv"), recursive=True):
        for r in csv.DictReader(open(f)):
            k = r.get("Kernel_Name", "")
            if pat not in k or "nnsx" not in k:
                continue
            n = short(k)
            c = r["Counter_Name"]
            tot[n][c] += float(r["Counter_Value"])
            disp[n][c].add(r.get("Dispatch_Id"))
    print(f"{'kernel':58s} {'MFMA':>9s} {'VALU/MFMA':>9s} {'LDS-conf%':>9s} {'wait%':>6s} "
          f"{'ldsw%':>6s} {'FETCH KB':>9s} {'WRITE KB':>9s} {'LDS/MFMA':>8s}  (per dispatch)")
    for n in sorted(tot):
        c = tot[n]
        nd = {k: max(1, len(v)) for k, v in disp[n].items()}
        per = lambda k: c.get(k, 0.0) / nd.get(k, 1)  # noqa: E731
        mfma = per("SQ_INSTS_MFMA")
        valu = per("SQ_INSTS_VALU")
        conf = 100 * per("SQ_LDS_BANK_CONFLICT") / per("SQ_LDS_IDX_ACTIVE") if per("SQ_LDS_IDX_ACTIVE") else 0
        wait = 100 * per("SQ_WAIT_ANY") / per("SQ_WAVE_CYCLES") if per("SQ_WAVE_CYCLES") else 0
        ldsw = 100 * per("SQ_WAIT_INST_LDS") / per("SQ_WAVE_CYCLES") if per("SQ_WAVE_CYCLES") else 0
        lds = per("SQ_INSTS_LDS")
        print(f"{n[:58]:58s} {mfma:9.3g} {valu / mfma if mfma else 0:9.2f} {conf:9.1f} {wait:6.1f} {ldsw:6.1f} "
              f"{per('FETCH_SIZE'):9.0f} {per('WRITE_SIZE'):9.0f} {lds / mfma if mfma else 0:8.2f}")
        # wave-time split (SQ_WAVE_CYCLES counts 4-cycle units): issuing, parked on
        # s_waitcnt / barriers, the rest stalled on dependencies; MFMA pipe busy =
        # SQ_VALU_MFMA_BUSY_CYCLES / SQ_BUSY_CYCLES / 32 SIMDs per SE
        wc = per("SQ_WAVE_CYCLES")
        if wc:
            iss = per("SQ_ACTIVE_INST_ANY") / wc
            wt = per("SQ_WAIT_ANY") / wc
            busy = per("SQ_VALU_MFMA_BUSY_CYCLES") / per("SQ_BUSY_CYCLES") / 32 if per("SQ_BUSY_CYCLES") else 0
            life = 4 * wc / per("SQ_WAVES") if per("SQ_WAVES") else 0
            salu = per("SQ_INSTS_SALU") / mfma if mfma else 0
            print(f"{'':58s}   wave lifetime {life:.0f} cycles; issuing {iss:.2f}, waitcnt/barrier {wt:.2f}, "
                  f"dependency stalls {max(0.0, 1 - iss - wt):.2f}; MFMA pipe busy {busy:.2f}; SALU/MFMA {salu:.2f}")


if __name__ == "__main__":
    main()
