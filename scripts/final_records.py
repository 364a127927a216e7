"""Copy a gpu_r5_final.sh run (gpurun_out/final) into the tracked records under profiles/.

    python scripts/final_records.py <head-sha>
"""
import csv
import glob
import json
import os
import shutil
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "gpurun_out", "final")
DST = os.path.join(ROOT, "profiles")
head = sys.argv[1]


def last_json(path):
    for line in reversed(open(path).read().splitlines()):
        if line.startswith("{"):
            return json.loads(line)
    raise ValueError(path)


def kernel_stats(prof, title):
    f = glob.glob(os.path.join(prof, "**", "*kernel_stats.csv"), recursive=True)[0]
    rows = list(csv.DictReader(open(f)))
    total = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [title, f"# all kernels: {total / 1e6:.2f} ms over the run (including export / warm-up / check launches: "
                  "at::native and rocclr entries are outside the timed pipeline)",
           " calls  total ms    avg us      %  kernel"]
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"])):
        t = float(r["TotalDurationNs"])
        out.append(f"{int(r['Calls']):6d} {t / 1e6:9.2f} {t / int(r['Calls']) / 1e3:9.1f} {100 * t / total:6.1f}  "
                   f"{r['Name'][:160]}")
    return "\n".join(out) + "\n"


# default bench record
shutil.copy(os.path.join(SRC, "bench_default.json"), os.path.join(DST, "r5_bench_mbv2_b512_fp32_1gpu.json"))
# configs
lines = [f"# configs 3-5 (and the multi-rank configs at N=1) at the target batches and at 512, HEAD {head} defaults, "
         "1 x MI355X, fp32 (x3 products), bench.py --steps 100 --warmup 20 (scripts/gpu_drivers.sh gpu_r5_final)"]
recs = []
for f in sorted(glob.glob(os.path.join(SRC, "cfg_*.json"))):
    j = last_json(f)
    recs.append((j["config"]["model"][:60], j["config"]["global_batch"], j["value"], j["ms_per_step"], j.get("p50_latency_ms"),
                 j.get("fp32_method")))
for m, b, v, ms, p50, meth in sorted(recs):
    lines.append(f"{m:60s} batch {b:4d}  {v:11.1f} frames/s  {ms:9.4f} ms/step  p50 {p50} ms  fp32_method {meth}")
open(os.path.join(DST, "r5_bench_configs.txt"), "w").write("\n".join(lines) + "\n")
# kernel stats
open(os.path.join(DST, "r5_bench_kernel_stats.txt"), "w").write(kernel_stats(
    os.path.join(SRC, "prof_default"),
    f"# rocprofv3 --kernel-trace --stats of bench.py (MobileNetV2 b512 fp32, HEAD {head} defaults, 20 timed + 5 "
    "warm-up steps)"))
for c in ("ssd_b64", "posenet_b64", "deeplab_b8"):
    open(os.path.join(DST, f"r5_config_kernel_stats_{c}.txt"), "w").write(kernel_stats(
        os.path.join(SRC, f"prof_{c}"),
        f"# rocprofv3 --kernel-trace --stats of bench.py --config {c.replace('_b', ' --batch ')} (HEAD {head}, "
        "20 + 5 steps), 1 x MI355X"))
# per-layer split and GPU suite
shutil.copy(os.path.join(SRC, "layers_b512.txt"), os.path.join(DST, "r5_fp32_layers_b512.txt"))
suite = [l for l in open(os.path.join(SRC, "gpu_suite.txt")).read().splitlines() if "amdgpu.ids" not in l]
open(os.path.join(DST, f"r5_gpu_suite_{head}.txt"), "w").write(
    f"# python -m pytest tests -m gpu -q --timeout 300 -x at HEAD {head}, 1 x MI355X (scripts/gpu_drivers.sh gpu_r5_final)\n"
    + "\n".join(suite[-40:]) + "\n")
print("records written for", head)
