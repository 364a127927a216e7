#!/bin/bash
# The one-shot GPU drivers of rounds 2-6, one case each, kept so that every
# committed profile that names a driver can be regenerated:
#   scripts/gpu_drivers.sh <name> [args...]      (scripts/gpu_drivers.sh list)
# Each case is the driver as it ran in its round, from the repository root; some
# exercise A/B switches (NNSX_* variables) that later rounds removed -- run them
# on the commit the profile names.  Current evidence: scripts/gpu_r6_round.sh.
cd "$(dirname "$0")/.."
name=$1
shift || true
case "$name" in
blaslt_probe)
python3 - "$@" <<'PY'
"""hipBLASLt path numerics probe (pw_conv shapes that take it)."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch  # noqa: E402

import nnstreamer_amd  # noqa: F401,E402

torch.manual_seed(0)
for M, K, N, act, use_res in [(4096, 128, 64, 0, False), (4096, 128, 64, 1, False), (4096, 128, 64, 0, True),
                              (6272, 320, 1280, 0, False), (6272, 320, 1280, 1, False)]:
    x = torch.randn(M, K, device="cuda")
    wt = torch.randn((N + 15) // 16 * 16, K, device="cuda") / K ** 0.5
    bias = torch.randn(wt.shape[0], device="cuda")
    res = torch.randn(M, N, device="cuda") if use_res else None
    y = torch.ops.nnsx.pw_conv(x, wt, bias, res, N, act, True)
    ref = x @ wt[:N].t()
    nob = ref.clone()
    ref = ref + bias[:N]
    if use_res:
        ref = ref + res
    if act == 1:
        ref = ref.clamp(0, 6)
    err = (y - ref).abs().max().item()
    print(f"M={M} K={K} N={N} act={act} res={use_res}: max err {err:.3g}; y[0,:4] {y[0, :4].tolist()} "
          f"ref {ref[0, :4].tolist()} nobias {nob[0, :4].tolist()} relu6(nobias) {nob[0, :4].clamp(0, 6).tolist()}")
PY
;;
gpu_ab_variant)
(
# same-box A/B: HEAD tree vs variants/$V (a copy of the package from another commit)
set -eo pipefail
:
mkdir -p gpurun_out
V=${V:-base}
for rep in 1 2; do
  for spec in ${SPECS:-mbv2:512 posenet:64 deeplab:8}; do
    c=${spec%%:*}; B=${spec##*:}
    for arm in new $V; do
      if [ $arm = new ]; then b=bench.py; else b=variants/$V/bench.py; fi
      timeout -k 10 300 python $b --config $c --batch $B --sweep "" --latency-frames 0 > gpurun_out/ab_${arm}_$c.json 2>/dev/null
      echo "$rep $arm $c $(grep -h -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${arm}_$c.json)"
    done
  done
done
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > gpurun_out/ab_layers_new.txt 2>&1
timeout -k 10 300 python -u variants/$V/scripts/bench_ir_f32.py 512 > gpurun_out/ab_layers_$V.txt 2>&1
)
;;
gpu_b1_combine_ab)
(
# Batch-1 launch-count A/B: hidden-part combine (NNSX_F32_IRW_INLAUNCH 0 =
# irw_reduce launches, 2 = in-launch spread combine) x small-M GEMMs
# (NNSX_F32_SMALLM 0 = split-K GEMM + reduce launch, 1 = one-launch pw_small_f32
# and the fused head + pool).  Numerics first (bitwise / fp64 gates), then
# back-to-back graph replays and the live-camera latency probe per setting.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NNSX_F32_IRW_INLAUNCH=2 timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q --timeout 120 --timeout-method thread \
  -k "inlaunch_combine or small_m or conv_pool or top1_matches or split_k" > gpurun_out/b1c_numerics.log 2>&1 || { echo "numerics failed"; tail -30 gpurun_out/b1c_numerics.log; exit 1; }
tail -1 gpurun_out/b1c_numerics.log
for C in ${COMBOS:-"0 0" "0 1" "2 1" "0 0" "0 1" "2 1"}; do
  set -- $C
  tag=inl$1_sm$2
  NNSX_F32_IRW_INLAUNCH=$1 NNSX_F32_SMALLM=$2 timeout -k 10 200 python3 scripts/b1_graph_probe.py > gpurun_out/b1c_probe_$tag.log 2>&1 || { echo "probe $tag failed"; tail -20 gpurun_out/b1c_probe_$tag.log; exit 1; }
  echo "$tag: $(grep -E 'back-to-back' gpurun_out/b1c_probe_$tag.log)"
done
for C in ${LAT_COMBOS:-"0 0" "2 1"}; do
  set -- $C
  tag=inl$1_sm$2
  NNSX_F32_IRW_INLAUNCH=$1 NNSX_F32_SMALLM=$2 timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/b1c_lat_$tag.json 2> gpurun_out/b1c_lat_$tag.err || { echo "latency $tag failed"; tail -20 gpurun_out/b1c_lat_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b1c_lat_$tag.json')); print('$tag b1 latency', d['latency_us'], 'device', d['filter_device_us_median'])"
done
)
;;
gpu_b1_lat_ab)
(
# Batch-1 live-camera latency A/B (500 fps, 600 frames per run), settings
# interleaved so box drift hits each equally.  A setting is
# "<NNSX_F32_IRW_INLAUNCH>:<NNSX_F32_SMALLM>".
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for C in ${SETTINGS:-0:0 2:1 0:1 2:0 0:0 2:1 0:1 2:0}; do
  inl=${C%%:*}; sm=${C##*:}; i=$((i + 1))
  tag=r${i}_inl${inl}_sm${sm}
  NNSX_F32_IRW_INLAUNCH=$inl NNSX_F32_SMALLM=$sm timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/b1lat_$tag.json 2> gpurun_out/b1lat_$tag.err || { echo "latency $tag failed"; tail -20 gpurun_out/b1lat_$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/b1lat_$tag.json')); l=d['latency_us']; print('$tag p50 %.1f p99 %.1f device %.1f' % (l['p50'], l['p99'], d['filter_device_us_median']))"
done
)
;;
gpu_b1_prof)
(
# Batch-1 forward under rocprofv3 (kernel trace + stats): back-to-back graph
# replays of the fp32 engine (scripts/b1_graph_probe.py), and the live-camera
# latency probe.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/b1prof -o b1 --output-format csv -- python3 $R/scripts/b1_graph_probe.py > $R/gpurun_out/b1prof.log 2>&1 || { echo "b1 prof failed"; tail -20 $R/gpurun_out/b1prof.log; exit 1; }
grep -E "graph replay|eager" $R/gpurun_out/b1prof.log
cd $R && timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/b1_latency.json 2> gpurun_out/b1_latency.err || { echo "b1 latency failed"; tail -20 gpurun_out/b1_latency.json; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/b1_latency.json')); print('b1 latency', d['latency_us'], 'device', d['filter_device_us_median'])"
)
;;
gpu_b1_upload_ab)
(
# Batch-1 single-frame upload: copy engine (hipMemcpyAsync, default) vs the
# gather kernel reading the pinned frame over the bus (NNSX_CONV_KERNEL_UPLOAD=1).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NNSX_CONV_KERNEL_UPLOAD=1 timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q --timeout 120 --timeout-method thread \
  -k "decoder_argmax_absorbed or benched_launch_string" > gpurun_out/upload_numerics.log 2>&1 || { echo "numerics failed"; tail -30 gpurun_out/upload_numerics.log; exit 1; }
tail -1 gpurun_out/upload_numerics.log
for U in ${UPLOADS:-0 1 0 1 0 1}; do
  NNSX_CONV_KERNEL_UPLOAD=$U timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/upload_lat_$U.json 2> gpurun_out/upload_lat_$U.err || { echo "latency upload=$U failed"; tail -20 gpurun_out/upload_lat_$U.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/upload_lat_$U.json')); l=d['latency_us']; print('kernel_upload=$U p50 %.1f p99 %.1f device %.1f' % (l['p50'], l['p99'], d['filter_device_us_median']))"
done
)
;;
gpu_config_traces)
(
# fp32 records + one rocprofv3 kernel trace per single-GPU BASELINE config
# (bench.py --config ...), each step under its own time limit.  Summaries:
# gpurun_out/cfgtrace_<config>.txt (scripts/config_trace_report.py).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for spec in ${SPECS:-ssd:64 deeplab:8 posenet:64}; do
  c=${spec%%:*}; B=${spec##*:}
  cd $R && timeout -k 10 300 python3 bench.py --config $c --batch $B --steps 20 --warmup 5 --sweep "" > gpurun_out/bench_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/bench_$c.log; exit 1; }
  tail -1 gpurun_out/bench_$c.log | cut -c1-300
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/cfg_$c -o k --output-format csv -- python3 $R/bench.py --config $c --batch $B --steps 6 --warmup 3 --sweep "" --latency-frames 0 > $R/gpurun_out/cfgprof_$c.log 2>&1 || { echo "trace $c failed"; tail -20 $R/gpurun_out/cfgprof_$c.log; exit 1; }
  cd $R && python3 scripts/config_trace_report.py gpurun_out/cfg_$c > gpurun_out/cfgtrace_$c.txt && head -40 gpurun_out/cfgtrace_$c.txt
done
)
;;
gpu_final_check)
(
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_round.sh test && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && cut -c1-300 gpurun_out/bench_default.json
)
;;
gpu_host_argmax_ab)
(
# Absorbed-argmax indices copied to pinned host memory after each replay
# (NNSX_TORCH_HOST_ARGMAX=1) vs a device clone read back by the decoder (0): GPU tests,
# then the batch-1 live latency, settings interleaved.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
NNSX_TORCH_HOST_ARGMAX=1 timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
for H in ${HOSTS:-0 1 0 1 0 1}; do
  NNSX_TORCH_HOST_ARGMAX=$H timeout -k 10 300 python3 scripts/b1_latency_probe.py 600 500 > gpurun_out/hargmax_lat_$H.json 2> gpurun_out/hargmax_lat_$H.err || { echo "latency host_argmax=$H failed"; tail -20 gpurun_out/hargmax_lat_$H.err; exit 1; }
  python3 -c "import json; d=json.load(open('gpurun_out/hargmax_lat_$H.json')); l=d['latency_us']; print('host_argmax=$H p50 %.1f p99 %.1f device %.1f' % (l['p50'], l['p99'], d['filter_device_us_median']))"
done
)
;;
gpu_pipe_ab)
(
# Pipelined-expand (VAR = 1) irw variants: numerics under the variant selection,
# then per-layer A/B at batch 512 against the defaults.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
SKIP_ALL=${SKIP_ALL:-0,1,2,3,13,14,15,16}
NNSX_IRW_SKIP=$SKIP_ALL timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q --timeout 120 --timeout-method thread \
  -k "ir_block_f32 or bench_batch_matches" > gpurun_out/pipe_numerics.log 2>&1 || { echo "numerics failed"; tail -30 gpurun_out/pipe_numerics.log; exit 1; }
tail -2 gpurun_out/pipe_numerics.log
NNSX_STEM_WAVE=3 timeout -k 10 300 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -q --timeout 120 --timeout-method thread \
  -k "stem_ir1 or bench_batch_matches" > gpurun_out/spipe_numerics.log 2>&1 || { echo "stem numerics failed"; tail -30 gpurun_out/spipe_numerics.log; exit 1; }
tail -2 gpurun_out/spipe_numerics.log
NNSX_STEM_WAVE=3 timeout -k 10 300 python scripts/bench_ir_f32.py 512 > gpurun_out/spipe_ab.txt 2>&1 || { echo "stem bench failed"; tail -20 gpurun_out/spipe_ab.txt; exit 1; }
echo "== stem pipelined"; grep -E "stem|TOTAL" gpurun_out/spipe_ab.txt
VARIANTS=${VARIANTS:-"0,1,13,14,15,16 $SKIP_ALL"} bash scripts/irw_ab.sh
)
;;
gpu_pmc_early)
(
# PMC passes on the early fused fp32 blocks at batch 512 (scripts/pmc_f32.sh per block)
set -o pipefail
export TMPDIR=/tmp
for S in "112,16,96,24,2" "56,24,144,24,1"; do
  tag=${S//,/_}
  OUT=gpurun_out/pmc_early_$tag SHAPE=$S B=512 bash scripts/pmc_f32.sh > gpurun_out/pmc_early_$tag.txt 2>&1 || { echo "pmc $S failed"; tail -5 gpurun_out/pmc_early_$tag.txt; exit 1; }
  cat gpurun_out/pmc_early_$tag.txt
done
)
;;
gpu_r3_hiptrace)
(
# Host-side view of the bench step: HIP runtime API + kernel + copy trace of a
# short default bench run (where the per-step GPU idle comes from).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --hip-trace --kernel-trace --memory-copy-trace --stats -d $R/gpurun_out/hiptrace -o run --output-format csv -- python3 $R/bench.py --steps 12 --warmup 4 --latency-frames 0 --sweep "" > $R/gpurun_out/hiptrace.log 2>&1 || { echo "trace failed"; tail -30 $R/gpurun_out/hiptrace.log; exit 1; }
grep -o '"value": [0-9.]*' $R/gpurun_out/hiptrace.log
ls -la $R/gpurun_out/hiptrace/*
python3 $R/scripts/stall_report.py $R/gpurun_out/hiptrace > $R/gpurun_out/stall_report.txt 2>&1 && tail -22 $R/gpurun_out/stall_report.txt
)
;;
gpu_r4_b512cfg)
(
# configs 3-5 at bench.py's default batch (512 frames per invoke)
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/b512cfg.txt
: > $out
for c in ssd deeplab posenet; do
  timeout -k 10 200 python bench.py --config $c --steps 30 --warmup 5 --sweep "" --latency-frames 0 > gpurun_out/b512_$c.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/b512_$c.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/b512_$c.log') if l.startswith('{')][-1]); print('$c', d['config'].get('global_batch'), d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))" | tee -a $out
done
)
;;
gpu_r4_cfgprof)
(
# Per-kernel time of one single-GPU config (CFG, B) under rocprofv3 --kernel-trace --stats.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
C=${CFG:-ssd}; B=${B:-64}
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_$C -o run -- python3 $R/bench.py --config $C --batch $B --steps 10 --warmup 5 --sweep "" --latency-frames 0 > $R/gpurun_out/prof_$C.log 2>&1 || { echo "prof failed"; tail -30 $R/gpurun_out/prof_$C.log; exit 1; }
cd $R
db=gpurun_out/prof_$C/run_results.db
python3 - "$db" > gpurun_out/prof_${C}_streams.txt <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
for s, n, t in c.execute("select stream_id, count(*), sum(end-start) from kernels group by stream_id order by 3 desc"):
    print(f"stream {s}: {n} dispatches, {t/1e3:.1f} us")
PY
cat gpurun_out/prof_${C}_streams.txt
for st in $(grep "^stream" gpurun_out/prof_${C}_streams.txt | head -2 | awk '{print $2}' | tr -d :); do python3 scripts/rocpd_stats.py "$db" 45 --stream $st > gpurun_out/prof_${C}_stream_$st.txt 2>&1; done
tail -1 gpurun_out/prof_$C.log | cut -c1-300
)
;;
gpu_r4_configs)
(
# Round 4: every BASELINE config on one GPU (incl. the multi-rank configs at N=1) plus
# kernel traces of DeepLab / PoseNet (padded-frame upload path).
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for spec in ${SPECS:-ssd:64 deeplab:8 deeplab:16 deeplab:32 posenet:64 deeplab_fan:8 posenet_multi:64}; do
  c=${spec%%:*}; B=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --batch $B --steps ${STEPS:-20} --warmup ${WARMUP:-5} --sweep "" > gpurun_out/bench_${c}_b$B.log 2>&1 || { echo "bench $c failed"; tail -30 gpurun_out/bench_${c}_b$B.log; exit 1; }
  tail -1 gpurun_out/bench_${c}_b$B.log | cut -c1-300
done
for spec in ${TRACES:-deeplab:8 posenet:64}; do
  c=${spec%%:*}; B=${spec##*:}
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof_$c -o $c -- \
     python $GRAFT_REPO_ROOT/bench.py --config $c --batch $B --steps 10 --warmup 3 --sweep "" --latency-frames 0 > $GRAFT_REPO_ROOT/gpurun_out/prof_$c.log 2>&1) || { echo "trace $c failed"; exit 1; }
done
echo done
)
;;
gpu_r4_dllanes)
(
# DeepLab at small batches: replay lanes auto (3 below 33 frames / 8 MB) vs 1
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dllanes.txt
: > $out
for B in 8 16; do
  for L in 1 3 1 3; do
    NNSX_TORCH_LANES=$L timeout -k 10 200 python bench.py --config deeplab --batch $B --steps 60 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/dll_b${B}_$L.log 2>&1 || { echo "bench $B $L failed"; tail -20 gpurun_out/dll_b${B}_$L.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/dll_b${B}_$L.log') if l.startswith('{')][-1]); print('deeplab b$B lanes=$L', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'), d.get('p50_latency_ms'))" | tee -a $out
  done
done
)
;;
gpu_r4_dwdil)
(
# dilation-2 depthwise as 4x4 column lanes: gates, kernel A/B, DeepLab benches A/B
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dw or deeplab" > gpurun_out/dwdil_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/dwdil_pytest.log; exit 1; }
tail -1 gpurun_out/dwdil_pytest.log
timeout -k 10 120 python scripts/dw_roofline.py 2>/dev/null | grep "^B=" > gpurun_out/dwdil_roof.txt
NNSX_F32_DW_DIL_COL=0 timeout -k 10 120 python scripts/dw_roofline.py 2>/dev/null | grep "^B=" > gpurun_out/dwdil_roof_off.txt
out=gpurun_out/dwdil_bench.txt
: > $out
for B in 8 32; do
  for v in 1 0; do
    NNSX_F32_DW_DIL_COL=$v timeout -k 10 200 python bench.py --config deeplab --batch $B --steps 40 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/dwdil_b${B}_$v.log 2>&1 || { echo "bench $B $v failed"; tail -20 gpurun_out/dwdil_b${B}_$v.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/dwdil_b${B}_$v.log') if l.startswith('{')][-1]); print('deeplab b$B dil_col=$v', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))" | tee -a $out
  done
done
)
;;
gpu_r4_dwnew)
(
# 4x4 / 2x2 depthwise lanes as the default: depthwise + model gates, then the config benches
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "dw or sep_heads or models_f32 or posenet or ssd or deeplab or mbv2_f32" > gpurun_out/dwnew_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/dwnew_pytest.log; exit 1; }
tail -1 gpurun_out/dwnew_pytest.log
timeout -k 10 120 python scripts/dw_roofline.py 2>/dev/null | grep "^B=" > gpurun_out/dwnew_roof.txt
out=gpurun_out/dwnew_bench.txt
: > $out
for spec in mbv2:512 posenet:64 ssd:64 deeplab:8 posenet:512; do
  c=${spec%%:*}; B=${spec##*:}
  for v in 44:22 0:0; do
    a=${v%%:*}; b=${v##*:}
    NNSX_F32_DW_S1=$a NNSX_F32_DW_S2=$b timeout -k 10 200 python bench.py --config $c --batch $B --steps 60 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/dwnew_${c}_$a.log 2>&1 || { echo "bench $c $a failed"; tail -20 gpurun_out/dwnew_${c}_$a.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/dwnew_${c}_$a.log') if l.startswith('{')][-1]); print('$c b$B dw=$a/$b', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))" | tee -a $out
  done
done
)
;;
gpu_r4_dwsweep)
(
# depthwise lane shapes (rows x columns per lane), stride 1 / stride 2: scripts/dw_roofline.py per pair
set -o pipefail
mkdir -p gpurun_out
out=gpurun_out/dw_sweep.txt
: > $out
for pair in 0:0 42:22 44:12 81:14 82:42 22:0 24:0; do
  a=${pair%%:*}; b=${pair##*:}
  echo "# NNSX_F32_DW_S1=$a NNSX_F32_DW_S2=$b" >> $out
  NNSX_F32_DW_S1=$a NNSX_F32_DW_S2=$b timeout -k 10 120 python scripts/dw_roofline.py 2>/dev/null | grep "^B=" >> $out || { echo "run $pair failed"; exit 1; }
done
)
;;
gpu_r4_final)
(
# Round 4 final check: whole GPU suite, smoke, default bench, the three single-GPU configs.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_final.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_final.log; exit 1; }
tail -2 gpurun_out/pytest_final.log
timeout -k 10 150 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke_final.log 2>&1 || { echo "smoke failed"; tail -20 gpurun_out/smoke_final.log; exit 1; }
tail -1 gpurun_out/smoke_final.log
timeout -k 10 170 python bench.py > gpurun_out/bench_final.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/bench_final.log; exit 1; }
tail -1 gpurun_out/bench_final.log | cut -c1-400
for spec in posenet:64 ssd:64 deeplab:8 deeplab:32; do
  c=${spec%%:*}; B=${spec##*:}
  timeout -k 10 170 python bench.py --config $c --batch $B --steps 30 --warmup 10 --sweep "" > gpurun_out/final_${c}_b$B.log 2>&1 || { echo "bench $c failed"; tail -20 gpurun_out/final_${c}_b$B.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/final_${c}_b$B.log') if l.startswith('{')][-1]); print('$c b$B', d['value'], d['ms_per_step'], d.get('p50_latency_ms'), d.get('p50_latency_ms_b1'), d.get('p99_latency_ms_b1'))"
done
)
;;
gpu_r4_heads)
(
# SSD heads: grouped depthwise + grouped GEMM (sep_heads mode 0, default) vs 2 launches per head
# (NNSX_SSD_SEP_HEADS=0): fp64 gates, then bench.py --config ssd at batch 64 and 512.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_models_f32.py -x -q --timeout 120 --timeout-method thread -k "sep_heads or ssd" > gpurun_out/heads_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/heads_pytest.log; exit 1; }
tail -1 gpurun_out/heads_pytest.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "ssd or bbox or bounding" > gpurun_out/heads_pytest2.log 2>&1 || { echo "pytest2 failed"; tail -40 gpurun_out/heads_pytest2.log; exit 1; }
tail -1 gpurun_out/heads_pytest2.log
out=gpurun_out/heads_ab.txt
: > $out
for B in 64 512; do
  for v in 1 0 1 0; do
    NNSX_SSD_SEP_HEADS=$v timeout -k 10 200 python bench.py --config ssd --batch $B --steps ${STEPS:-60} --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/heads_b${B}_$v.log 2>&1 || { echo "bench B=$B v=$v failed"; tail -20 gpurun_out/heads_b${B}_$v.log; exit 1; }
    python3 -c "import json; d=json.loads([l for l in open('gpurun_out/heads_b${B}_$v.log') if l.startswith('{')][-1]); print('ssd b$B grouped_heads=$v', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))" | tee -a $out
  done
done
)
;;
gpu_r4_lanes512)
(
# Replay lanes at the headline batch (and 128): bench.py frames/s with NNSX_TORCH_LANES=1/2/3.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
out=gpurun_out/lanes512.txt
: > $out
for B in ${BATCHES:-512 128}; do
  for L in ${LANES:-1 3 2}; do
    NNSX_TORCH_LANES=$L timeout -k 10 200 python bench.py --batch $B --steps ${STEPS:-100} --warmup 10 --sweep "" --latency-frames 0 ${QARGS} > gpurun_out/lanes_b${B}_l$L.log 2>&1 || { echo "bench B=$B L=$L failed"; tail -20 gpurun_out/lanes_b${B}_l$L.log; exit 1; }
    python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/lanes_b${B}_l$L.log') if l.startswith('{')][-1]); print('b$B lanes=$L', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'), d.get('p50_latency_ms'))" | tee -a $out
  done
done
)
;;
gpu_r4_mbv2_ab)
(
# Round 4: headline-engine A/B (layer timings + short bench) of the candidate changes,
# then the PMC of the line-buffer stem.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python3 scripts/bench_ir_f32.py 512 > gpurun_out/r4_fp32_layers_b512.txt 2>&1 || { echo "layers failed"; tail -20 gpurun_out/r4_fp32_layers_b512.txt; exit 1; }
cat gpurun_out/r4_fp32_layers_b512.txt
NNSX_IRW_SKIP=6 timeout -k 10 300 python3 scripts/bench_ir_f32.py 512 > gpurun_out/r4_fp32_layers_b512_t77.txt 2>&1 || { echo "layers t714 failed"; exit 1; }
grep -E "H=14|TOTAL" gpurun_out/r4_fp32_layers_b512_t77.txt
run() {  # name, env... (BENCH_ARGS: extra bench.py arguments)
  local name=$1; shift
  env "$@" timeout -k 10 300 python bench.py --steps 30 --warmup 10 --latency-frames 0 --sweep "" $BENCH_ARGS > gpurun_out/ab_$name.log 2>&1 || { echo "ab $name failed"; tail -20 gpurun_out/ab_$name.log; return 1; }
  python3 -c "import json,sys; d=json.loads([l for l in open('gpurun_out/ab_$name.log') if l.startswith('{')][-1]); print('$name', d['value'], d['ms_per_step'], d['gpu_invoke_ms_median'], d['p50_latency_ms'])"
}
run base NNSX_NONE=1 && run t77_64 NNSX_IRW_SKIP=6 && run headpool_off NNSX_F32_HEAD_POOL=0 && run dwpw_all NNSX_DWPW_ALL=1 && run gemm128 NNSX_F32_GEMM_TILE=128128 && run base2 NNSX_NONE=1 && BENCH_ARGS="--queue 1 --queue-in 1" run q11 NNSX_NONE=1 && BENCH_ARGS="--queue 2 --queue-in 1" run q21 NNSX_NONE=1 || exit 1
for S in stem stemband; do
  OUT=gpurun_out/pmc_$S SHAPE=$S B=512 bash scripts/pmc_f32.sh > gpurun_out/pmc_$S.txt 2>&1 || { echo "pmc $S failed"; tail -5 gpurun_out/pmc_$S.txt; exit 1; }
  cat gpurun_out/pmc_$S.txt
done
)
;;
gpu_r4_pmc)
(
# PMC of the early fused blocks and the stem at batch 512 (current defaults) + the layer table
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/bench_ir_f32.py 512 > gpurun_out/r4_fp32_layers_b512_final.txt 2>&1 || { echo "layers failed"; exit 1; }
grep -E "fused|stem|TOTAL|head|chain" gpurun_out/r4_fp32_layers_b512_final.txt | head -30
rm -f gpurun_out/pmc_early_all.txt
for S in stem "112,16,96,24,2" "56,24,144,24,1" "56,24,144,32,2" "28,32,192,32,1" "14,64,384,64,1"; do
  n=$(echo $S | tr ',' '_')
  OUT=gpurun_out/pmc_fin_$n SHAPE=$S B=512 bash scripts/pmc_f32.sh > gpurun_out/pmc_fin_$n.txt 2>&1 || { echo "pmc $S failed"; tail -5 gpurun_out/pmc_fin_$n.txt; exit 1; }
  cat gpurun_out/pmc_fin_$n.txt >> gpurun_out/pmc_early_all.txt
done
cat gpurun_out/pmc_early_all.txt
)
;;
gpu_r4_posehead)
(
# PoseNet heads as one grouped GEMM (nnsx::pw_conv_group): fp64 gates, pose goldens, bench b64 / b512.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_models_f32.py -x -q --timeout 120 --timeout-method thread -k "pw_conv_group or posenet" > gpurun_out/ph_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/ph_pytest.log; exit 1; }
tail -1 gpurun_out/ph_pytest.log
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "pose" > gpurun_out/ph_pytest2.log 2>&1 || { echo "pytest2 failed"; tail -40 gpurun_out/ph_pytest2.log; exit 1; }
tail -1 gpurun_out/ph_pytest2.log
out=gpurun_out/posehead_ab.txt
: > $out
for B in 64 512; do
  timeout -k 10 200 python bench.py --config posenet --batch $B --steps 60 --warmup 10 --sweep "" --latency-frames ${LATF:-0} > gpurun_out/ph_b$B.log 2>&1 || { echo "bench B=$B failed"; tail -20 gpurun_out/ph_b$B.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ph_b$B.log') if l.startswith('{')][-1]); print('posenet b$B', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'), d.get('p50_latency_ms_b1'))" | tee -a $out
done
)
;;
gpu_r4_prof)
(
# Round 4: per-kernel time of the default bench (batch-512 throughput run + batch-1 live run) under
# rocprofv3 --kernel-trace --stats; tables per stream via scripts/rocpd_stats.py.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof_r4 -o run -- python3 $R/bench.py --steps 10 --warmup 5 > $R/gpurun_out/prof_r4.log 2>&1 || { echo "prof failed"; tail -30 $R/gpurun_out/prof_r4.log; exit 1; }
cd $R
db=$(find gpurun_out/prof_r4 -name "*results.db" | head -1)
echo "db=$db"
python3 scripts/rocpd_stats.py "$db" 40 > gpurun_out/prof_r4_all.txt 2>&1
python3 - "$db" > gpurun_out/prof_r4_streams.txt <<'PY'
import sqlite3, sys
c = sqlite3.connect(sys.argv[1])
cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
sc = "stream_id" if "stream_id" in cols else ("queue_id" if "queue_id" in cols else None)
print("columns:", cols)
if sc:
    for s, n, t in c.execute(f"select {sc}, count(*), sum(end-start) from kernels group by {sc} order by 3 desc"):
        print(f"stream {s}: {n} dispatches, {t/1e3:.1f} us")
PY
cat gpurun_out/prof_r4_streams.txt
for st in $(grep "^stream" gpurun_out/prof_r4_streams.txt | head -3 | awk '{print $2}' | tr -d :); do python3 scripts/rocpd_stats.py "$db" 25 --stream $st > gpurun_out/prof_r4_stream_$st.txt 2>&1; done
tail -1 gpurun_out/prof_r4.log | cut -c1-300
)
;;
gpu_r4_small)
(
# Round 4: small-batch forward traces (batch 1 and 8: back-to-back graph replays)
# and the ATen-origin analysis of a short bench run.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for B in 1 8; do
  cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/fwdprof_b$B -o fwd --output-format csv -- python3 $R/scripts/b1_graph_probe.py $B > $R/gpurun_out/fwdprof_b$B.log 2>&1 || { echo "fwd prof $B failed"; tail -20 $R/gpurun_out/fwdprof_b$B.log; exit 1; }
  grep -E "graph replay" $R/gpurun_out/fwdprof_b$B.log
done
# padded-frame upload micro-bench (DeepLab 513 / PoseNet 257 wide): DMA + unpad vs the gather kernel
rm -f gpurun_out/upload_bench.txt
cd $R && for w in 513:8 257:64; do
  UPLOAD_BENCH_HOST=1 timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 >> gpurun_out/upload_bench.txt 2>&1 && \
  timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 >> gpurun_out/upload_bench.txt 2>&1 && \
  NNSX_CONVERTER_DMA_SPLIT=2 timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 >> gpurun_out/upload_bench.txt 2>&1 && \
  NNSX_CONVERTER_DMA_SPLIT=4 timeout -k 10 120 python3 scripts/upload_bench.py ${w%%:*} ${w##*:} 100 >> gpurun_out/upload_bench.txt 2>&1 || { echo "upload bench failed"; tail -20 gpurun_out/upload_bench.txt; exit 1; }
done
cat gpurun_out/upload_bench.txt
# batch 8 as the headline run (long window): pipeline ms per batch vs device ms per invoke
# (replay lanes: auto = 2 at these batches, NNSX_TORCH_LANES=1 the single-stream A/B)
cd $R && for B in 8 16 32; do for L in 1 2 3 4; do
  NNSX_TORCH_LANES=$L timeout -k 10 300 python3 bench.py --batch $B --steps 400 --warmup 20 --latency-frames 0 --sweep "" > gpurun_out/bench_b${B}_l$L.log 2>&1 || { echo "bench b$B lanes $L failed"; tail -20 gpurun_out/bench_b${B}_l$L.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/bench_b${B}_l$L.log') if l.startswith('{')][-1]); print('b$B lanes=$L', d['value'], d['ms_per_step'], d['gpu_invoke_ms_median'], d['p50_latency_ms'])"
done; done
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace -d $R/gpurun_out/prof_aten -o aten -- python3 $R/bench.py --steps 10 --warmup 3 --latency-frames 50 --sweep 8 > $R/gpurun_out/prof_aten.log 2>&1 || { echo "aten prof failed"; tail -20 $R/gpurun_out/prof_aten.log; exit 1; }
cd $R && python3 scripts/aten_origin.py gpurun_out/prof_aten/aten_results.db > gpurun_out/aten_origin.txt 2>&1; tail -30 gpurun_out/aten_origin.txt
)
;;
gpu_r4_ssd5)
(
# 5x5 tiles for SSD's 10x10 stage: numerics, then SSD A/B (NNSX_IRW_SKIP=17,18: the 7x7 tiles as before)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pt_ssd5.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/pt_ssd5.log; exit 1; }
tail -1 gpurun_out/pt_ssd5.log
for spec in "new:NNSX_NONE=1" "old:NNSX_IRW_SKIP=17,18" "new2:NNSX_NONE=1"; do
  n=${spec%%:*}; e=${spec#*:}
  env $e timeout -k 10 170 python bench.py --config ssd --batch 64 --steps 30 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/ssd5_$n.log 2>&1 || { echo "bench $n failed"; tail -20 gpurun_out/ssd5_$n.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/ssd5_$n.log') if l.startswith('{')][-1]); print('ssd $n', d['value'], d['ms_per_step'])"
done
)
;;
gpu_r4_stage)
(
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_decode_stage.py tests/test_gpu_mbv2_f32.py tests/test_gpu_comm.py tests/test_gpu_models_f32.py tests/test_gpu_elements.py tests/test_gpu_decoders_golden.py tests/test_gpu_pipelines.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_stage.log 2>&1 || { echo "pytest failed"; tail -60 gpurun_out/pytest_stage.log; exit 1; }
tail -3 gpurun_out/pytest_stage.log
# A/B of the new fusions (env toggles) on the config benches
for spec in "posenet:64:NNSX_POSENET_DWPW=0" "deeplab:8:NNSX_DWPW_DILATED=0" "ssd:64:NNSX_SSD_SEP_HEADS=0"; do
  IFS=: read c B envv <<< "$spec"
  env $envv timeout -k 10 300 python bench.py --config $c --batch $B --steps 20 --warmup 5 --sweep "" --latency-frames 0 > gpurun_out/bench_${c}_b${B}_off.log 2>&1 || { echo "bench $c off failed"; tail -20 gpurun_out/bench_${c}_b${B}_off.log; exit 1; }
  echo "$envv: $(tail -1 gpurun_out/bench_${c}_b${B}_off.log | cut -c1-200)"
done
bash scripts/gpu_drivers.sh gpu_r4_configs
)
;;
gpu_r4_stem)
(
# stem staging change: gates, PoseNet bench, per-kernel trace
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "stem or posenet or pose" > gpurun_out/stem_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/stem_pytest.log; exit 1; }
tail -1 gpurun_out/stem_pytest.log
for B in 64 512; do
  timeout -k 10 170 python bench.py --config posenet --batch $B --steps 40 --warmup 10 --sweep "" --latency-frames 0 > gpurun_out/stem_b$B.log 2>&1 || { echo "bench failed"; tail -20 gpurun_out/stem_b$B.log; exit 1; }
  python3 -c "import json; d=json.loads([l for l in open('gpurun_out/stem_b$B.log') if l.startswith('{')][-1]); print('posenet b$B', d['value'], d['ms_per_step'], d.get('gpu_invoke_ms_median'))"
done
)
;;
gpu_r5_final)
(
# Round-5 records at HEAD defaults: GPU suite, default bench, configs 3-5 (target batches and 512),
# kernel stats of the default bench and of each config, per-layer split at batch 512
# (PART=1: suite, bench, configs; PART=2: per-layer split and kernel traces; unset: both)
set -eo pipefail
:
mkdir -p gpurun_out/final
export TMPDIR=/tmp
R=$PWD
O=gpurun_out/final
if [ "${PART:-1}" = 1 ]; then
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread -x > $O/gpu_suite.txt 2>&1
tail -2 $O/gpu_suite.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-220
for spec in ssd:64 posenet:64 deeplab:8 ssd:512 posenet:512 deeplab:512 deeplab_fan:8 posenet_multi:64; do
  c=${spec%%:*}; B=${spec##*:}
  timeout -k 10 300 python bench.py --config $c --batch $B --steps 100 --warmup 20 --sweep "" > $O/cfg_${c}_b$B.json 2> $O/cfg_${c}_b$B.err
  echo "$c b$B $(grep -h -o '"value": [0-9.]*' $O/cfg_${c}_b$B.json) $(grep -h -o '"ms_per_step": [0-9.]*' $O/cfg_${c}_b$B.json)"
done
fi
if [ "${PART:-2}" = 2 ]; then
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > $O/layers_b512.txt 2>&1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $R/$O/prof_default -o run --output-format csv -- \
   python3 $R/bench.py --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/$O/prof_default.log 2>&1)
for spec in ssd:64 posenet:64 deeplab:8; do
  c=${spec%%:*}; B=${spec##*:}
  (cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof_${c}_b$B -o run --output-format csv -- \
     python3 $R/bench.py --config $c --batch $B --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/$O/prof_${c}_b$B.log 2>&1)
done
fi
echo done
)
;;
gpu_r5_pmc_early)
(
# PMC of the stem and the early fused blocks at batch 512 (HEAD defaults) + the layer table (round 5)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 scripts/bench_ir_f32.py 512 > gpurun_out/r5_layers_pmc_run.txt 2>&1 || { echo "layers failed"; exit 1; }
grep -E "fused|stem|TOTAL|head|chain" gpurun_out/r5_layers_pmc_run.txt | head -30
rm -f gpurun_out/pmc_early_all.txt
for S in stem "112,16,96,24,2" "56,24,144,24,1" "56,24,144,32,2" "28,32,192,32,1" "14,64,384,64,1"; do
  n=$(echo $S | tr ',' '_')
  OUT=gpurun_out/pmc_fin_$n SHAPE=$S B=512 bash scripts/pmc_f32.sh > gpurun_out/pmc_fin_$n.txt 2>&1 || { echo "pmc $S failed"; tail -5 gpurun_out/pmc_fin_$n.txt; exit 1; }
  cat gpurun_out/pmc_fin_$n.txt >> gpurun_out/pmc_early_all.txt
done
cat gpurun_out/pmc_early_all.txt
)
;;
gpu_r5_pmc_gemm)
(
# PMC of the fp32 GEMM, x3 (pre-split weights) vs native, on the chain / PoseNet shapes
set -eo pipefail
:
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES"
P3="FETCH_SIZE"
P4="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_ANY SQ_INSTS_VALU_MFMA_F32 SQ_INSTS_VALU_MFMA_BF16"
for spec in ${SPECS:-25088,960,320,x3,128064 25088,960,320,fp32,128064 18496,1024,1024,x3,64064}; do
  IFS=, read M K N meth tile <<< "$spec"
  OUT=gpurun_out/pmc_gemm_${M}_${K}_${N}_${meth}_${tile}
  mkdir -p $OUT
  i=0
  for P in "$P1" "$P2" "$P3" "$P4"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $P -d $OUT/p$i -o p$i --output-format csv -- python3 scripts/gemm_one.py $M $K $N $meth $tile 10 > $OUT/p$i.log 2>&1
  done
  echo "== $spec"
  python3 scripts/pmc_report.py $OUT pw_gemm
done
)
;;
gpu_r6_check)
(
# Round-6 GPU check: comm tests (forced one-rank RCCL rounds), the 14x14 irp kernel's
# accuracy gate, the load-time lowering tests, per-layer A/B (NNSX_IRP=0 / 1) at batch
# 512, then the default bench and the lowered-plain-model bench.
set -eo pipefail
:
O=gpurun_out/r6check
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_comm.py tests/test_gpu_rccl_ranks.py -x -q --timeout 120 --timeout-method thread > $O/comm_tests.txt 2>&1 || { tail -30 $O/comm_tests.txt; exit 1; }
tail -2 $O/comm_tests.txt
timeout -k 10 400 python -u -m pytest tests/test_gpu_irp.py tests/test_gpu_lowering.py -q --timeout 200 --timeout-method thread > $O/irp_low_tests.txt 2>&1 || true
tail -25 $O/irp_low_tests.txt
for f in 14,64,384,64,1 14,64,384,96,1 14,96,576,96,1; do
  NNSX_IR_ONLY=$f NNSX_IRP=0 timeout -k 10 120 python -u scripts/bench_ir_f32.py 512 2>&1 | grep -v amdgpu.ids >> $O/layers_irp0.txt
  NNSX_IR_ONLY=$f NNSX_IRP=1 timeout -k 10 120 python -u scripts/bench_ir_f32.py 512 2>&1 | grep -v amdgpu.ids >> $O/layers_irp1.txt
done
cat $O/layers_irp0.txt $O/layers_irp1.txt | grep fused
timeout -k 10 400 python bench.py --sweep "" > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-300
NNSX_IRP=0 timeout -k 10 400 python bench.py --sweep "" --latency-frames 0 > $O/bench_irp0.json 2> $O/bench_irp0.err
tail -1 $O/bench_irp0.json | cut -c1-200
timeout -k 10 400 python bench.py --engine lowered --sweep "" --latency-frames 0 > $O/bench_lowered.json 2> $O/bench_lowered.err
tail -1 $O/bench_lowered.json | cut -c1-200
)
;;
gpu_session)
(
# One GPU-box session.  Each GPU step has its own time limit; the first failing
# step ends the session (no retries).  STEPS: comma list of
#   f32      new fp32 kernel tests            (tests/test_gpu_mbv2_f32.py)
#   test     the whole GPU suite
#   smoke    __graft_entry__.smoke()
#   bench    bench.py (BENCH_ARGS)
#   prof     rocprofv3 kernel stats of bench.py (PROF_ARGS)
#   irf32    per-layer fp32 engine micro-benchmark (scripts/bench_ir_f32.py)
#   latprof  rocprofv3 host+device trace of the batch-1 latency run
#   irvar    bench_ir_f32 once per IR_VARIANTS env set
#   pmcf32   PMC counter passes over it (scripts/pmc_f32.sh; SHAPE=, KERNEL=)
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${STEPS:-f32,test,smoke,bench}
R=$GRAFT_REPO_ROOT
[ -z "$R" ] && R=$(pwd)
for s in ${STEPS//,/ }; do
  case $s in
    f32)
      timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_f32.log 2>&1 || { echo "f32 tests failed"; tail -60 gpurun_out/pytest_f32.log; exit 1; }
      tail -3 gpurun_out/pytest_f32.log ;;
    test)
      timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { echo "gpu tests failed"; tail -60 gpurun_out/pytest_gpu.log; exit 1; }
      tail -3 gpurun_out/pytest_gpu.log ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || { echo "smoke failed"; tail -30 gpurun_out/smoke.log; exit 1; }
      tail -2 gpurun_out/smoke.log ;;
    bench)
      timeout -k 10 600 python bench.py ${BENCH_ARGS} > gpurun_out/bench.log 2>&1 || { echo "bench failed"; tail -40 gpurun_out/bench.log; exit 1; }
      tail -1 gpurun_out/bench.log ;;
    prof)
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $R/gpurun_out/prof -o run --output-format csv -- python3 $R/bench.py ${PROF_ARGS} > $R/gpurun_out/prof.log 2>&1) || { echo "prof failed"; tail -30 gpurun_out/prof.log; exit 1; }
      find gpurun_out/prof -name "*kernel_stats.csv" ;;
    latprof)
      # host (HIP API) + device timeline of the batch-1 latency run
      (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --hip-trace --memory-copy-trace -d $R/gpurun_out/latprof -o run --output-format csv -- python3 $R/bench.py --precision fp32 --steps 3 --warmup 2 --latency-frames 200 > $R/gpurun_out/latprof.log 2>&1) || { echo "latprof failed"; tail -30 gpurun_out/latprof.log; exit 1; }
      tail -1 gpurun_out/latprof.log | cut -c1-300 ;;
    irf32)
      timeout -k 10 300 python -u scripts/bench_ir_f32.py ${IR_B:-128} > gpurun_out/bench_ir_f32.log 2>&1 || { echo "bench_ir_f32 failed"; tail -30 gpurun_out/bench_ir_f32.log; exit 1; }
      cat gpurun_out/bench_ir_f32.log ;;
    irvar)
      # IR_VARIANTS: ';'-separated env assignments, one bench_ir_f32 run each
      IFS=';' read -ra VARS <<< "${IR_VARIANTS:-NNSX_F32_IRW=1}"
      for V in "${VARS[@]}"; do
        env $V timeout -k 10 300 python -u scripts/bench_ir_f32.py ${IR_B:-128} > gpurun_out/irvar.log 2>&1 || { echo "irvar $V failed"; tail -30 gpurun_out/irvar.log; exit 1; }
        echo "== $V"; grep -v amdgpu.ids gpurun_out/irvar.log
      done ;;
    gemmf32)
      for R in ${DW_ROWS:-4}; do
        NNSX_F32_DW_ROWS=$R timeout -k 10 300 python -u scripts/bench_gemm_f32.py ${IR_B:-128} > gpurun_out/bench_gemm_f32_r$R.log 2>&1 || { echo "bench_gemm_f32 failed"; tail -30 gpurun_out/bench_gemm_f32_r$R.log; exit 1; }
        echo "== dw rows $R"; cat gpurun_out/bench_gemm_f32_r$R.log
      done ;;
    pmcf32)
      timeout -k 10 600 bash scripts/pmc_f32.sh > gpurun_out/pmc_f32.log 2>&1 || { echo "pmc failed"; tail -30 gpurun_out/pmc_f32.log; exit 1; }
      cat gpurun_out/pmc_f32.log ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
)
;;
stem_ab)
(
# A/B of the fused stem + block-1 kernel variants (NNSX_STEM_WAVE) at batch 512.
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
for V in ${VARIANTS:-2 1}; do
  NNSX_STEM_WAVE=$V NNSX_IR_ONLY=stem timeout -k 10 120 python scripts/bench_ir_f32.py ${B:-512} > gpurun_out/stem_ab_$V.txt 2>&1 || { echo "stem variant $V failed"; tail -5 gpurun_out/stem_ab_$V.txt; exit 1; }
  echo "variant $V: $(grep stem gpurun_out/stem_ab_$V.txt)"
done
)
;;
gpu_r6_irw2)
(
# irw_f32 stride-2 tiles with per-quad hidden planes one cell apart (GSH): fp32 block numerics, per-block times at
# batch 512, LDS counters of the 56 -> 28 and 112 -> 56 blocks, the headline bench.
#   scripts/gpu_drivers.sh gpu_r6_irw2 [outdir]
set -eo pipefail
O=${1:-gpurun_out/r6irw2}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_x3.py tests/test_gpu_models_f32.py -q -x --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
tail -1 $O/tests.txt
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > $O/layers_b512.txt 2>&1
grep -E "H=112|H=56|TOTAL" $O/layers_b512.txt
for spec in "56,24,144,32,2 irw_f32" "112,16,96,24,2 irw_f32"; do
  set -- $spec
  tag=$(echo "$1_$2" | tr ',' '_')
  OUT=$O/$tag SHAPE=$1 B=512 KERNEL=$2 bash scripts/pmc_f32.sh > $O/$tag.txt 2>&1
  echo "== $1 $2"; tail -2 $O/$tag.txt
done
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-300; echo
)
;;
gpu_r6_midsplit)
(
# Split-K for mid-size GEMM grids (NNSX_GEMM_MIDSPLIT=1: 128-511 tiles in two k-slices, residual added by the reduce):
# fp32 numerics under the switch, then each config with it off / on (DeepLab b8's 8712 x 960 -> 160 projects).
#   scripts/gpu_drivers.sh gpu_r6_midsplit [outdir]
set -eo pipefail
O=${1:-gpurun_out/r6mid}
mkdir -p $O
export TMPDIR=/tmp
NNSX_GEMM_MIDSPLIT=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_x3.py tests/test_gpu_models_f32.py tests/test_gpu_decode_stage.py -q -x --timeout 300 --timeout-method thread > $O/tests_mid.txt 2>&1
tail -1 $O/tests_mid.txt
for rep in 1 2; do
  for c in "deeplab 8" "ssd 64" "posenet 64"; do
    set -- $c
    for m in 0 1; do
      NNSX_GEMM_MIDSPLIT=$m timeout -k 10 300 python bench.py --config $1 --batch $2 --steps 200 --warmup 30 --sweep "" > $O/${1}_m${m}_r${rep}.json 2> $O/${1}_m${m}_r${rep}.err
      echo "$1 b$2 mid=$m rep $rep $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/${1}_m${m}_r${rep}.json | tr '\n' ' ')"
    done
  done
done
)
;;
gpu_r6_parts)
(
# Hidden-channel parts of the wave-split kernels on 128-255 tiles (NNSX_IRW_PARTS_MID=2 default / 3 / 4): DeepLab b8's 33x33
# blocks (200 tiles, 400 workgroups at 2 parts).  Numerics under 4 parts first.
#   scripts/gpu_drivers.sh gpu_r6_parts [outdir]
set -eo pipefail
O=${1:-gpurun_out/r6parts}
mkdir -p $O
export TMPDIR=/tmp
NNSX_IRW_PARTS_MID=4 timeout -k 10 600 python -u -m pytest tests/test_gpu_mbv2_f32.py tests/test_gpu_models_f32.py tests/test_gpu_decode_stage.py -q -x --timeout 300 --timeout-method thread > $O/tests_p4.txt 2>&1
tail -1 $O/tests_p4.txt
for rep in 1 2; do
  for p in 2 4 3; do
    NNSX_IRW_PARTS_MID=$p timeout -k 10 300 python bench.py --config deeplab --batch 8 --steps 200 --warmup 30 --sweep "" > $O/dl_p${p}_r${rep}.json 2> $O/dl_p${p}_r${rep}.err
    echo "deeplab b8 parts=$p rep $rep $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/dl_p${p}_r${rep}.json | tr '\n' ' ')"
  done
done
)
;;
gpu_r6_lanes)
(
# DeepLab b8 with its absorbed segmentation stage on 1 / 2 / 3 replay lanes (the stage writes only its output
# frames: DecodeStage::lane_safe), byte-exact check of the lanes against the decoder's own kernels first.
#   scripts/gpu_drivers.sh gpu_r6_lanes [outdir]
set -eo pipefail
O=${1:-gpurun_out/r6lanes}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_decode_stage.py -q --timeout 200 --timeout-method thread > $O/decode_stage.txt 2>&1
tail -1 $O/decode_stage.txt
for rep in 1 2; do
  for l in 1 2 3; do
    NNSX_TORCH_LANES=$l timeout -k 10 300 python bench.py --config deeplab --batch 8 --steps 200 --warmup 30 --sweep "" \
      > $O/deeplab_b8_l${l}_$rep.json 2> $O/deeplab_b8_l${l}_$rep.err
    echo "lanes $l rep $rep $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/deeplab_b8_l${l}_$rep.json | tr '\n' ' ')"
  done
done
)
;;
gpu_r6_irw7)
(
# irw_x3 7 x 7 tiles with the kIrw7Px / kIrw7Dc pixel assignment: x3 numerics, per-block times, LDS counters, headline.
set -eo pipefail
O=gpurun_out/r6irw7; mkdir -p $O; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_x3.py tests/test_gpu_models_f32.py tests/test_gpu_mbv2_f32.py -q -x --timeout 300 --timeout-method thread > $O/tests.txt 2>&1
tail -1 $O/tests.txt
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > $O/layers_b512.txt 2>&1
grep -E "H=7 |TOTAL" $O/layers_b512.txt
OUT=$O/p7 SHAPE=7,160,960,160,1 B=512 KERNEL=irw_x3 bash scripts/pmc_f32.sh > $O/p7.txt 2>&1
tail -2 $O/p7.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-200; echo
)
;;
gpu_r6_ab2)
(
# After the LDS layouts: irp variants per 14x14 block again (pipelined / tiles per wave), and a sustained
# 1000-step headline with every invoke's device time (NNSX_BENCH_SERIES=1).
set -eo pipefail
O=${1:-gpurun_out/r6ab2}
mkdir -p $O
export TMPDIR=/tmp
for v in "NNSX_NONE=1" "NNSX_IRP_PIPE=1" "NNSX_IRP_PIPE=0" "NNSX_IRP_TPW=1" "NNSX_IRP_PIPE=1 NNSX_IRP_TPW=1"; do
  tag=$(echo "$v" | tr ' =' '__')
  env $v NNSX_IR_ONLY=14,64,384,64,1 timeout -k 10 120 python -u scripts/bench_ir_f32.py 512 > $O/l_a_$tag.txt 2>&1
  env $v NNSX_IR_ONLY=14,64,384,96,1 timeout -k 10 120 python -u scripts/bench_ir_f32.py 512 > $O/l_b_$tag.txt 2>&1
  env $v NNSX_IR_ONLY=14,96,576,96,1 timeout -k 10 120 python -u scripts/bench_ir_f32.py 512 > $O/l_c_$tag.txt 2>&1
  echo "$v | $(grep -h 'fused' $O/l_a_$tag.txt $O/l_b_$tag.txt $O/l_c_$tag.txt | awk '{print $2, $3, $4}' | tr '\n' ' ')"
done
NNSX_BENCH_SERIES=1 timeout -k 10 400 python bench.py --steps 1000 --warmup 20 --sweep "" --latency-frames 0 > $O/bench_1000.json 2> $O/bench_1000.err
tail -1 $O/bench_1000.json | grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"gpu_invoke_ms_median": [0-9.]*' | tr '\n' ' '; echo
)
;;
list) echo blaslt_probe gpu_ab_variant gpu_b1_combine_ab gpu_b1_lat_ab gpu_b1_prof gpu_b1_upload_ab gpu_config_traces gpu_final_check gpu_host_argmax_ab gpu_pipe_ab gpu_pmc_early gpu_r3_hiptrace gpu_r4_b512cfg gpu_r4_cfgprof gpu_r4_configs gpu_r4_dllanes gpu_r4_dwdil gpu_r4_dwnew gpu_r4_dwsweep gpu_r4_final gpu_r4_heads gpu_r4_lanes512 gpu_r4_mbv2_ab gpu_r4_pmc gpu_r4_posehead gpu_r4_prof gpu_r4_small gpu_r4_ssd5 gpu_r4_stage gpu_r4_stem gpu_r5_final gpu_r5_pmc_early gpu_r5_pmc_gemm gpu_r6_ab2 gpu_r6_check gpu_r6_irw2 gpu_r6_irw7 gpu_r6_lanes gpu_r6_midsplit gpu_r6_parts gpu_session stem_ab ;;
*) echo "usage: $0 <name> [args]; names: blaslt_probe gpu_ab_variant gpu_b1_combine_ab gpu_b1_lat_ab gpu_b1_prof gpu_b1_upload_ab gpu_config_traces gpu_final_check gpu_host_argmax_ab gpu_pipe_ab gpu_pmc_early gpu_r3_hiptrace gpu_r4_b512cfg gpu_r4_cfgprof gpu_r4_configs gpu_r4_dllanes gpu_r4_dwdil gpu_r4_dwnew gpu_r4_dwsweep gpu_r4_final gpu_r4_heads gpu_r4_lanes512 gpu_r4_mbv2_ab gpu_r4_pmc gpu_r4_posehead gpu_r4_prof gpu_r4_small gpu_r4_ssd5 gpu_r4_stage gpu_r4_stem gpu_r5_final gpu_r5_pmc_early gpu_r5_pmc_gemm gpu_r6_ab2 gpu_r6_check gpu_r6_irw2 gpu_r6_irw7 gpu_r6_lanes gpu_r6_midsplit gpu_r6_parts gpu_session stem_ab" >&2; exit 2 ;;
esac
