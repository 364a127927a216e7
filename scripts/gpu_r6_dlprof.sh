#!/bin/bash
# DeepLab b8 kernel time per step in the timed window (rocprofv3 --kernel-trace --marker-trace, scripts/kstats.py --window).
#   scripts/gpu_r6_dlprof.sh [outdir]
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6dl}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
timeout -k 10 300 python bench.py --config deeplab --batch 8 --steps 100 --warmup 20 --sweep "" > $O/bench.json 2> $O/bench.err
echo "no profiler: $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*' $O/bench.json | tr '\n' ' ')"
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d $R/$O/prof -o run --output-format csv -- \
   python3 $R/bench.py --config deeplab --batch 8 --steps 40 --warmup 10 --sweep "" --latency-frames 0 > $R/$O/prof.log 2>&1)
python3 scripts/kstats.py $O/prof --window --per-step 40 > $O/kstats_window.txt
head -40 $O/kstats_window.txt
