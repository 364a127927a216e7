#!/bin/bash
# Round-6 GPU evidence in one call: new GPU tests (irp gate, shared-ring ingest,
# lifetime mutations, TorchScript lowering), the per-shape x3 error table, the
# shared-ring ingest rate, the default bench, and the headline kernel stats
# windowed to the timed steps (roctx marks from tensor_sink, scripts/kstats.py --window).
#   scripts/gpu_r6_round.sh [outdir] [tests...]
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6}
shift || true
T=${@:-tests/test_gpu_irp.py tests/test_gpu_shm_ingest.py tests/test_gpu_memcheck.py tests/test_gpu_lowering.py}
mkdir -p $O
export TMPDIR=/tmp
R=$PWD
rc=0
timeout -k 10 600 python -u -m pytest $T -v -s --timeout 240 --timeout-method thread > $O/tests.txt 2>&1 || rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $O/tests.txt | tail -40
[ $rc -le 1 ] || exit $rc  # (assertion failures go on; a fault, abort or time limit ends the call)
timeout -k 10 300 python -u scripts/x3_error_table.py --batch 512 > $O/x3_error_table.txt 2>&1
tail -2 $O/x3_error_table.txt
timeout -k 10 300 python -u scripts/shm_ingest.py 8 8 32 > $O/shm_ingest.txt 2>&1
cat $O/shm_ingest.txt
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-300
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --marker-trace --stats -d $R/$O/prof -o run --output-format csv -- \
   python3 $R/bench.py --steps 20 --warmup 5 --sweep "" --latency-frames 0 > $R/$O/prof.log 2>&1)
python3 scripts/kstats.py $O/prof --window --per-step 20 > $O/kstats_window.txt
head -30 $O/kstats_window.txt
