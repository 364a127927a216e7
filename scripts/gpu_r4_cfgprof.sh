#!/bin/bash
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
