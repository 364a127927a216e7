#!/bin/bash
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
