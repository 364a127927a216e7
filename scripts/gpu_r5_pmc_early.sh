#!/bin/bash
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
