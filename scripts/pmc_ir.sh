#!/bin/bash
# PMC counters for one fused ir_block shape (one pass per counter set).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc
SHAPE=${1:-56,24,144,24,1}
export NNSX_IR_ONLY=$SHAPE
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES"
i=0
for P in "$P1" "$P2"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $P -d gpurun_out/pmc/p$i -o p$i --output-format csv -- python3 scripts/bench_ir.py 256 > gpurun_out/pmc/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 gpurun_out/pmc/p$i.log; exit 1; }
done
python3 scripts/pmc_summary.py gpurun_out/pmc ir_block
