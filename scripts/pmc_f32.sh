#!/bin/bash
# PMC counters for the fp32 engine's layers (scripts/bench_ir_f32.py), one
# rocprofv3 pass per counter set.  SHAPE=H,cin,hid,cout,s limits it to one block.
set -o pipefail
export TMPDIR=/tmp
OUT=${OUT:-gpurun_out/pmc_f32}
mkdir -p $OUT
[ -n "$SHAPE" ] && export NNSX_IR_ONLY=$SHAPE
P1="SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES"
P2="SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVES SQ_BUSY_CYCLES"
P3="FETCH_SIZE"
P4="WRITE_SIZE"
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P -d $OUT/p$i -o p$i --output-format csv -- python3 scripts/bench_ir_f32.py ${B:-128} > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; exit 1; }
done
python3 scripts/pmc_report.py $OUT "${KERNEL:-}"
