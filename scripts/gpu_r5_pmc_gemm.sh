#!/bin/bash
# PMC of the fp32 GEMM, x3 (pre-split weights) vs native, on the chain / PoseNet shapes
set -eo pipefail
cd "$(dirname "$0")/.."
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
