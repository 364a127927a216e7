#!/bin/bash
# PMC of the round-6 image-per-workgroup kernels at batch 512 (scripts/pmc_f32.sh per block; 4 passes each) and
# of the wave-split kernel they replaced on one shape.
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6pmc}
mkdir -p $O
for spec in "14,64,384,64,1 irp_x3 NNSX_NONE=1" "14,96,576,96,1 irpp_x3 NNSX_NONE=1" "14,96,576,160,2 irps_x3 NNSX_NONE=1" \
            "28,32,192,32,1 irh_x3 NNSX_NONE=1" "28,32,192,64,2 irh_x3 NNSX_NONE=1" "14,64,384,64,1 irw NNSX_IRP=0"; do
  set -- $spec
  tag=$(echo "$1_$2" | tr ',' '_')
  env $3 OUT=$O/$tag SHAPE=$1 B=512 KERNEL=$2 bash scripts/pmc_f32.sh > $O/$tag.txt 2>&1
  echo "== $1 $2 ($3)"; tail -4 $O/$tag.txt
done
