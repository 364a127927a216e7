#!/bin/bash
# LDS bank-conflict layouts of the image-per-workgroup kernels (kIrpRow 17, wsw-swizzled weight stages):
# accuracy gate, per-block times at batch 512, LDS counters of two blocks, the headline bench.
#   scripts/gpu_r6_lds.sh [outdir]
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6lds}
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_irp.py -q --timeout 200 --timeout-method thread > $O/irp_tests.txt 2>&1
tail -1 $O/irp_tests.txt
timeout -k 10 300 python -u scripts/bench_ir_f32.py 512 > $O/layers_b512.txt 2>&1
grep -E "H=14|H=28|TOTAL" $O/layers_b512.txt
# PMC blocks: "H,cin,hid,cout,s kernel" pairs separated by ';' (default: the three stride-1 kernels)
IFS=';' read -ra SPECS <<< "${PMC_SPECS:-14,64,384,64,1 irp_x3;14,96,576,96,1 irpp_x3;28,32,192,32,1 irh_x3}"
for spec in "${SPECS[@]}"; do
  set -- $spec
  tag=$(echo "$1_$2" | tr ',' '_')
  OUT=$O/$tag SHAPE=$1 B=512 KERNEL=$2 bash scripts/pmc_f32.sh > $O/$tag.txt 2>&1
  echo "== $1 $2"; tail -2 $O/$tag.txt
done
timeout -k 10 400 python bench.py > $O/bench_default.json 2> $O/bench_default.err
tail -1 $O/bench_default.json | cut -c1-300; echo
