#!/bin/bash
# why is the unprofiled 100-step bench slower than the profiled 20-step one?  Per-invoke device ms series
# (NNSX_BENCH_SERIES=1) for 100/20 and 20/5 runs, with and without rocprofv3 --kernel-trace, and variants.
set -eo pipefail
cd "$(dirname "$0")/.."
O=${1:-gpurun_out/r6slow}
mkdir -p $O
export NNSX_BENCH_SERIES=1 TMPDIR=/tmp
R=$PWD
run() {  # tag, env..., -- bench args
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --sweep "" --latency-frames 0 > $O/$tag.json 2> $O/$tag.err
  echo "$tag $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"gpu_invoke_ms_median": [0-9.]*' $O/$tag.json | tr '\n' ' ')"
}
run a_default NNSX_NONE=1
run b_irh0_terms0 NNSX_IRH=0 NNSX_IRPS_TERMS=0
run c_irp0 NNSX_IRP=0
(cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $R/$O/prof100 -o run --output-format csv -- \
   python3 $R/bench.py --sweep "" --latency-frames 0 > $R/$O/prof100.json 2> $R/$O/prof100.err)
echo "prof100 $(grep -o '"value": [0-9.]*\|"ms_per_step": [0-9.]*\|"gpu_invoke_ms_median": [0-9.]*' $O/prof100.json | tr '\n' ' ')"
run d_default_again NNSX_NONE=1
grep -h "device ms per invoke" $O/*.err | cut -c1-400
