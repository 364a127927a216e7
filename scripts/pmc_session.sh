set -o pipefail
OUT=gpurun_out/pmc_b3new SHAPE=56,24,144,24,1 KERNEL=irw bash scripts/pmc_f32.sh > gpurun_out/pmc_b3new.txt 2>&1 && \
OUT=gpurun_out/pmc_b3old SHAPE=56,24,144,24,1 KERNEL=ir_block NNSX_F32_IRW=0 bash scripts/pmc_f32.sh > gpurun_out/pmc_b3old.txt 2>&1 && \
OUT=gpurun_out/pmc_b12 SHAPE=14,96,576,96,1 KERNEL=irw bash scripts/pmc_f32.sh > gpurun_out/pmc_b12.txt 2>&1
cat gpurun_out/pmc_b3new.txt gpurun_out/pmc_b3old.txt gpurun_out/pmc_b12.txt
