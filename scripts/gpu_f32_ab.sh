set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_models_f32.py tests/test_gpu_mbv2_f32.py > gpurun_out/t_f32.txt 2>&1 && tail -3 gpurun_out/t_f32.txt && \
timeout -k 10 300 python scripts/bench_ir_f32.py 512 > gpurun_out/layers_new.txt 2>&1 && cat gpurun_out/layers_new.txt | grep -v amdgpu.ids && \
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench_new.json 2> gpurun_out/bench_new.err && cut -c1-400 gpurun_out/bench_new.json
