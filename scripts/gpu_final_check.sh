set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash scripts/gpu_round.sh test && \
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 && tail -2 gpurun_out/smoke.log && \
timeout -k 10 300 python bench.py > gpurun_out/bench_default.json 2> gpurun_out/bench_default.err && cut -c1-300 gpurun_out/bench_default.json
