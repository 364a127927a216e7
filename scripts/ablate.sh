for A in 0 1 2 4 8 16 6 31; do echo "ablate $A"; NNSX_ABLATE=$A timeout -k 10 120 python -u scripts/bench_ir_f32.py 128 2>&1 | grep "stem+block1"; done
