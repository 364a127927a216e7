#!/bin/bash
# ThreadSanitizer build of the host runtime (no libtorch / pybind sources) +
# tests/native/tsan_main.cc; runs on a CPU-only host.  Exit 66 = races found.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${TSAN_BUILD:-/tmp/nnsx_tsan}
mkdir -p "$OUT"
CXX=/opt/rocm/lib/llvm/bin/clang++
HIPCC=/opt/rocm/bin/hipcc
FLAGS="-O1 -g -fPIC -std=c++17 -I$ROOT/csrc -I$ROOT/include -D__HIP_PLATFORM_AMD__=1 -isystem /opt/rocm/include -w"
SKIP="filter/pytorch.cc filter/torch_trainer.cc ops/torch_ops.cc bindings/module.cc bindings/python_bridge.cc"
objs=()
jobs=0
cd "$ROOT/csrc"
for f in $(find . -name '*.cc' -o -name '*.hip' | sed 's|^\./||' | sort); do
  case " $SKIP " in *" $f "*) continue;; esac
  o="$OUT/$(echo "$f" | tr / _).o"
  objs+=("$o")
  if [ "$f" -nt "$o" ] || [ ! -f "$o" ]; then
    if [[ $f == *.hip ]]; then
      $HIPCC -x hip --offload-arch=gfx950 $FLAGS -Xarch_host -fsanitize=thread -c "$f" -o "$o" &
    else
      $CXX $FLAGS -fsanitize=thread -c "$f" -o "$o" &
    fi
    jobs=$((jobs + 1))
    if [ $jobs -ge ${MAX_JOBS:-8} ]; then wait -n; jobs=$((jobs - 1)); fi
  fi
done
wait
cat > "$OUT/stubs.cc" <<'STUB'
// frameworks / bridges that live in the libtorch and pybind translation units
#include <string>
namespace nnsx {
void register_torch_frameworks() {}
void register_torch_trainer() {}
}
STUB
$CXX $FLAGS -fsanitize=thread -c "$OUT/stubs.cc" -o "$OUT/stubs.o"
$CXX $FLAGS -fsanitize=thread -c "$ROOT/tests/native/tsan_main.cc" -o "$OUT/tsan_main.o"
# host link (the fat objects register their device code through libamdhip64)
$CXX -fsanitize=thread "${objs[@]}" "$OUT/stubs.o" "$OUT/tsan_main.o" -o "$OUT/tsan_main" \
  -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -lamdhip64 -ldl -lpthread
cd "$ROOT"
NNSX_DISABLE_GPU=1 TSAN_OPTIONS="suppressions=$ROOT/scripts/tsan.supp second_deadlock_stack=1 exitcode=66" \
  timeout 600 "$OUT/tsan_main"
