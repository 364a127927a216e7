#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer build of the host runtime (the
# same translation units and driver as scripts/tsan_check.sh: no libtorch /
# pybind sources, tests/native/tsan_main.cc runs the pipelines on the host).
# Device code is compiled without sanitizers (-fsanitize only after
# -Xarch_host).  Exit 67 = an ASan/UBSan report.
set -e -o pipefail
ROOT=$(cd "$(dirname "$0")/.." && pwd)
OUT=${ASAN_BUILD:-/tmp/nnsx_asan}
mkdir -p "$OUT"
CXX=/opt/rocm/lib/llvm/bin/clang++
HIPCC=/opt/rocm/bin/hipcc
SAN="-fsanitize=address,undefined -fno-sanitize=vptr -fno-omit-frame-pointer"
FLAGS="-O1 -g -fPIC -std=c++17 -I$ROOT/csrc -I$ROOT/include -D__HIP_PLATFORM_AMD__=1 -isystem /opt/rocm/include -w"
SKIP="filter/pytorch.cc filter/torch_trainer.cc ops/torch_ops.cc bindings/module.cc bindings/python_bridge.cc tools/tool_main.cc"
objs=()
jobs=0
cd "$ROOT/csrc"
for f in $(find . -name '*.cc' -o -name '*.hip' | sed 's|^\./||' | sort); do
  case " $SKIP " in *" $f "*) continue;; esac
  o="$OUT/$(echo "$f" | tr / _).o"
  objs+=("$o")
  if [ "$f" -nt "$o" ] || [ ! -f "$o" ]; then
    if [[ $f == *.hip ]]; then
      $HIPCC -x hip --offload-arch=gfx950 $FLAGS -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
        -Xarch_host -fno-sanitize=vptr -c "$f" -o "$o" &
    else
      $CXX $FLAGS $SAN -c "$f" -o "$o" &
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
$CXX $FLAGS $SAN -c "$OUT/stubs.cc" -o "$OUT/stubs.o"
$CXX $FLAGS $SAN -c "$ROOT/tests/native/tsan_main.cc" -o "$OUT/san_main.o"
$CXX $SAN "${objs[@]}" "$OUT/stubs.o" "$OUT/san_main.o" -o "$OUT/san_main" \
  -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib -lrccl -lrocprofiler-sdk-roctx -lamdhip64 -ldl -lpthread
cd "$ROOT"
# leak checking is off: the registries are process-lifetime singletons by design
NNSX_DISABLE_GPU=1 ASAN_OPTIONS="detect_leaks=0 exitcode=67 abort_on_error=0" \
  UBSAN_OPTIONS="print_stacktrace=1 halt_on_error=1 exitcode=67" timeout 900 "$OUT/san_main"
