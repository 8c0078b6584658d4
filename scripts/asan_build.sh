#!/bin/bash
# CPU-only AddressSanitizer + UndefinedBehaviorSanitizer build of the C ABI's host
# code: every csrc/*.hip translation unit is compiled with the sanitizers
# on its HOST half only (-Xarch_host; GPU sanitizers are not used on this pool) and
# linked with scripts/asan_plans.cpp into build/asan/asan_plans, which exercises plan
# creation, the flat parameter layout, workspace sizing and saved-tensor lookups for
# every BASELINE shape without touching a GPU.  Usage: scripts/asan_build.sh [--run]
set -eu
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
PKG="$ROOT/spff-unet-spcct_amd"
OUT="$PKG/build/asan"
mkdir -p "$OUT"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
SAN="-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=undefined -Xarch_host -fno-omit-frame-pointer"
FLAGS="-O1 -g -std=c++17 -fPIC --offload-arch=gfx950 -I$ROOT/include -I$PKG/csrc -Wno-unused-result"
pids=()
# the newest header any translation unit may include (csrc/*.h, include/*.h): an object
# older than it is rebuilt, so a header edit never leaves stale sanitizer objects
newest_h="$(ls -t "$PKG"/csrc/*.h "$ROOT"/include/*.h | head -1)"
for src in "$PKG"/csrc/*.hip; do
  obj="$OUT/$(basename "${src%.hip}").o"
  if [ ! -f "$obj" ] || [ "$src" -nt "$obj" ] || [ "$newest_h" -nt "$obj" ]; then
    $HIPCC $FLAGS $SAN -c "$src" -o "$obj" &
    pids+=($!)
  fi
done
for p in "${pids[@]}"; do wait "$p"; done
# the driver is plain host C++ (no HIP): amdclang++, then one hipcc link of everything
/opt/rocm/llvm/bin/clang++ -O1 -g -std=c++17 -I"$ROOT/include" -fsanitize=address,undefined \
  -fno-sanitize-recover=undefined -fno-omit-frame-pointer -c "$ROOT/scripts/asan_plans.cpp" \
  -o "$OUT/asan_plans.main.o"
$HIPCC -fsanitize=address,undefined --offload-arch=gfx950 "$OUT"/*.o -o "$OUT/asan_plans"
echo "built $OUT/asan_plans"
if [ "${1:-}" = "--run" ]; then
  ASAN_OPTIONS="${ASAN_OPTIONS:-detect_leaks=1:abort_on_error=0:halt_on_error=1}" \
  LSAN_OPTIONS="suppressions=$ROOT/scripts/asan_runtime.supp:print_suppressions=0" \
  UBSAN_OPTIONS="print_stacktrace=1:halt_on_error=1" "$OUT/asan_plans"
fi
