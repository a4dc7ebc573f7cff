#!/bin/bash
# AddressSanitizer + UndefinedBehaviorSanitizer over the HOST code (SURVEY.md §5 "Race detection /
# sanitizers"): liblgx.so's host backend (csrc/lgx_env_host.cpp, the --sim_device=cpu step with its
# fixed-size per-env arrays) and the C oracle, built with -fsanitize=address,undefined (UBSan's
# -fsanitize=bounds checks the indexing of the fixed-size arrays inside the per-env structs, which
# ASan's object-granular redzones do not), then the CPU parity suites that drive them:
# tests/test_host_parity.py (golden replays, one-step oracle comparisons on plane / trimesh /
# heightfield, crowded contacts, 200-step trajectories, NaN guard, command curriculum, C1 training)
# and tests/test_oracle_golden.py. No GPU: this runs in the build container.
# Usage: bash tools/san/run_asan.sh [extra pytest args]   (report: build/asan/report.txt)
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=$ROOT/build/asan
mkdir -p "$OUT"
SAN="-fsanitize=address,undefined -fno-sanitize-recover=undefined -fno-omit-frame-pointer -g"
CSRC=$ROOT/legged_gym_custom_amd/csrc
# host backend (sanitized) + the product's HIP object (device code is not instrumented: GPU
# sanitizers are unavailable on this pool, and the host tests never launch it)
g++ -O1 -std=c++17 -fPIC -fopenmp -ffp-contract=off -fno-fast-math -Wall $SAN -c -o "$OUT/lgx_env_host.o" \
    "$CSRC/lgx_env_host.cpp"
hipcc --offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -c -o "$OUT/lgx_env_hip.o" "$CSRC/lgx_env.hip"
GOMP=$(g++ -print-file-name=libgomp.so)
g++ -shared -o "$OUT/liblgx.so" "$OUT/lgx_env_hip.o" "$OUT/lgx_env_host.o" $SAN -fopenmp "$GOMP" \
    -L/opt/rocm/lib -lamdhip64 -Wl,-rpath,/opt/rocm/lib
make -s -C "$ROOT/oracle" OUT="$OUT/liblgx_oracle.so" CFLAGS="-O1 -ffp-contract=off -fno-fast-math -fPIC -Wall -fopenmp $SAN"
ASAN_RT=$(gcc -print-file-name=libasan.so)
UBSAN_RT=$(gcc -print-file-name=libubsan.so)
cd "$ROOT"
# python itself is not instrumented: no leak checking (the interpreter's allocations are not ours)
LGX_LIB="$OUT/liblgx.so" LGX_ORACLE_LIB="$OUT/liblgx_oracle.so" LD_PRELOAD="$ASAN_RT:$UBSAN_RT" \
ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:log_path=$OUT/asan \
UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path=$OUT/ubsan \
OMP_NUM_THREADS=4 \
  python -m pytest tests/test_host_parity.py tests/test_oracle_golden.py -q -p no:cacheprovider "$@" \
  2>&1 | tee "$OUT/report.txt"
ls "$OUT"/asan.* "$OUT"/ubsan.* 2>/dev/null && { echo "sanitizer reports above"; exit 1; } || echo "no sanitizer reports"
