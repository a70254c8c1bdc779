#!/bin/bash
# Build the native env runtime + fuzz driver with ASan/UBSan (host code only) and run it.
set -euo pipefail
ROOT=$(cd "$(dirname "$0")/../.." && pwd)
OUT=${1:-/tmp/ia_env_fuzz}
/opt/rocm/bin/hipcc -O1 -g -std=c++17 -fsanitize=address,undefined -fno-gpu-sanitize -fno-omit-frame-pointer \
  -I"$ROOT/csrc/include" -I"$ROOT/csrc/runtime" \
  "$ROOT/tools/sanitize/env_fuzz.cpp" "$ROOT/csrc/runtime/vec_env.cpp" -o "$OUT"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 UBSAN_OPTIONS=halt_on_error=1:print_stacktrace=1 "$OUT" "${2:-600}"
