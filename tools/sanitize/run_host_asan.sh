#!/bin/bash
# Build the runtime's host-side native code with AddressSanitizer + UndefinedBehaviorSanitizer (host side only:
# each sanitizer flag follows -Xarch_host, so no device code is instrumented) and run the host driver on the CPU.
# Usage: bash tools/sanitize/run_host_asan.sh [outdir]
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/../.." && pwd)"
OUT="${1:-/tmp/dtf_host_asan}"
mkdir -p "$OUT"
HIPCC="${HIPCC:-/opt/rocm/bin/hipcc}"
SAN=(-Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined -Xarch_host -fno-sanitize-recover=all
     -Xarch_host -fno-omit-frame-pointer)
"$HIPCC" -O1 -g -std=c++17 "${SAN[@]}" -x c++ "$ROOT/distributedtf_amd/ops/csrc/host.hip" \
    "$ROOT/tools/sanitize/host_check.cpp" -o "$OUT/host_check"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=0 UBSAN_OPTIONS=print_stacktrace=1 "$OUT/host_check" "${@:2}"
