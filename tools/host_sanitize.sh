#!/usr/bin/env bash
# Build csrc/host/host_check.hip with ASan + UBSan on the host half (gfx950 device half unsanitised:
# GPU ASan is not available on this pool) and run its self-test.  CPU only; no GPU is touched.
# Usage: tools/host_sanitize.sh [out_dir]   (default build/host)
set -euo pipefail
ROOT="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-$ROOT/build/host}"
mkdir -p "$OUT"
"${ROCM_PATH:-/opt/rocm}/bin/hipcc" --offload-arch=gfx950 -O1 -g -fno-omit-frame-pointer \
  -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
  -Xarch_host -fno-sanitize-recover=undefined -I "$ROOT/csrc" \
  "$ROOT/csrc/host/host_check.hip" -o "$OUT/host_check"
ASAN_OPTIONS="detect_leaks=0:abort_on_error=0" UBSAN_OPTIONS="print_stacktrace=1" "$OUT/host_check" selftest
