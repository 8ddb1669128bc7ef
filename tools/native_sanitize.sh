#!/bin/bash
# Host-side sanitizer runs of the native runtime (csrc/native) through a standalone self-test:
# AddressSanitizer + UndefinedBehaviorSanitizer, then ThreadSanitizer (the threaded prefetcher).
# GPU sanitizers (ASan / XNACK code objects) are unavailable on the MI355X pool by policy.
set -e
R="$(cd "$(dirname "$0")/.." && pwd)"
OUT="${1:-/tmp/dtf_sanitize}"
mkdir -p "$OUT"
SRC="$R/csrc/native/crc32c.cpp $R/csrc/native/records.cpp $R/csrc/native/bundle.cpp $R/csrc/native/data.cpp $R/csrc/native/test/selftest.cpp"
g++ -std=c++17 -O1 -g -msse4.2 -pthread -fno-omit-frame-pointer -fsanitize=address,undefined \
    -fno-sanitize-recover=all $SRC -o "$OUT/selftest_asan"
ASAN_OPTIONS=detect_leaks=1:abort_on_error=1 "$OUT/selftest_asan" "$OUT"
g++ -std=c++17 -O1 -g -msse4.2 -pthread -fsanitize=thread $SRC -o "$OUT/selftest_tsan"
TSAN_OPTIONS=halt_on_error=1 "$OUT/selftest_tsan" "$OUT"
echo "sanitizers clean"
