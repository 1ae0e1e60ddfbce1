#!/bin/bash
# The CPU suite (pytest -m "not gpu", which includes the mutation fuzz of
# tests/test_fuzz_inputs.py) against the AddressSanitizer + UBSan build of the library
# (make -C fhe-regex_amd asan).  The python interpreter is not instrumented,
# so the clang ASan runtime is preloaded; leak checking is off (the interpreter's own
# allocations at exit are not ours); any ASan or UBSan report aborts the test run.
#   bash tools/asan_check.sh LOGFILE [pytest args]      (CPU only: run it in this container)
set -o pipefail
cd "$(dirname "$0")/.."
log=${1:-profiles/asan_check.log}
shift
make -C fhe-regex_amd asan -j8 > /dev/null || exit 1
RT=$(/opt/rocm/llvm/bin/clang++ -print-file-name=libclang_rt.asan-x86_64.so)
rep=/tmp/fr_sanitizer_report
rm -f "$rep".*
{
  echo "# $(date -u +%FT%TZ) sanitized library: fhe-regex_amd/build-asan/libfheregex.so ($(git rev-parse --short HEAD))"
  echo "# runtime: $RT"
  echo "# ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1"
  echo "# (reports are written to $rep.<pid> and appended below; none means clean)"
  LD_PRELOAD=$RT ASAN_OPTIONS=detect_leaks=0:halt_on_error=1:abort_on_error=1:log_path=$rep \
    UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1:log_path=$rep FHEREGEX_LIB=fhe-regex_amd/build-asan/libfheregex.so \
    python -m pytest tests -m "not gpu" -q -p no:cacheprovider "$@" 2>&1
} > "$log"
rc=$?
if ls "$rep".* > /dev/null 2>&1; then
  { echo "# ---- sanitizer reports ----"; cat "$rep".*; } >> "$log"
  rc=1
else
  echo "# sanitizer reports: none" >> "$log"
fi
grep -E "ERROR: AddressSanitizer|runtime error:|passed|failed" "$log" | tail -5
exit $rc
