#!/bin/bash
# ASan + UBSan run of the C++ CPU restatement (oracle/cpu_ref.cpp) under every CPU test that
# loads it.  The sanitizer build is loaded into the (uninstrumented) python through
# CPUREF_LIB with the ASan runtime preloaded; leak checking is off (the interpreter's own
# allocations are not ours), every UBSan report aborts.  CPU only (this container): GPU sanitizers
# are not available on the pool.  Log: profiles/r5/asan_cpu_ref.log
set -euo pipefail
cd "$(dirname "$0")/.."
make -C oracle asan
log=${ASAN_LOG:-profiles/r6/asan_cpu_ref.log}
mkdir -p "$(dirname "$log")"
{
  echo "# $(date -u +%FT%TZ)  $(g++ --version | head -1)"
  echo "# build: make -C oracle asan (-fsanitize=address,undefined -fno-sanitize-recover=undefined -O1 -g)"
  CPUREF_LIB=$PWD/oracle/lib/libcpuref_asan.so LD_PRELOAD=$(g++ -print-file-name=libasan.so) \
  ASAN_OPTIONS=detect_leaks=0 python -c "from oracle import cpu_ref; cpu_ref.load(); \
print('# loaded:', sorted({l.split()[-1] for l in open('/proc/self/maps') if 'asan' in l}))"
  CPUREF_LIB=$PWD/oracle/lib/libcpuref_asan.so \
  LD_PRELOAD=$(g++ -print-file-name=libasan.so) \
  ASAN_OPTIONS=detect_leaks=0:abort_on_error=1:halt_on_error=1 \
  UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
  OMP_NUM_THREADS=4 \
    python -m pytest -p no:cacheprovider -q -m "not gpu" tests/test_cpu_ref.py tests/test_semantics_cpu.py 2>&1 \
    && rc=0 || rc=$?
  echo "# pytest exit status: $rc"
  echo "$rc" > "$log.rc"
} > "$log" 2>&1 || true
tail -5 "$log"
rc=$(cat "$log.rc" 2>/dev/null || echo 1)
rm -f "$log.rc"
if grep -qE "ERROR: AddressSanitizer|runtime error:" "$log"; then echo "sanitizer reports found"; exit 1; fi
if [ "$rc" != 0 ]; then echo "the tests failed under the sanitizers (pytest exit $rc)"; exit 1; fi
echo "no sanitizer reports, tests passed"
