#!/bin/bash
# Host AddressSanitizer + UBSan check of libadmmq's host code, no GPU needed:
# builds build/asan/libadmmq_asan.so (-Xarch_host -fsanitize=address,undefined) and runs
# tools/asan_host_check.c over the C3 / C5 plans, 400 random batches and the argument checks.
# Leak detection is off: the HIP runtime's process-lifetime allocations are not ours.
cd "$(dirname "$0")/.." || exit 1
make -s -C admm-quantization_amd/csrc -j8 asan || exit $?
ASAN_OPTIONS=detect_leaks=0:abort_on_error=1 UBSAN_OPTIONS=print_stacktrace=1 build/asan/asan_host_check
