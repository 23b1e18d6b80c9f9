#!/bin/bash
# Host-side sanitizer pass over the CPU checker: rebuild oracle/liborc.so with
# ASan + UBSan, run tests/test_oracle.py against it, restore the optimised build.
set -e
cd "$(dirname "$0")/.."
tmp=$(mktemp -d)
gcc -O1 -g -std=c11 -fPIC -shared -fsanitize=address,undefined -fno-omit-frame-pointer -D_GNU_SOURCE \
    oracle/inccl_oracle.c -o "$tmp/liborc.so" -lm
cp oracle/liborc.so "$tmp/liborc_opt.so"
cp "$tmp/liborc.so" oracle/liborc.so
trap 'cp "$tmp/liborc_opt.so" oracle/liborc.so; rm -rf "$tmp"' EXIT
LD_PRELOAD="$(gcc -print-file-name=libasan.so) $(gcc -print-file-name=libubsan.so)" \
ASAN_OPTIONS=detect_leaks=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1 \
    python -m pytest tests/test_oracle.py -q
