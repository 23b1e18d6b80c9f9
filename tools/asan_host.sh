#!/bin/bash
# Host-side ASan + UBSan pass over the library's C code on the GPU box: the C
# host objects are rebuilt with -fsanitize=address,undefined (the HIP kernels
# are reused as built; GPU code is never sanitized here), linked into
# container_inc_amd/obj_asan/libinccl_amd_asan.so, and tests/c/host_stress.c
# (itself sanitized, so the runtime loads first without any preload) runs
# world 1, two local ranks, and two TCP-rendezvous processes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}" || exit 3
mkdir -p gpurun_out
CSRC=container_inc_amd/csrc
B=container_inc_amd/obj_asan
mkdir -p $B
SAN="-fsanitize=address,undefined -fno-omit-frame-pointer -g"
CF="-O1 -std=c11 -fPIC -Wall -D__HIP_PLATFORM_AMD__ -I/opt/rocm/include -Iinclude -I$CSRC $SAN"
for f in api bootstrap transport p2p ll mesh switch copypool hostdma; do
  gcc $CF -c $CSRC/$f.c -o $B/$f.o || exit 4
done
# linked by gcc, whose sanitizer runtime the host objects were built for; the
# HIP objects carry their device code and registration constructors themselves
gcc -shared -fPIC $SAN -o $B/libinccl_amd_asan.so $B/*.o $CSRC/obj/inccl_*.o \
  -Wl,--version-script=$CSRC/exports.map -L/opt/rocm/lib -Wl,-rpath,/opt/rocm/lib \
  -lamdhip64 -lrccl -lstdc++ -lpthread -lm -lrt || exit 5
gcc -O1 -g -std=c11 $SAN -Iinclude tests/c/host_stress.c -o $B/host_stress -L$B -linccl_amd_asan -lpthread \
  -Wl,-rpath,$(pwd)/$B || exit 6
[ -n "$BUILD_ONLY" ] && exit 0
export ASAN_OPTIONS=detect_leaks=0:abort_on_error=0:use_sigaltstack=0 UBSAN_OPTIONS=print_stacktrace=1:halt_on_error=1
N=${N:-$(( (9 << 22) + 1000 ))}
timeout -k 10 300 $B/host_stress 1 local 0 $N 3 > gpurun_out/asan_w1.log 2>&1; rc=$?; echo "world 1 rc=$rc"; tail -2 gpurun_out/asan_w1.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 $B/host_stress 2 local 0 $N 2 > gpurun_out/asan_local2.log 2>&1; rc=$?; echo "local 2 rc=$rc"; tail -2 gpurun_out/asan_local2.log
[ $rc -eq 0 ] || exit $rc
PORT=$((30000 + RANDOM % 20000))
for r in 0 1; do
  INCCL_MASTER_PORT=$PORT INCCL_DEVICE=0 INCCL_BOOT_TIMEOUT=120 timeout -k 10 300 $B/host_stress 2 127.0.0.1 $r $N 2 \
    > gpurun_out/asan_tcp_r$r.log 2>&1 &
done
rc=0
for j in $(jobs -p); do wait $j || rc=$?; done
echo "tcp 2 rc=$rc"; tail -2 gpurun_out/asan_tcp_r0.log gpurun_out/asan_tcp_r1.log
exit $rc
