#!/bin/bash
# Round 3: which runtime layer hangs a 2600 MiB IPC import -- HIP or HSA?
# The linked C sibling probe with the two layers mixed through a directory of
# soname links (each library's $ORIGIN resolves to that directory):
#   HIP 7.0 (torch) over HSA 7.2 (/opt/rocm), then HIP 7.2 over HSA 7.0 (torch).
# Every process prints the HIP and HSA files it mapped.  Bounded; stops at the
# first hang.  Then the apply frames-per-wave sweep of the switch bench.
set -u
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03j
mkdir -p $O
TL=$(python3 -c "import os, importlib.util as u; print(os.path.dirname(u.find_spec('torch').origin) + '/lib')")
for k in 2 4 8; do
  INCCL_APPLY_FRAMES=$k timeout -k 10 200 python -u -m pytest tests/test_gpu_switch.py -m gpu -x -q --timeout 200 --timeout-method thread -k "batches or serial" > $O/pytest_switch_apply$k.log 2>&1
  rc=$?; echo "switch tests apply frames $k rc=$rc"; tail -1 $O/pytest_switch_apply$k.log; [ $rc -eq 0 ] || exit $rc
  INCCL_APPLY_FRAMES=$k timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof_apply$k -o run --output-format csv -- python3 tools/switch_bench.py > $O/prof_apply$k.log 2>&1 || exit 6
  grep -h "k_ingress_apply\|k_egress" $O/prof_apply$k/run_kernel_stats.csv | cut -d, -f2-4 | sed "s/^/apply$k /"
done
A=$(mktemp -d); B=$(mktemp -d)
ln -s "$TL/libamdhip64.so" "$A/libamdhip64.so.7"                        # HIP 7.0 ...
ln -s /opt/rocm/lib/libhsa-runtime64.so.1 "$A/libhsa-runtime64.so"     # ... over HSA 7.2
ln -s /opt/rocm/lib/libamdhip64.so.7 "$B/libamdhip64.so.7"              # HIP 7.2 ...
ln -s "$TL/libhsa-runtime64.so" "$B/libhsa-runtime64.so.1"             # ... over HSA 7.0
for dep in libelf.so libdrm.so libdrm_amdgpu.so libnuma.so librocprofiler-register.so; do
  ln -s "$TL/$dep" "$B/$dep"                                          # torch HSA's own deps ($ORIGIN = B)
done
for combo in A B; do
  d=$A; [ $combo = B ] && d=$B
  LD_LIBRARY_PATH=$d timeout -k 10 60 tools/probes/ipc_size_probe 0 2600 sib > $O/c_sib_2600_mix$combo.log 2>&1
  rc=$?; echo "mix $combo rc=$rc"; cat $O/c_sib_2600_mix$combo.log
  [ $rc -eq 0 ] || exit $rc
done
