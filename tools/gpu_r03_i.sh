#!/bin/bash
# Round 3: is loading the HIP runtime with dlopen (as a Python process does
# through ctypes) what makes a 2600 MiB IPC import hang?  The C sibling probe
# with the runtime dlopen()ed RTLD_LOCAL in each process, /opt/rocm's 7.2 first,
# then torch's 7.0.  Bounded; stops at the first hang.
set -u
cd "$GRAFT_REPO_ROOT" || exit 3
O=gpurun_out/r03i
mkdir -p $O
TL=$(python3 -c "import os, importlib.util as u; print(os.path.dirname(u.find_spec('torch').origin) + '/lib')")
for lib in /opt/rocm/lib/libamdhip64.so.7 $TL/libamdhip64.so; do
  tag=$(basename $(dirname $(dirname $lib)))
  PROBE_HIP_LIB=$lib timeout -k 10 60 tools/probes/ipc_size_probe_dl 0 2600 sib > $O/c_dlopen_sib_2600_$tag.log 2>&1
  rc=$?; echo "C dlopen siblings ($lib) rc=$rc"; cat $O/c_dlopen_sib_2600_$tag.log
  [ $rc -eq 0 ] || exit $rc
done
