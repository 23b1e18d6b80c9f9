#!/bin/bash
# Which component makes a >2 GiB hipIpcOpenMemHandle hang (DESIGN.md
# "Runtimes")?  The same C probe (ipc_size_probe.c) at 2600 MiB, bound to
# /opt/rocm's HIP 7.2 and to torch's bundled HIP 7.0 (through a directory of
# soname links to torch/lib), one-way (round 2's probe) and then symmetric
# (both processes export and import at once, as the mesh engine's ranks do),
# then symmetric with 2 GiB of other device memory held first.  Every run is
# bounded; the script stops at the first failure or hang.
set -u
OUT=$(realpath -m "${1:-gpurun_out/ipc_runtime_probe}")
cd "$(dirname "$0")"
mkdir -p "$OUT"
TL=$(python3 -c "import os, importlib.util as u; print(os.path.dirname(u.find_spec('torch').origin) + '/lib')")
LNK=$(mktemp -d)
ln -s "$TL/libamdhip64.so" "$LNK/libamdhip64.so.7"
ln -s "$TL/libhsa-runtime64.so" "$LNK/libhsa-runtime64.so.1"
run() {   # name libpath args...
  local name=$1 lp=$2; shift 2
  LD_LIBRARY_PATH=$lp timeout -k 5 60 ./ipc_size_probe "$@" > "$OUT/$name.txt" 2>&1
  local rc=$?
  echo "$name ($*): rc=$rc" | tee -a "$OUT/log.txt"
  sed 's/^/    /' "$OUT/$name.txt" >> "$OUT/log.txt"
  if [ $rc -ne 0 ]; then echo "stopping after a failed/hung run" | tee -a "$OUT/log.txt"; exit $rc; fi
}
run rocm72_one /opt/rocm/lib 0 2600 one
run torch70_one "$LNK" 0 2600 one
run rocm72_sym_small /opt/rocm/lib 0 256 sym
run torch70_sym_small "$LNK" 0 256 sym
run rocm72_sym /opt/rocm/lib 0 2600 sym
run torch70_sym "$LNK" 0 2600 sym
run rocm72_sym_uncached /opt/rocm/lib 3 2600 sym
run torch70_sym_uncached "$LNK" 3 2600 sym
run torch70_sym_prealloc "$LNK" 0 2600 sym 2048
echo "all runs passed" | tee -a "$OUT/log.txt"
