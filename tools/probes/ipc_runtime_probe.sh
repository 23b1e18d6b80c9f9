#!/bin/bash
# Isolates the runtime as the cause of the >2 GiB hipIpcOpenMemHandle hang
# (DESIGN.md "Runtimes"): the same C probe (ipc_size_probe.c: fork, export a
# hipMalloc'd buffer, import it in the child, read its last MiB) at 2600 MiB,
# bound first to /opt/rocm's HIP 7.2 and then to torch's bundled HIP 7.0
# (through a directory of soname links to torch/lib).  Each run is bounded.
set -u
cd "$(dirname "$0")"
OUT=${1:-../../gpurun_out/ipc_runtime_probe}
mkdir -p "$OUT"
TL=$(python3 -c "import os, importlib.util as u; print(os.path.dirname(u.find_spec('torch').origin) + '/lib')")
LNK=$(mktemp -d)
ln -s "$TL/libamdhip64.so" "$LNK/libamdhip64.so.7"
ln -s "$TL/libhsa-runtime64.so" "$LNK/libhsa-runtime64.so.1"
for rt in rocm72 torch70; do
  if [ $rt = rocm72 ]; then LP=/opt/rocm/lib; else LP=$LNK; fi
  echo "== $rt (LD_LIBRARY_PATH=$LP)" | tee -a "$OUT/log.txt"
  LD_LIBRARY_PATH=$LP timeout -k 5 20 ./ipc_size_probe 0 64 > "$OUT/$rt.small.txt" 2>&1
  echo "$rt 64 MiB rc=$?" | tee -a "$OUT/log.txt"
  cat "$OUT/$rt.small.txt" >> "$OUT/log.txt"
  LD_LIBRARY_PATH=$LP timeout -k 5 60 ./ipc_size_probe 0 2600 > "$OUT/$rt.big.txt" 2>&1
  rc=$?
  echo "$rt 2600 MiB rc=$rc" | tee -a "$OUT/log.txt"
  cat "$OUT/$rt.big.txt" >> "$OUT/log.txt"
  if [ $rc -ne 0 ]; then echo "stopping after a failed/hung run" | tee -a "$OUT/log.txt"; exit $rc; fi
done
