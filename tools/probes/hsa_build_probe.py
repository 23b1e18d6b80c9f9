"""Print what each mapped HSA runtime (ROCr) reports about its own version.

One child process per runtime (never two ROCr copies in one process): the
runtime is loaded by path, hsa_init'ed, and asked for
HSA_AMD_SYSTEM_INFO_BUILD_VERSION (0x200, a string), the extension-interface
version (0x207 / 0x208, uint16) and the HSA spec version (0 / 1, uint16).
Used to choose the version query in csrc/runtime.c."""
import ctypes
import json
import os
import subprocess
import sys


def probe(path: str) -> dict:
    h = ctypes.CDLL(path)
    out = {"path": os.path.realpath(path), "hsa_init": h.hsa_init()}
    s = ctypes.c_char_p()
    out["build_rc"] = h.hsa_system_get_info(0x200, ctypes.byref(s))
    out["build"] = s.value.decode(errors="replace") if s.value else None
    for name, attr in (("spec_major", 0), ("spec_minor", 1), ("ext_major", 0x207), ("ext_minor", 0x208)):
        v = ctypes.c_uint16(0)
        rc = h.hsa_system_get_info(attr, ctypes.byref(v))
        out[name] = v.value if rc == 0 else f"rc={rc:#x}"
    h.hsa_shut_down()
    return out


if __name__ == "__main__":
    if len(sys.argv) > 1:
        print(json.dumps(probe(sys.argv[1])))
        sys.exit(0)
    import torch  # noqa: F401  (only to locate its lib directory; the GPU is not touched here)
    tl = os.path.join(os.path.dirname(torch.__file__), "lib", "libhsa-runtime64.so")
    for p in ("/opt/rocm/lib/libhsa-runtime64.so.1", tl):
        r = subprocess.run([sys.executable, __file__, p], capture_output=True, text=True, timeout=60)
        print(r.stdout.strip() or f"{p}: rc={r.returncode} {r.stderr.strip()[-300:]}")
