"""The C-ABI boundary: libinccl_amd.so loads and exports exactly what
include/api.h and include/inccl_amd.h declare; the headers compile as plain C
with no HIP/RCCL/torch headers.  No compute calls (CPU only)."""
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADERS = [os.path.join(ROOT, "include", h) for h in ("api.h", "inccl_amd.h")]


def declared_functions():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(inccl_\w+)\s*\(", text):
            names.add(m.group(1))
    return names


def exported_symbols(path):
    out = subprocess.check_output(["nm", "-D", "--defined-only", path], text=True)
    return {ln.split()[-1] for ln in out.splitlines() if " T " in ln}


def test_reference_six_entry_points_declared():
    # repository/include/api.h:93-101
    ref = {"inccl_group_create", "inccl_group_destroy", "inccl_communicator_create",
           "inccl_communicator_destroy", "inccl_allreduce_sendrecv", "inccl_allreduce_write"}
    assert ref <= declared_functions()


def test_library_exports_every_declared_symbol(lib):
    import container_inc_amd as cia
    decl = declared_functions()
    exp = exported_symbols(cia.LIB_PATH)
    missing = decl - exp
    assert not missing, f"declared but not exported: {sorted(missing)}"
    extra = {s for s in exp if s.startswith("inccl_")} - decl
    assert not extra, f"exported but undeclared: {sorted(extra)}"
    for name in decl:
        assert hasattr(lib, name)


def test_library_has_no_unresolved_internal_symbols(lib):
    """Every inccl_* function the library calls is defined in it (an undefined
    one would only fail when the .so is loaded on the GPU box)."""
    import container_inc_amd as cia
    out = subprocess.check_output(["nm", "-D", "--undefined-only", cia.LIB_PATH], text=True)
    undef = [ln.split()[-1] for ln in out.splitlines() if "inccl_" in ln]
    assert not undef, undef


def test_rccl_symbols_resolve_in_every_librccl_it_may_bind(lib):
    """libinccl_amd.so is compiled against /opt/rocm's RCCL headers but, in a
    Python process that imported torch first, binds torch's bundled librccl (the
    same soname; BENCH "runtime": rccl_compiled 22707, rccl_loaded 22606).
    Every nccl* symbol the library imports must be defined -- as a function --
    in both copies, or a multi-GPU call would fail only at bind time on an
    8-GPU node.  The ABI-relevant constants (ncclUniqueId size, the int32 / sum
    enum values) are checked against the header the library was built with."""
    import container_inc_amd as cia
    from container_inc_amd._lib import runtime_libs
    out = subprocess.check_output(["nm", "-D", "--undefined-only", cia.LIB_PATH], text=True)
    need = {ln.split()[-1] for ln in out.splitlines() if ln.split()[-1].startswith("nccl")}
    assert {"ncclReduceScatter", "ncclAllGather", "ncclCommInitRank", "ncclGetLastError"} <= need
    import torch  # noqa: F401 -- the process a user runs: torch first, then the library
    bound = runtime_libs().get("librccl")
    copies = {p for p in (bound, "/opt/rocm/lib/librccl.so.1") if p and os.path.exists(p)}
    assert bound, "no librccl mapped in this process"
    for path in copies:
        have = exported_symbols(path)
        missing = sorted(need - have)
        assert not missing, f"{path} lacks {missing}"
    hdr = open("/opt/rocm/include/rccl/rccl.h").read()
    assert re.search(r"#define\s+NCCL_UNIQUE_ID_BYTES\s+128\b", hdr)
    assert re.search(r"ncclInt32\s*=\s*2\b", hdr) and re.search(r"ncclSum\s*=\s*0\b", hdr)


def test_python_binding_covers_abi():
    from container_inc_amd._lib import SIGNATURES
    assert set(SIGNATURES) == declared_functions()


def test_headers_compile_as_plain_c(tmp_path):
    src = tmp_path / "t.c"
    src.write_text('#include "api.h"\n#include "inccl_amd.h"\n#include "util.h"\n#include "topo_parser.h"\n'
                   'int main(void){return INCCL_OK;}\n')
    subprocess.check_call(["gcc", "-std=c11", "-Wall", "-Werror", "-fsyntax-only", "-I", os.path.join(ROOT, "include"),
                           str(src)])


def test_host_example_links(tmp_path):
    exe = tmp_path / "host_example"
    subprocess.check_call(["gcc", "-O2", "-std=c11", "-Wall", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "host_example.c"), "-o", str(exe),
                           "-L", os.path.join(ROOT, "container_inc_amd"), "-linccl_amd", "-lpthread"])
    assert exe.exists()


REF_HOST_C = "/root/reference/repository/src/host.c"


@pytest.mark.skipif(not os.path.isfile(REF_HOST_C), reason="reference tree absent (GPU box)")
def test_reference_host_c_builds_unchanged(tmp_path):
    """The drop-in claim itself: the reference's own caller (host.c, by path,
    unmodified) compiles warning-free against include/ alone -- its includes of
    api.h, util.h and topo_parser.h (host.c:1-4) all resolve here, and api.h
    supplies the system headers (reference api.h:1-18) behind its printf,
    atoi, clock_t and CLOCKS_PER_SEC -- and links against libinccl_amd.so."""
    exe = tmp_path / "host"
    subprocess.check_call(["gcc", "-std=gnu11", "-O2", "-Wall", "-Werror", "-I", os.path.join(ROOT, "include"),
                           REF_HOST_C, "-o", str(exe), "-L", os.path.join(ROOT, "container_inc_amd"),
                           "-linccl_amd", "-lpthread"])
    assert exe.exists()
    undef = subprocess.check_output(["nm", "--undefined-only", str(exe)], text=True)
    used = {ln.split()[-1] for ln in undef.splitlines() if "inccl_" in ln}
    assert used == {"inccl_group_create", "inccl_communicator_create", "inccl_allreduce_write"}, used


def test_ipc_bound_follows_the_hsa_runtime(lib, tmp_path):
    """The IPC engines' largest shared buffer follows the ROCm release the mapped
    HSA runtime reports about itself (csrc/runtime.c): its build string is
    parsed for "rocm-rel-X.Y", 7.2 or later lifts the 2 GiB - 2 MiB bound.  On
    this GPU-less host the runtime cannot be asked, so the bound stays, in this
    Python process and in a C program alike; $INCCL_IPC_MAX_BYTES overrides in
    whole MiB, and a value below 1 MiB is ignored.  The parser runs on the two
    build strings the MI355X box's runtimes report (tests/c/hsa_release.c);
    tests/test_gpu_comm.py checks the query there."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present: tests/test_gpu_comm.py::test_ipc_bound_on_the_gpu covers it")
    bound = (2 << 30) - (2 << 20)
    assert lib.inccl_hsa_runtime_release() == 0 and lib.inccl_hsa_runtime_build() == b""
    assert lib.inccl_ipc_max_bytes() == bound
    src = tmp_path / "ipcmax.c"
    src.write_text('#include <stdio.h>\n#include "inccl_amd.h"\n'
                   'int main(void){printf("%zu %u\\n", inccl_ipc_max_bytes(), inccl_hsa_runtime_release());}\n')
    exe = tmp_path / "ipcmax"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe), "-L",
                           os.path.join(ROOT, "container_inc_amd"), "-linccl_amd",
                           "-Wl,-rpath," + os.path.join(ROOT, "container_inc_amd")])
    env = {k: v for k, v in os.environ.items() if k != "INCCL_IPC_MAX_BYTES"}
    assert subprocess.check_output([str(exe)], env=env, text=True).split() == [str(bound), "0"]
    for val, want in (("12345", bound), (str((5 << 20) + 123), 5 << 20), (str(16 << 30), 16 << 30)):
        env["INCCL_IPC_MAX_BYTES"] = val
        r = subprocess.run([str(exe)], env=env, capture_output=True, text=True, check=True)
        assert int(r.stdout.split()[0]) == want, (val, r.stdout)
        assert ("below 1 MiB" in r.stderr) == (want == bound)
    parser = tmp_path / "hsa_release"
    subprocess.check_call(["gcc", "-std=gnu11", "-D__HIP_PLATFORM_AMD__", "-I", "/opt/rocm/include", "-I",
                           os.path.join(ROOT, "include"), "-I", os.path.join(ROOT, "container_inc_amd", "csrc"),
                           os.path.join(ROOT, "tests", "c", "hsa_release.c"), "-o", str(parser), "-L",
                           "/opt/rocm/lib", "-lamdhip64", "-lrccl", "-Wl,-rpath,/opt/rocm/lib"])
    out = subprocess.check_output([str(parser)], text=True)
    assert "parser ok" in out and f"release 0 build  bound {bound}" in out, out


def test_rccl_version_reported(lib):
    """The RCCL the library was compiled against (/opt/rocm's headers) and the
    one the process bound to (torch's librccl in Python) are both reported."""
    import ctypes
    c, ld = ctypes.c_int(0), ctypes.c_int(0)
    assert lib.inccl_rccl_version(ctypes.byref(c), ctypes.byref(ld)) == 0
    assert c.value >= 22700 and ld.value >= 22000, (c.value, ld.value)
    from container_inc_amd._lib import runtime_libs
    rt = runtime_libs()
    assert rt["rccl_compiled"] == c.value and rt["rccl_loaded"] == ld.value


def test_version_and_host_helpers(lib):
    assert lib.inccl_version().startswith(b"inccl-amd")
    from container_inc_amd import inccl
    assert inccl.choose_scale(6.0, 8) == 24


def test_choose_scale_host_matches_oracle(lib, orc):
    from container_inc_amd import inccl
    for amax in (0.0, 1e-30, 1e-3, 0.25, 0.5, 1.0, 6.0, 7.999, 1e6, 3e38, float("inf")):
        for R in (1, 2, 3, 8, 64):
            assert inccl.choose_scale(amax, R) == orc.choose_scale(amax, R), (amax, R)


def test_no_device_means_loud_failure(lib):
    """Without a GPU the product fails; it never computes on the CPU."""
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    from container_inc_amd import inccl
    g = inccl.inccl_group_create(1, 0, "127.0.0.1")
    assert g is None
    assert lib.inccl_last_error()


def _prototypes():
    """name -> (return type text, [parameter type texts]) for every function
    declared in the public headers (comments stripped; prototypes may span lines)."""
    protos = {}
    for h in HEADERS:
        text = re.sub(r"/\*.*?\*/", "", open(h).read(), flags=re.S)
        text = re.sub(r"//[^\n]*", "", text)
        for m in re.finditer(r"([A-Za-z_][\w \t\*]*?)\b(inccl_\w+)\s*\(([^;{]*?)\)\s*;", text, flags=re.S):
            ret, name, params = m.group(1).strip(), m.group(2), " ".join(m.group(3).split())
            plist = [] if params in ("", "void") else [p.strip() for p in params.split(",")]
            protos[name] = (ret, plist)
    return protos


def _ctype_class(c_text):
    """the ctypes class a C parameter / return type must be bound with"""
    import ctypes
    t = c_text.replace("const", " ").strip()
    if "*" in t:
        return "char*" if re.match(r"^char\s*\*\s*\w*$", t) else "ptr"
    base = t.split()[-1] if t.split() else t
    return {"int": ctypes.c_int, "int32_t": ctypes.c_int, "uint32_t": ctypes.c_uint32, "size_t": ctypes.c_size_t,
            "uint64_t": ctypes.c_uint64, "int64_t": ctypes.c_int64, "float": ctypes.c_float, "void": None,
            "unsigned": ctypes.c_uint, "long": ctypes.c_long}.get(base, base)


def test_python_binding_matches_prototypes():
    """Every binding in _lib.SIGNATURES has the header prototype's argument count
    and, argument by argument, the same C type class (pointer, char*, int,
    uint32_t, size_t, ...): a binding that drifted from its header would pass
    arguments in the wrong registers on the GPU box."""
    import ctypes
    from container_inc_amd._lib import SIGNATURES
    protos = _prototypes()
    assert set(protos) == set(SIGNATURES)
    ptr_ok = {ctypes.c_void_p, ctypes.c_char_p}
    for name, (restype, argtypes) in SIGNATURES.items():
        ret, params = protos[name]
        assert len(argtypes) == len(params), (name, params, argtypes)
        for i, (p, a) in enumerate(zip(params, argtypes)):
            m = re.match(r"^(.*[\s\*])\w+$", p)   # drop the parameter's name
            want = _ctype_class(m.group(1) if m else p)
            if want == "ptr":
                assert a in ptr_ok, (name, i, p, a)
            elif want == "char*":
                assert a in ptr_ok, (name, i, p, a)
            else:
                assert a is want, (name, i, p, a)
        rwant = _ctype_class(ret)
        if rwant in ("ptr", "char*"):
            assert restype in ptr_ok, (name, ret, restype)
        else:
            assert restype is rwant, (name, ret, restype)
