"""Communicator paths on the GPU (gpu): the reference's host API
(inccl_allreduce_write / _sendrecv) and the fp32 allreduce, over the
in-process transport (ranks = threads sharing one GPU, the GPU's sum kernel is
the switch) and over RCCL at world size 1.  Checked against the oracle."""
import os
import socket
import subprocess
import threading

import numpy as np
import pytest

from conftest import GOLDEN, ROOT

pytestmark = pytest.mark.gpu

INT32_MIN, INT32_MAX = -(2 ** 31), 2 ** 31 - 1


def _run_ranks(world, fn):
    """Run fn(rank) on `world` threads; re-raise the first failure."""
    errs = [None] * world
    out = [None] * world

    def body(r):
        try:
            out[r] = fn(r)
        except BaseException as e:  # noqa: BLE001
            errs[r] = e

    ts = [threading.Thread(target=body, args=(r,)) for r in range(world)]
    for t in ts:
        t.start()
    for t in ts:
        t.join(timeout=300)
    for e in errs:
        if e is not None:
            raise e
    return out


def test_host_example_binary(gpu, tmp_path):
    """tests/c/host_example.c: host.c's known answer through the C ABI alone."""
    exe = tmp_path / "host_example"
    subprocess.check_call(["gcc", "-O2", "-std=c11", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "host_example.c"), "-o", str(exe),
                           "-L", os.path.join(ROOT, "container_inc_amd"), "-linccl_amd", "-lpthread",
                           "-Wl,-rpath," + os.path.join(ROOT, "container_inc_amd")])
    for world in (2, 4):
        r = subprocess.run([str(exe), str(world), "local"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and "result ok" in r.stdout, r.stdout + r.stderr
    # exactly as host.c is run: one process per rank, rank 0 the TCP master
    # (both on GPU 0 here, so RCCL refuses and the ranks fall back to p2p together)
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, INCCL_MASTER_PORT=str(port), INCCL_DEVICE="0", INCCL_BOOT_TIMEOUT="120")
    ps = [subprocess.Popen([str(exe), "2", "127.0.0.1", str(r)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True, env=env) for r in range(2)]
    outs = [p.communicate(timeout=240) for p in ps]
    for p, (out, err) in zip(ps, outs):
        assert p.returncode == 0 and "result ok" in out, out + err


def test_reference_host_binary(gpu):
    """The reference's own program, repository/src/host.c compiled unchanged
    against include/ and linked with libinccl_amd.so (oracle/Makefile `ref`,
    built in the container where the reference lives), run exactly as the
    reference runs it: `host <world> <master_ip> <rank>`, one process per rank.
    Its own assert (host.c:51-55, dst[i] == 3*i) is the check; it prints
    "result ok" only if every lane passed."""
    exe = os.path.join(ROOT, "oracle", "_ref", "host_ref")
    if not os.path.isfile(exe):
        # .gpurunignore keeps oracle/_ref off the GPU box; there
        # tests/c/host_example.c asserts the same known answer (host.c:51-55)
        pytest.skip("oracle/_ref/host_ref absent (built only where the reference tree is; not shipped to GPU boxes)")
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, INCCL_MASTER_PORT=str(port), INCCL_DEVICE="0", INCCL_BOOT_TIMEOUT="120")
    ps = [subprocess.Popen([exe, "2", "127.0.0.1", str(r)], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True, env=env) for r in range(2)]
    outs = [p.communicate(timeout=240) for p in ps]
    for p, (out, err) in zip(ps, outs):
        assert p.returncode == 0 and "result ok" in out, out + err


def _c_release(tmp_path):
    """(release, bound) that a C program linked against /opt/rocm's runtime
    reports: the HSA runtime's own build string, csrc/runtime.c."""
    src = tmp_path / "release.c"
    src.write_text('#include <stdio.h>\n#include "inccl_amd.h"\nint main(void){printf("%u %zu %s\\n", '
                   'inccl_hsa_runtime_release(), inccl_ipc_max_bytes(), inccl_hsa_runtime_build());}\n')
    exe = tmp_path / "release"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe), "-L",
                           os.path.join(ROOT, "container_inc_amd"), "-linccl_amd",
                           "-Wl,-rpath," + os.path.join(ROOT, "container_inc_amd")])
    env = {k: v for k, v in os.environ.items() if k != "INCCL_IPC_MAX_BYTES"}
    out = subprocess.check_output([str(exe)], env=env, text=True).split()
    return int(out[0]), int(out[1]), " ".join(out[2:])


def test_ipc_bound_on_the_gpu(gpu, lib, tmp_path):
    """The IPC bound follows the ROCm release each process's HSA runtime
    reports (hsa_system_get_info BUILD_VERSION), not a file name: this Python
    process runs on PyTorch's bundled ROCr (release 7.0 here: bound 2 GiB -
    2 MiB), a C program on /opt/rocm's (7.2 on this image: no bound)."""
    import re
    build = lib.inccl_hsa_runtime_build().decode()
    rel = lib.inccl_hsa_runtime_release()
    assert re.search(r"rocm-rel-\d+\.\d+", build), build
    want = (1 << 40) if rel >= 702 else (2 << 30) - (2 << 20)
    if "INCCL_IPC_MAX_BYTES" not in os.environ:
        assert lib.inccl_ipc_max_bytes() == want
    crel, cbound, cbuild = _c_release(tmp_path)
    assert re.search(r"rocm-rel-\d+\.\d+", cbuild), cbuild
    assert cbound == ((1 << 40) if crel >= 702 else (2 << 30) - (2 << 20)), (crel, cbound, cbuild)
    print(f"python process: release {rel} ({build}); C process: release {crel} ({cbuild}), bound {cbound}")


@pytest.mark.parametrize("engine", ["p2p", "mesh"])
def test_ipc_engine_over_2gib_c_hosted(gpu, tmp_path, engine):
    """The IPC engines on a 2.25 GiB bucket (p2p: 2.25 GiB IPC buffers; mesh:
    a 2.25 GiB inbox) in C processes, which map /opt/rocm's HSA runtime where
    importing such buffers works (csrc/runtime.c lifts the 2 GiB bound there;
    under PyTorch's bundled ROCr the import hangs).  Two processes
    on GPU 0, rank 0 the TCP master, two calls, every lane exact."""
    crel, cbound, cbuild = _c_release(tmp_path)
    if cbound < (9 << 28):
        pytest.skip(f"/opt/rocm's HSA runtime reports release {crel} ({cbuild}): the 2 GiB IPC bound stays")
    exe = tmp_path / "big_ipc"
    subprocess.check_call(["gcc", "-O2", "-std=gnu11", "-D__HIP_PLATFORM_AMD__", "-I", os.path.join(ROOT, "include"),
                           "-I", "/opt/rocm/include", os.path.join(ROOT, "tests", "c", "big_ipc.c"), "-o", str(exe),
                           "-L", os.path.join(ROOT, "container_inc_amd"), "-linccl_amd", "-L", "/opt/rocm/lib",
                           "-lamdhip64", "-Wl,-rpath," + os.path.join(ROOT, "container_inc_amd"),
                           "-Wl,-rpath,/opt/rocm/lib"])
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = {k: v for k, v in os.environ.items() if k != "INCCL_IPC_MAX_BYTES"}
    env.update(INCCL_MASTER_PORT=str(port), INCCL_DEVICE="0", INCCL_BOOT_TIMEOUT="120", INCCL_ENGINE=engine)
    n = str(9 << 26)   # 603 979 776 elements: 2.25 GiB of int32 partials
    ps = [subprocess.Popen([str(exe), "2", str(r), n, engine], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True, env=env) for r in range(2)]
    outs = [p.communicate(timeout=200) for p in ps]
    for p, (out, err) in zip(ps, outs):
        assert p.returncode == 0 and "result ok" in out, out + err
        assert "group bound 1099511627776" in out, out


def test_host_stress_binary(gpu, tmp_path):
    """tests/c/host_stress.c through the C ABI alone: allreduce_write on pageable
    and on registered memory and allreduce_f32_host on pageable memory, 5 pipeline
    chunks plus a ragged tail, several calls -- world 1, two local ranks, and two
    processes over the TCP rendezvous.  (tools/asan_host.sh runs the same program
    under ASan + UBSan.)"""
    exe = tmp_path / "host_stress"
    subprocess.check_call(["gcc", "-O2", "-std=c11", "-I", os.path.join(ROOT, "include"),
                           os.path.join(ROOT, "tests", "c", "host_stress.c"), "-o", str(exe),
                           "-L", os.path.join(ROOT, "container_inc_amd"), "-linccl_amd", "-lpthread",
                           "-Wl,-rpath," + os.path.join(ROOT, "container_inc_amd")])
    n = str((5 << 22) + 1000)
    for world in (1, 2):
        r = subprocess.run([str(exe), str(world), "local", "0", n, "2"], capture_output=True, text=True, timeout=300)
        assert r.returncode == 0 and "result ok" in r.stdout, r.stdout + r.stderr
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    env = dict(os.environ, INCCL_MASTER_PORT=str(port), INCCL_DEVICE="0", INCCL_BOOT_TIMEOUT="120")
    ps = [subprocess.Popen([str(exe), "2", "127.0.0.1", str(r), n, "2"], stdout=subprocess.PIPE, stderr=subprocess.PIPE,
                           text=True, env=env) for r in range(2)]
    outs = [p.communicate(timeout=300) for p in ps]
    for p, (out, err) in zip(ps, outs):
        assert p.returncode == 0 and "result ok" in out, out + err


@pytest.mark.parametrize("variant", ["write", "sendrecv"])
def test_allreduce_write_known_answer(gpu, variant):
    """host.c:20-25,41,47,51-55 with the reference's two ranks."""
    from container_inc_amd import inccl
    g = np.load(os.path.join(GOLDEN, "host_known_answer.npz"))
    hub = f"known-{variant}"

    def rank(r):
        grp = inccl.inccl_group_create_local(2, r, hub)
        comm = inccl.inccl_communicator_create(grp, int(g["comm_size_bytes"]))
        dst = np.zeros_like(g["expected"])
        fn = inccl.inccl_allreduce_write if variant == "write" else inccl.inccl_allreduce_sendrecv
        fn(comm, g["inputs"][r].copy(), g["inputs"].shape[1], dst)
        comm.destroy()
        grp.destroy()
        return dst

    for dst in _run_ranks(2, rank):
        np.testing.assert_array_equal(dst, g["expected"])


@pytest.mark.parametrize("world", [2, 3, 8])
def test_allreduce_write_random_ragged(gpu, orc, world):
    """Random int32 with wrap, len not a multiple of 1024: tail untouched (api.c:406),
    with a small communicator (16 KiB; the reference sizes its registered buffers
    from it, the direct DMA pipeline does not depend on it)."""
    from container_inc_amd import inccl
    n = 1024 * 37 + 500
    rng = np.random.default_rng(world)
    xs = [rng.integers(INT32_MIN, INT32_MAX, n, dtype=np.int64, endpoint=True).astype(np.int32) for _ in range(world)]
    want = orc.sum_q32(xs)
    hub = f"ragged-{world}"

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, hub)
        comm = inccl.inccl_communicator_create(grp, 16384)
        dst = np.full(n, 77, np.int32)
        comm.allreduce_write(xs[r], n, dst)
        comm.destroy()
        grp.destroy()
        return dst

    for dst in _run_ranks(world, rank):
        np.testing.assert_array_equal(dst[: 37 * 1024], want[: 37 * 1024])
        assert np.all(dst[37 * 1024:] == 77)


@pytest.mark.parametrize("n", [0, 500, 1024, 1500, 2048])
def test_allreduce_write_short_messages(gpu, orc, n):
    """Lengths around the reference's message size (1024 int32, api.h:40): below
    one message nothing is written (api.c:406 counts whole messages only); one
    message works here, where the reference's window posts two messages
    unconditionally (api.c:408) and so needs len >= 2048; the tail beyond the
    last whole message stays untouched."""
    from container_inc_amd import inccl
    world = 2
    m = n // 1024 * 1024
    rng = np.random.default_rng(900 + n)
    xs = [rng.integers(INT32_MIN, INT32_MAX, max(n, 1), dtype=np.int64, endpoint=True).astype(np.int32)
          for _ in range(world)]
    want = orc.sum_q32(xs)
    hub = f"short-{n}"

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, hub)
        comm = inccl.inccl_communicator_create(grp, 4096 * 4)
        dst = np.full(max(n, 1), 123, np.int32)
        comm.allreduce_write(xs[r], n, dst)
        comm.destroy()
        grp.destroy()
        return dst

    for dst in _run_ranks(world, rank):
        np.testing.assert_array_equal(dst[:m], want[:m])
        assert np.all(dst[m:] == 123)


@pytest.mark.parametrize("world", [1, 2, 3])
def test_allreduce_write_registered(gpu, orc, world):
    """Registered src/dst (the ibv_reg_mr analogue): direct DMA, several 16 MiB
    chunks + a ragged tail, then the same arrays unregistered (pageable DMA with
    the helper thread's D2Hs); a partially registered call (dst only) also takes
    the pageable path."""
    from container_inc_amd import inccl
    n = 1024 * (4096 * 9 + 3) + 77          # 9 chunks of 16 MiB + 3 messages + a partial one
    m = n // 1024 * 1024
    rng = np.random.default_rng(40 + world)
    xs = [rng.integers(INT32_MIN, INT32_MAX, n, dtype=np.int64, endpoint=True).astype(np.int32) for _ in range(world)]
    want = orc.sum_q32(xs)
    hub = f"reg-{world}"

    def rank(r):
        grp = (inccl.inccl_group_create(1, 0, "127.0.0.1") if world == 1
               else inccl.inccl_group_create_local(world, r, hub))
        comm = inccl.inccl_communicator_create(grp, 1 << 20)
        src = xs[r].copy()
        dst = np.full(n, 5, np.int32)
        comm.host_register(src)
        comm.host_register(dst)
        with pytest.raises(RuntimeError):
            comm.host_register(dst[10:])          # overlaps a registered range
        outs = []
        comm.allreduce_write(src, n, dst)
        outs.append(dst.copy())
        comm.allreduce_write(src, n, dst)         # again: buffers reused
        outs.append(dst.copy())
        comm.host_deregister(src)
        dst[:] = 5
        comm.allreduce_write(src, n, dst)         # dst registered only -> pageable path
        outs.append(dst.copy())
        comm.host_deregister(dst)
        with pytest.raises(RuntimeError):
            comm.host_deregister(dst)
        comm.destroy()
        grp.destroy()
        return outs

    for outs in _run_ranks(world, rank):
        for dst in outs:
            np.testing.assert_array_equal(dst[:m], want[:m])
            assert np.all(dst[m:] == 5)


@pytest.mark.parametrize("pipeline", ["direct-1MiB", "direct-default", "pool"])
@pytest.mark.parametrize("world", [1, 2])
def test_allreduce_write_unregistered_pipelines(gpu, orc, monkeypatch, pipeline, world):
    """Plain (pageable) numpy src/dst -- host.c's malloc'ed buffers -- through both
    host pipelines: direct pageable DMA with the D2Hs issued from the helper
    thread (1 MiB chunks: 37 chunks, the helper's job ring wraps many times) and
    the staged copy pool; three calls on the same arrays, dst prefilled with a
    sentinel each time, tail beyond the last whole message untouched (api.c:406)."""
    from container_inc_amd import inccl
    if pipeline == "pool":
        monkeypatch.setenv("INCCL_HOST_STAGING", "pool")
    elif pipeline == "direct-1MiB":
        monkeypatch.setenv("INCCL_HOST_CHUNK_MIB", "1")
    n = 1024 * (256 * 37 + 5) + 300
    m = n // 1024 * 1024
    rng = np.random.default_rng(7 + world)
    xs = [rng.integers(INT32_MIN, INT32_MAX, n, dtype=np.int64, endpoint=True).astype(np.int32) for _ in range(world)]
    want = orc.sum_q32(xs)
    hub = f"unreg-{pipeline}-{world}"

    def rank(r):
        grp = (inccl.inccl_group_create(1, 0, "127.0.0.1") if world == 1
               else inccl.inccl_group_create_local(world, r, hub))
        comm = inccl.inccl_communicator_create(grp, 1 << 20)
        outs = []
        for call in range(3):
            dst = np.full(n, -3 - call, np.int32)
            comm.allreduce_write(xs[r], n, dst)
            outs.append((call, dst))
        comm.destroy()
        grp.destroy()
        return outs

    for outs in _run_ranks(world, rank):
        for call, dst in outs:
            np.testing.assert_array_equal(dst[:m], want[:m], err_msg=f"call {call}")
            assert np.all(dst[m:] == -3 - call)


@pytest.mark.parametrize("world,R,n,chunks,k", [
    (2, 2, 1 << 20, 1, 25),
    (2, 2, (1 << 20) + 77, 3, 25),
    (3, 1, 100_001, 1, 20),
    (4, 2, 1 << 18, 4, "auto"),
    (8, 1, 65_536, 2, 22),
])
def test_allreduce_f32_local(gpu, orc, world, R, n, chunks, k):
    """quant+local sum -> reduce-scatter (the GPU sum kernel over every rank's
    shard) -> dequant shard -> all-gather, vs oracle.reduce_f32 of all W*R buckets."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(world * 100 + R)
    xs = [[(rng.standard_normal(n) * 2).astype(np.float32) for _ in range(R)] for _ in range(world)]
    every = [x for per in xs for x in per]
    kk = orc.choose_scale(orc.absmax(every), world * R) if k == "auto" else k
    want = orc.reduce_f32(every, kk)
    dev_in = [[torch.from_numpy(x).to(gpu) for x in per] for per in xs]
    torch.cuda.synchronize()
    hub = f"f32-{world}-{R}-{n}-{chunks}"

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, hub)
        comm = inccl.inccl_communicator_create(grp, 0)
        out = torch.empty(n, dtype=torch.float32, device=gpu)
        comm.allreduce_f32(dev_in[r], out=out, scale_exp=inccl.SCALE_AUTO if k == "auto" else k, chunks=chunks,
                           stream=comm.stream)
        torch.cuda.synchronize()
        comm.barrier()
        res = out.cpu().numpy()
        comm.destroy()
        grp.destroy()
        return res

    for res in _run_ranks(world, rank):
        np.testing.assert_array_equal(res.view(np.uint32), want.view(np.uint32))


@pytest.mark.parametrize("world,chunks", [(1, 1), (2, 1), (4, 3), (8, 1)])
def test_allreduce_average_local(gpu, orc, world, chunks):
    """inccl_comm_set_average: the mean, bit-identical to oracle sum / W, fp32 and bf16."""
    import torch
    from container_inc_amd import inccl
    rng = np.random.default_rng(600 + world)
    n = (1 << 18) + 64 * 3
    xs = [[(rng.standard_normal(n) * 2).astype(np.float32) for _ in range(2)] for _ in range(world)]
    every = [x for per in xs for x in per]
    k = orc.choose_scale(orc.absmax(every), world * 2)
    want = orc.reduce_f32(every, k) / np.float32(world)
    hs = [[torch.from_numpy(x).to(torch.bfloat16).view(torch.int16).numpy().view(np.uint16) for x in per]
          for per in xs]
    every16 = [h for per in hs for h in per]
    k16 = orc.choose_scale(orc.absmax_bf16(every16), world * 2)
    s16 = torch.from_numpy(orc.reduce_bf16(every16, k16).view(np.int16)).view(torch.bfloat16)
    want16 = (s16 / world).view(torch.int16).numpy().view(np.uint16)
    dev_in = [[torch.from_numpy(x).to(gpu) for x in per] for per in xs]
    dev16 = [[torch.from_numpy(h.view(np.int16)).to(gpu).view(torch.bfloat16) for h in per] for per in hs]
    torch.cuda.synchronize()
    hub = f"avg-{world}-{chunks}"

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, hub)
        comm = inccl.inccl_communicator_create(grp, 0)
        comm.set_average(True)
        out = torch.empty(n, dtype=torch.float32, device=gpu)
        out16 = torch.empty(n, dtype=torch.bfloat16, device=gpu)
        comm.allreduce_f32(dev_in[r], out=out, scale_exp=inccl.SCALE_AUTO, chunks=chunks, stream=comm.stream)
        comm.allreduce_bf16(dev16[r], out=out16, scale_exp=inccl.SCALE_AUTO, stream=comm.stream)
        torch.cuda.synchronize()
        comm.barrier()
        res = (out.cpu().numpy(), out16.view(torch.int16).cpu().numpy().view(np.uint16))
        comm.destroy()
        grp.destroy()
        return res

    for res, res16 in _run_ranks(world, rank):
        np.testing.assert_array_equal(res.view(np.uint32), want.view(np.uint32))
        np.testing.assert_array_equal(res16, want16)


@pytest.fixture()
def force_rccl(monkeypatch):
    monkeypatch.setenv("INCCL_FORCE_RCCL", "1")
    monkeypatch.setenv("INCCL_FORCE_SHARDED", "1")
    monkeypatch.setenv("INCCL_MASTER_PORT", "0")


def test_rccl_world1_paths(gpu, orc, force_rccl):
    """RCCL transport at world size 1: ncclReduceScatter / ncclAllGather /
    ncclAllReduce are real RCCL calls on a one-rank communicator."""
    import torch
    from container_inc_amd import inccl
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    assert grp is not None and grp.transport == "rccl"
    comm = inccl.inccl_communicator_create(grp, 1 << 20)
    rng = np.random.default_rng(5)
    for engine in ("rccl", "ar", "a2a", "p2p", "mesh", "meshw"):
        comm.set_engine(engine)
        assert comm.engine == engine
        for n, chunks in ((1 << 20, 1), ((1 << 20) + 5, 3)):
            xs = [rng.standard_normal(n).astype(np.float32) for _ in range(2)]
            out = comm.allreduce_f32([torch.from_numpy(x).to(gpu) for x in xs], scale_exp=25, chunks=chunks)
            torch.cuda.synchronize()   # the call ran on the communicator's own (non-blocking) stream
            np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32),
                                          orc.reduce_f32(xs, 25).view(np.uint32), err_msg=engine)
    comm.set_engine("rccl")
    q = rng.integers(INT32_MIN, INT32_MAX, 4096, dtype=np.int64, endpoint=True).astype(np.int32)
    qa = comm.allreduce_q32(torch.from_numpy(q).to(gpu))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(qa.cpu().numpy(), q)
    dst = np.zeros(4096, np.int32)
    comm.allreduce_write(q, 4096, dst)
    np.testing.assert_array_equal(dst, q)
    comm.destroy()
    grp.destroy()


@pytest.mark.parametrize("ar_bytes", [None, "0", str(1 << 16)])
def test_rccl_small_bucket_route(gpu, orc, force_rccl, monkeypatch, ar_bytes):
    """The rccl engine's small buckets (int32 partials within
    INCCL_RCCL_AR_BYTES, default 1 MiB) take one ncclAllReduce instead of
    reduce-scatter + all-gather; 0 disables it, 64 KiB splits the sizes below
    across both routes.  Every size and format is bit-exact either way."""
    import torch
    from container_inc_amd import inccl
    if ar_bytes is not None:
        monkeypatch.setenv("INCCL_RCCL_AR_BYTES", ar_bytes)
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    assert grp.transport == "rccl" and comm.engine == "rccl"
    rng = np.random.default_rng(17)
    for n in (1, 1000, 16384, 16385, (1 << 18) + 3, (1 << 18) + 64):
        xs = [rng.standard_normal(n).astype(np.float32) for _ in range(2)]
        out = comm.allreduce_f32([torch.from_numpy(x).to(gpu) for x in xs], scale_exp=inccl.SCALE_AUTO)
        torch.cuda.synchronize()
        k = orc.choose_scale(orc.absmax(xs), 2)
        np.testing.assert_array_equal(out.cpu().numpy().view(np.uint32), orc.reduce_f32(xs, k).view(np.uint32),
                                      err_msg=str(n))
        hs = [orc.f32_to_bf16(x) for x in xs]
        srcs = [torch.from_numpy(h.view(np.int16)).to(gpu).view(torch.bfloat16) for h in hs]
        out16 = torch.empty(n, dtype=torch.bfloat16, device=gpu)
        comm.allreduce_bf16(srcs, out=out16, scale_exp=24, stream=comm.stream)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(out16.view(torch.int16).cpu().numpy().view(np.uint16),
                                      orc.reduce_bf16(hs, 24), err_msg=str(n))
    comm.destroy()
    grp.destroy()


@pytest.mark.parametrize("engine,chunks", [("rccl", 1), ("rccl", 3), ("ar", 1), ("a2a", 1)])
def test_rccl_world1_graph_capture(gpu, orc, force_rccl, engine, chunks):
    """allreduce_f32 captured into a hipGraph (as a framework that graphs its
    communication would) on the RCCL engines at world 1, including the chunked
    pipeline's side stream: three captured calls, replayed with fresh inputs
    each time, bit-exact vs the oracle."""
    import torch
    from container_inc_amd import inccl
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    comm.set_engine(engine)
    n = (1 << 18) + 64
    bufs = [torch.empty(n, device=gpu) for _ in range(2)]
    outs = [torch.empty(n, device=gpu) for _ in range(3)]
    st = torch.cuda.Stream(device=gpu)
    comm.allreduce_f32(bufs, out=outs[0], scale_exp=24, chunks=chunks, stream=st.cuda_stream)   # workspaces sized eagerly
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=st):
        for o in outs:
            comm.allreduce_f32(bufs, out=o, scale_exp=24, chunks=chunks, stream=st.cuda_stream)
    rng = np.random.default_rng(77)
    for _ in range(3):
        xs = [rng.standard_normal(n).astype(np.float32) for _ in range(2)]
        for b, x in zip(bufs, xs):
            b.copy_(torch.from_numpy(x))
        for o in outs:
            o.fill_(float("nan"))
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        want = orc.reduce_f32(xs, 24).view(np.uint32)
        for o in outs:
            np.testing.assert_array_equal(o.cpu().numpy().view(np.uint32), want)
    del graph
    comm.destroy()
    grp.destroy()


def test_allreduce_f32_host_buckets(gpu, orc):
    """BASELINE config 3 shape (scaled down): host fp32 -> 3-stream pipeline -> host."""
    import torch
    from container_inc_amd import inccl
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    n = (16 << 20) // 4 + 333
    x = torch.randn(n, dtype=torch.float32).pin_memory()
    y = torch.empty(n, dtype=torch.float32).pin_memory()
    comm.allreduce_f32_host(x, y, scale_exp=24, bucket_bytes=1 << 20)
    want = orc.reduce_f32([x.numpy()], 24)
    np.testing.assert_array_equal(y.numpy().view(np.uint32), want.view(np.uint32))
    # pageable numpy buffers work too (synchronous staging)
    xn = x.numpy().copy()
    yn = np.empty_like(xn)
    comm.allreduce_f32_host(xn, yn, scale_exp=24, bucket_bytes=3 << 20)
    np.testing.assert_array_equal(yn.view(np.uint32), want.view(np.uint32))
    comm.destroy()
    grp.destroy()


def test_allreduce_f32_host_config3_full_size(gpu, orc):
    """BASELINE config 3 at its real size: a 1 GiB fp32 gradient in pinned host
    memory, 16 buckets of 64 MiB through the three-stream H2D / reduce / D2H
    pipeline (the reference's registered staging buffers, api.c:164-176), plus a
    ragged tail bucket; every lane bit-exact vs the oracle."""
    import torch
    from container_inc_amd import inccl
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    n = (1 << 30) // 4 + 4099   # 16 full 64 MiB buckets + a ragged 17th
    gen = torch.Generator().manual_seed(3)
    x = torch.randn(n, generator=gen, dtype=torch.float32).pin_memory()
    y = torch.full((n,), float("nan"), dtype=torch.float32).pin_memory()
    comm.allreduce_f32_host(x, y, scale_exp=25, bucket_bytes=64 << 20)
    want = orc.reduce_f32([x.numpy()], 25)
    bad = np.flatnonzero(y.numpy().view(np.uint32) != want.view(np.uint32))
    assert bad.size == 0, f"{bad.size} lanes differ, first at {bad[:8]}"
    # a second call over the same buffers (pipeline state and events reused)
    y.fill_(float("nan"))
    comm.allreduce_f32_host(x, y, scale_exp=25, bucket_bytes=64 << 20)
    assert np.array_equal(y.numpy().view(np.uint32), want.view(np.uint32))
    comm.destroy()
    grp.destroy()
