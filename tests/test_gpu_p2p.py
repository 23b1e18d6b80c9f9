"""Multi-process groups on the GPU (gpu): one process per rank, TCP bootstrap
(api.c:34-144 replacement), the p2p engine (HIP IPC buffers, each rank pulls its
shard from every peer with the fused sum+dequantise kernel, then gathers every
result shard).  On a one-GPU box all ranks share device 0 -- IPC between
processes on one device exercises the same code as across xGMI.  RCCL itself
refuses two ranks on one GPU, so its multi-rank calls are covered by the
world-1 RCCL test and by the identical piece logic over the local transport."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _inputs(world, R, n, seed):
    out = []
    for r in range(world):
        rng = np.random.default_rng(seed + r)
        out.append([(rng.standard_normal(n) * 2).astype(np.float32) for _ in range(R)])
    return out


RCCL_ENGINES = ("rccl", "ar", "a2a")


def _rank_main(rank, world, port, cases, q, engine="p2p", device=0):
    try:
        if engine not in RCCL_ENGINES:
            os.environ["INCCL_ENGINE"] = engine
        if engine in ("p2p", "mesh", "meshw"):
            os.environ["INCCL_LL_MAX_BYTES"] = "0"   # the sharded exchange at every size
        os.environ["INCCL_DEVICE"] = str(device)
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        from oracle import oracle as O
        torch.cuda.set_device(device)
        dev = torch.device("cuda", device)
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port, device=device)
        assert grp is not None, "group create failed"
        comm = inccl.inccl_communicator_create(grp, 0)
        if engine in RCCL_ENGINES:
            comm.set_engine(engine)   # needs a live multi-rank RCCL communicator (one GPU per rank)
        assert comm is not None and comm.engine == engine
        side = torch.cuda.Stream(device=dev)
        results = []
        for case in cases:
            R, n, k, seed = case[:4]
            shift = case[4] if len(case) > 4 else 0   # element offset: unaligned src/dst
            xs = _inputs(world, R, n, seed)
            every = [x for per in xs for x in per]
            kk = O.choose_scale(O.absmax(every), world * R) if k == "auto" else k
            want = O.reduce_f32(every, kk)
            srcs = [torch.from_numpy(np.concatenate([np.zeros(shift, np.float32), x])).to(dev)[shift:]
                    for x in xs[rank]]
            out = torch.full((n + shift,), float("nan"), device=dev)[shift:]
            # the inputs and the NaN fill were made on torch's stream; the library
            # runs on its own non-blocking streams, so order them explicitly
            torch.cuda.synchronize()
            for it in range(4):   # repeated: buffer reuse across calls (and across two streams)
                comm.allreduce_f32(srcs, out=out, scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                                   stream=comm.stream if it % 2 == 0 else side.cuda_stream)
                torch.cuda.synchronize()
                got = out.cpu().numpy()
                results.append(bool(np.array_equal(got.view(np.uint32), want.view(np.uint32))))
            # back to back with no host synchronisation in between (the bench's timed loop)
            outs = [torch.full((n + shift,), float("nan"), device=dev)[shift:] for _ in range(12)]
            torch.cuda.synchronize()
            for o in outs:
                comm.allreduce_f32(srcs, out=o, scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                                   stream=comm.stream)
            torch.cuda.synchronize()
            for o in outs:
                results.append(bool(np.array_equal(o.cpu().numpy().view(np.uint32), want.view(np.uint32))))
        # a prepared allreduce (inccl_op_create_allreduce_f32): the same result
        # from the bound call, run back to back
        for R, n, k, seed in ((2, 4099, 25, 61), (2, 1 << 20, 24, 62)):
            xs = _inputs(world, R, n, seed)
            want = O.reduce_f32([x for per in xs for x in per], k)
            srcs = [torch.from_numpy(x).to(dev) for x in xs[rank]]
            out = torch.full((n,), float("nan"), device=dev)
            torch.cuda.synchronize()
            op = comm.prepare_allreduce_f32(srcs, out=out, scale_exp=k, stream=comm.stream)
            for _ in range(3):
                op()
            torch.cuda.synchronize()
            results.append(bool(np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))))
            op.destroy()
        # in place, dst = srcs[0] (the DDP hook's call, container_inc_amd/ddp.py): a
        # bucket inside the ll slot and one above it
        for R, n, k, seed in ((1, 200_003, "auto", 41), (2, 1 << 20, 25, 42)):
            xs = _inputs(world, R, n, seed)
            every = [x for per in xs for x in per]
            kk = O.choose_scale(O.absmax(every), world * R) if k == "auto" else k
            want = O.reduce_f32(every, kk)
            srcs = [torch.from_numpy(x).to(dev) for x in xs[rank]]
            torch.cuda.synchronize()
            comm.allreduce_f32(srcs, out=srcs[0], scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                               stream=comm.stream)
            torch.cuda.synchronize()
            results.append(bool(np.array_equal(srcs[0].cpu().numpy().view(np.uint32), want.view(np.uint32))))
        # the mean instead of the sum (inccl_comm_set_average): bit-identical to the
        # oracle's sum / W for a power-of-two world, refused otherwise
        pow2 = world & (world - 1) == 0
        try:
            comm.set_average(True)
            results.append(pow2)
        except Exception:  # noqa: BLE001
            results.append(not pow2)
        if pow2:
            for R, n, k, seed in ((2, 200_003, "auto", 51), (1, 1 << 20, 24, 52)):
                xs = _inputs(world, R, n, seed)
                every = [x for per in xs for x in per]
                kk = O.choose_scale(O.absmax(every), world * R) if k == "auto" else k
                want = O.reduce_f32(every, kk) / np.float32(world)
                srcs = [torch.from_numpy(x).to(dev) for x in xs[rank]]
                out = torch.empty(n, device=dev)
                torch.cuda.synchronize()
                comm.allreduce_f32(srcs, out=out, scale_exp=inccl.SCALE_AUTO if k == "auto" else k,
                                   stream=comm.stream)
                torch.cuda.synchronize()
                results.append(bool(np.array_equal(out.cpu().numpy().view(np.uint32), want.view(np.uint32))))
            comm.set_average(False)
        if engine in ("ll", "mesh", "meshw"):
            # hipGraph: three calls captured once, replayed with fresh inputs (the
            # call counter lives on the device, so every replay is a new call)
            n = 5000
            bufs = [torch.empty(n, device=dev) for _ in range(2)]
            outs = [torch.empty(n, device=dev) for _ in range(3)]
            cs = torch.cuda.Stream(device=dev)
            graph = torch.cuda.CUDAGraph()
            torch.cuda.synchronize()
            with torch.cuda.graph(graph, stream=cs):
                for o in outs:
                    comm.allreduce_f32(bufs, out=o, scale_exp=24, stream=cs.cuda_stream)
            for rep in range(5):
                xs = _inputs(world, 2, n, 100 + rep)
                want = O.reduce_f32([x for per in xs for x in per], 24)
                for b, x in zip(bufs, xs[rank]):
                    b.copy_(torch.from_numpy(x))
                for o in outs:
                    o.fill_(float("nan"))
                torch.cuda.synchronize()
                graph.replay()
                torch.cuda.synchronize()
                for o in outs:
                    results.append(bool(np.array_equal(o.cpu().numpy().view(np.uint32), want.view(np.uint32))))
            # eager calls keep working after the replays
            comm.allreduce_f32(bufs, out=outs[0], scale_exp=24, stream=comm.stream)
            torch.cuda.synchronize()
            results.append(bool(np.array_equal(outs[0].cpu().numpy().view(np.uint32), want.view(np.uint32))))
            del graph
        # the IPC buffer kind: the ll / mesh kernels poll memory that peers write
        # over xGMI while they run, so it is fine-grained uncached; p2p's
        # buffers are only read after a kernel boundary and a barrier
        if engine not in RCCL_ENGINES:
            results.append(comm.ipc_mem_kind(engine) == (0 if engine == "p2p" else 3))
        comm.destroy()
        grp.destroy()
        q.put((rank, results, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


P2P_CASES = [(2, 1 << 20, 25, 11), (1, 100_003, 20, 12), (2, 65_536 * 3 + 5, "auto", 13), (2, 4 << 20, 24, 14),
             (2, 300_001, 25, 15, 1), (2, 65_536 * 3 + 5, "auto", 16, 1)]
# the ll kernel: tiny, ragged, unaligned, one workgroup, the 256-workgroup cap, the
# 1 MiB slot exactly, and one bucket above it (served by the p2p exchange)
LL_CASES = [(2, 1, 25, 21), (1, 1000, 20, 22), (3, 4099, 25, 23, 1), (2, 65_536 * 3 + 5, "auto", 24),
            (8, 262_144, 22, 25), (2, 262_143, 25, 26, 3), (2, 300_000, 25, 27), (2, 4099, "auto", 28, 1)]


# the mesh kernel: one chunk, many chunks (256 per shard), ragged ends inside and
# beyond the last shard, unaligned buffers, R = 8 local buckets, a 1-element bucket
MESH_CASES = P2P_CASES + [(1, 1, 25, 31), (8, 3_000_017, 22, 32), (2, (8 << 20) + 3, 25, 33, 2),
                          (3, 64 * 3 - 1, 24, 34)]


# W = 8 is the 8-GPU bench's world size: all eight ranks on GPU 0 here
@pytest.mark.parametrize("world,engine", [(2, "p2p"), (3, "p2p"), (4, "p2p"), (8, "p2p"), (2, "ll"), (3, "ll"),
                                          (4, "ll"), (8, "ll"), (2, "mesh"), (3, "mesh"), (4, "mesh"), (8, "mesh"),
                                          (2, "meshw"), (3, "meshw"), (4, "meshw"), (8, "meshw")])
def test_p2p_engine_multiprocess(gpu, world, engine):
    """One process per rank on GPU 0 (IPC between processes; the same code as
    across xGMI).  "p2p" at large buckets, "ll" (one kernel, device flags),
    "mesh" (one persistent kernel, per-chunk flags, push + pull)."""
    cases = {"p2p": P2P_CASES, "ll": LL_CASES, "mesh": MESH_CASES, "meshw": MESH_CASES}[engine]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, cases, q, engine)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, ok, err = q.get(timeout=240)
            res[r] = (ok, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        ok, err = res[r]
        assert err is None, f"rank {r}: {err}"
        assert all(ok), f"rank {r}: {ok}"


def _gpu_count():
    import torch
    return torch.cuda.device_count()   # does not initialise the GPU in this process


def _config45_main(rank, world, port, q, engine, device):
    """BASELINE configs 4 and 5 as the 8-GPU bench runs them, one process per
    GPU: R = 2 resident 256 MiB fp32 buckets per rank (config 4) and one 4 KiB
    bucket (config 5's smallest, one reference message), inputs made on the
    GPU from torch.Generator(seed + rank) as bench.py makes them.  Every rank
    regenerates every rank's inputs on its own GPU and checks its result on a
    lane sample -- 2^16 strided lanes plus both sides of every shard boundary
    -- bit for bit against the oracle."""
    try:
        if engine not in RCCL_ENGINES:
            os.environ["INCCL_ENGINE"] = engine
        os.environ["INCCL_DEVICE"] = str(device)
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        from oracle import oracle as O
        torch.cuda.set_device(device)
        dev = torch.device("cuda", device)
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port, device=device)
        assert grp is not None, "group create failed"
        comm = inccl.inccl_communicator_create(grp, 0)
        if engine in RCCL_ENGINES:
            comm.set_engine(engine)
        assert comm.engine == engine
        results = []
        for n, seed in ((64 << 20, 1000), (1024, 7000)):
            def bucket(r, i):
                g = torch.Generator(device=dev)
                g.manual_seed(seed + 100 * i + r)
                return torch.randn(n, generator=g, device=dev, dtype=torch.float32)
            srcs = [bucket(rank, i) for i in range(2)]
            out = torch.full((n,), float("nan"), device=dev)
            torch.cuda.synchronize()
            for _ in range(3):   # repeated: the bench's back-to-back steps
                comm.allreduce_f32(srcs, out=out, scale_exp=25, stream=comm.stream)
            torch.cuda.synchronize()
            lanes = set(range(0, n, max(1, n // (1 << 16))))
            for w in range(1, world):
                b = w * n // world
                lanes |= {max(0, b - 1), b, min(n - 1, b + 1)}
            idx = torch.tensor(sorted(lanes), dtype=torch.int64, device=dev)
            every = [bucket(r, i)[idx].cpu().numpy() for r in range(world) for i in range(2)]
            want = O.reduce_f32(every, 25)
            got = out[idx].cpu().numpy()
            results.append(bool(np.array_equal(got.view(np.uint32), want.view(np.uint32))))
            results.append(not bool(torch.isnan(out).any()))
            del srcs, out
            torch.cuda.empty_cache()
        comm.destroy()
        grp.destroy()
        q.put((rank, results, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("engine", ["rccl", "ar", "a2a", "p2p", "ll", "mesh", "meshw"])
def test_configs_4_5_one_gpu_per_rank(gpu, engine):
    """BASELINE configs 4 (2 x 256 MiB per rank) and 5 (4 KiB) across every
    visible GPU (at most 8), one process per GPU, each engine, sampled-lane
    oracle parity (_config45_main).  On a one-GPU box the same code runs as a
    world-1 group (the exchange is then trivial, but the harness, the bucket
    generation and the lane check are the ones the multi-GPU run will use)."""
    world = min(_gpu_count(), 8)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_config45_main, args=(r, world, port, q, engine, r)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, ok, err = q.get(timeout=240)
            res[r] = (ok, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        ok, err = res[r]
        assert err is None, f"rank {r}: {err}"
        assert all(ok), f"rank {r}: {ok}"


@pytest.mark.parametrize("engine", ["rccl", "ar", "a2a", "p2p", "ll", "mesh", "meshw"])
def test_engines_one_gpu_per_rank(gpu, engine):
    """the multi-GPU paths with one process per GPU, as the
    8-GPU bench runs them -- RCCL's reduce-scatter / all-gather, all-reduce and
    grouped send/recv with more than one rank, and the IPC engines over real
    xGMI -- every case bit-exact against the oracle.  World = every visible GPU
    (at most 8); skipped on a one-GPU box, where RCCL refuses ranks sharing a
    device and the tests above cover the IPC engines on one card."""
    world = min(_gpu_count(), 8)
    if world < 2:
        pytest.skip("needs two or more GPUs (one process per GPU)")
    cases = {"ll": LL_CASES, "mesh": MESH_CASES, "meshw": MESH_CASES}.get(engine, P2P_CASES)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_rank_main, args=(r, world, port, cases, q, engine, r)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, ok, err = q.get(timeout=240)
            res[r] = (ok, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        ok, err = res[r]
        assert err is None, f"rank {r}: {err}"
        assert all(ok), f"rank {r}: {ok}"


def _timeout_main(rank, port, q, engine="ll"):
    """rank 1 skips the second call: rank 0's kernel must time out, finish, and
    report the failure on the next call instead of hanging the GPU."""
    try:
        os.environ["INCCL_ENGINE"] = engine
        if engine in ("mesh", "meshw"):
            os.environ["INCCL_LL_MAX_BYTES"] = "0"
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        os.environ["INCCL_LL_TIMEOUT_MS"] = "300"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        dev = torch.device("cuda:0")
        grp = inccl.inccl_group_create(2, rank, "127.0.0.1", port=port)
        comm = inccl.inccl_communicator_create(grp, 0)
        x = [torch.ones(4096, device=dev)]
        out = torch.empty(4096, device=dev)
        comm.allreduce_f32(x, out=out, scale_exp=20)
        torch.cuda.synchronize()
        first_ok = bool((out == 2).all().item())
        err = None
        if rank == 0:
            comm.allreduce_f32(x, out=out, scale_exp=20)   # the peer never arrives
            torch.cuda.synchronize()
            try:
                comm.allreduce_f32(x, out=out, scale_exp=20)
            except Exception as e:  # noqa: BLE001
                err = repr(e)
        # collective recovery: the timed-out rank reports it, both rebuild the
        # engine's IPC buffers, and the communicator works again
        had = comm.clear_error()
        out.fill_(0)
        torch.cuda.synchronize()
        comm.allreduce_f32(x, out=out, scale_exp=20)
        torch.cuda.synchronize()
        after_ok = bool((out == 2).all().item())
        kind = comm.ipc_mem_kind(engine)
        comm.destroy()
        grp.destroy()
        q.put((rank, {"first": first_ok, "after_clear": after_ok, "had": had == (rank == 0),
                      "uncached": kind == 3}, err))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, {"crash": False}, "crash " + repr(e)))


@pytest.mark.parametrize("engine", ["ll", "mesh", "meshw"])
def test_engine_peer_timeout(gpu, engine):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_timeout_main, args=(r, port, q, engine)) for r in range(2)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(2):
            r, ok, err = q.get(timeout=240)
            res[r] = (ok, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    assert all(res[0][0].values()) and all(res[1][0].values()), res
    assert res[1][1] is None, res
    assert res[0][1] is not None and "timed out" in res[0][1], res
    if engine in ("mesh", "meshw"):
        # the report (DESIGN.md "Mesh reduce-scatter route", liveness): the
        # expired wait, the rank's progress, and the flag census -- one chunk
        # per shard here: rank 0's own partial arrived, rank 1's never did;
        # rank 0's pushes reached both signal arrays
        e = res[0][1]
        # every wait of the call expires at about the same time (rank 0's own
        # reduce and ready never happen either); the last report stays
        assert "reduce's arrival flag of chunk 0" in e or "gather's ready flag of chunk 0" in e, e
        assert "pushes finished per destination [1,1]" in e, e
        assert "arrived from [1,0] of 1" in e and "mine at [1,1] of 1" in e, e
        assert "clock ms: timeout" in e, e


def _refapi_main(rank, world, port, q, engine):
    """The reference's own caller, one process per rank (host.c:28-59): group +
    communicator create, inccl_allreduce_write / _sendrecv on host int32 arrays,
    plus the device int32 allreduce -- over the IPC engines, no RCCL."""
    try:
        if engine != "default":
            os.environ["INCCL_ENGINE"] = engine
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port)
        assert grp is not None, "group create failed"
        comm = inccl.inccl_communicator_create(grp, 4096 * 4)       # host.c:41
        assert comm is not None
        res = {"engine": comm.engine}
        n = 4096                                                     # host.c:20-25
        src = (np.arange(n, dtype=np.int64) * (rank + 1)).astype(np.int32)
        for name, fn in (("write", inccl.inccl_allreduce_write), ("sendrecv", inccl.inccl_allreduce_sendrecv)):
            dst = np.zeros(n, np.int32)
            fn(comm, src, n, dst)
            res[name] = bool(np.array_equal(dst, np.arange(n, dtype=np.int64).astype(np.int32)
                                            * (world * (world + 1) // 2)))   # host.c:51-55 at world 2: 3*i
        m = 1024 * 37                                                # whole messages, int32 wrap-around
        xs = [np.random.default_rng(900 + r).integers(-2 ** 31, 2 ** 31, m, dtype=np.int64).astype(np.int32)
              for r in range(world)]
        xs[0][:4] = [2 ** 31 - 1, -2 ** 31, -1, 0]
        want = np.sum([x.astype(np.uint32) for x in xs], axis=0, dtype=np.uint32).view(np.int32)
        dst = np.zeros(m, np.int32)
        comm.allreduce_write(xs[rank], m, dst)
        res["random"] = bool(np.array_equal(dst, want))
        reg_src, reg_dst = xs[rank].copy(), np.zeros(m, np.int32)
        comm.host_register(reg_src)
        comm.host_register(reg_dst)
        comm.allreduce_write(reg_src, m, reg_dst)
        res["registered"] = bool(np.array_equal(reg_dst, want))
        k = 100_003                                                  # device int32 allreduce, ragged
        dev = torch.device("cuda:0")
        qs = [np.random.default_rng(950 + r).integers(-2 ** 31, 2 ** 31, k, dtype=np.int64).astype(np.int32)
              for r in range(world)]
        got = comm.allreduce_q32(torch.from_numpy(qs[rank]).to(dev))
        torch.cuda.synchronize()
        want_q = np.sum([x.astype(np.uint32) for x in qs], axis=0, dtype=np.uint32).view(np.int32)
        res["device"] = bool(np.array_equal(got.cpu().numpy(), want_q))
        comm.destroy()
        grp.destroy()
        q.put((rank, res, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("world,engine", [(2, "p2p"), (3, "p2p"), (2, "default")])
def test_reference_api_multiprocess(gpu, world, engine):
    """host.c's known answer with one process per rank on GPU 0.  "default"
    leaves the engine to the communicator: RCCL refuses ranks sharing a GPU, so
    every rank must agree to fall back to the p2p engine."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_refapi_main, args=(r, world, port, q, engine)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, ok, err = q.get(timeout=240)
            res[r] = (ok, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        ok, err = res[r]
        assert err is None, f"rank {r}: {err}"
        assert ok.pop("engine") == "p2p", ok
        assert all(ok.values()), f"rank {r}: {ok}"


def _host_path_main(rank, world, port, q, engine):
    """BASELINE config 3 with more than one rank: every rank's fp32 gradient in
    pinned host memory, buckets through the H2D / allreduce / D2H pipeline,
    where each bucket's allreduce is a multi-process exchange."""
    try:
        os.environ["INCCL_ENGINE"] = engine
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        from oracle import oracle as O
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port)
        comm = inccl.inccl_communicator_create(grp, 0)
        res = {}
        for n, bucket in (((64 << 20) // 4 + 333, 16 << 20), (1_000_003, 1 << 20)):
            xs = [np.random.default_rng(40 + r).standard_normal(n).astype(np.float32) for r in range(world)]
            want = O.reduce_f32(xs, 24)
            x = torch.from_numpy(xs[rank]).pin_memory()
            y = torch.full((n,), float("nan")).pin_memory()
            for rep in range(2):
                comm.allreduce_f32_host(x, y, scale_exp=24, bucket_bytes=bucket)
                res[f"n={n} rep={rep}"] = bool(np.array_equal(y.numpy().view(np.uint32), want.view(np.uint32)))
                y.fill_(float("nan"))
        comm.destroy()
        grp.destroy()
        q.put((rank, res, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("world,engine", [(2, "p2p"), (3, "mesh")])
def test_host_path_multiprocess(gpu, world, engine):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_host_path_main, args=(r, world, port, q, engine)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, ok, err = q.get(timeout=240)
            res[r] = (ok, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        ok, err = res[r]
        assert err is None, f"rank {r}: {err}"
        assert all(ok.values()), f"rank {r}: {ok}"


def _uneven_main(rank, world, port, q, engine, n, calls):
    """Back-to-back calls on one stream with no host synchronisation, each rank
    delaying its own kernels by a different random amount before every call
    (a spinning kernel on the same stream), so the ranks arrive at each call's
    flags unevenly; inputs rotate over three sets; every output is copied on
    the stream right after its call and checked at the end."""
    try:
        os.environ["INCCL_ENGINE"] = engine
        os.environ["INCCL_LL_MAX_BYTES"] = "0" if engine != "ll" else str(max(4 * n, 1 << 20))
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        os.environ["INCCL_LL_TIMEOUT_MS"] = "5000"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        from oracle import oracle as O
        dev = torch.device("cuda:0")
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port)
        assert grp is not None, "group create failed"
        comm = inccl.inccl_communicator_create(grp, 0)
        assert comm.engine == engine
        sets = [_inputs(world, 2, n, 500 + 10 * s) for s in range(3)]
        wants = [O.reduce_f32([x for per in xs for x in per], 24).view(np.uint32) for xs in sets]
        srcs = [[torch.from_numpy(x).to(dev) for x in xs[rank]] for xs in sets]
        out = torch.empty(n, device=dev)
        hist = torch.empty((calls, n), device=dev)
        st = torch.cuda.Stream(device=dev)
        torch.cuda.synchronize()
        comm.allreduce_f32(srcs[0], out=out, scale_exp=24, stream=st.cuda_stream)   # collective setup
        torch.cuda.synchronize()
        rng = np.random.default_rng(1234 + rank)
        delays = rng.integers(0, 200_000, calls)   # GPU clock cycles: 0 to ~80 us
        with torch.cuda.stream(st):
            for i in range(calls):
                if delays[i] > 20_000:
                    torch.cuda._sleep(int(delays[i]))
                comm.allreduce_f32(srcs[i % 3], out=out, scale_exp=24, stream=st.cuda_stream)
                hist[i].copy_(out)
        torch.cuda.synchronize()
        got = hist.cpu().numpy().view(np.uint32)
        bad = [i for i in range(calls) if not np.array_equal(got[i], wants[i % 3])]
        comm.destroy()
        grp.destroy()
        q.put((rank, bad, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("engine,world,n", [("ll", 2, 65_536), ("ll", 3, 262_144), ("mesh", 3, 1 << 20),
                                            ("meshw", 3, 1 << 20), ("mesh", 4, 300_001), ("p2p", 3, 1 << 20)])
def test_engines_uneven_arrival(gpu, engine, world, n):
    """The flag hand-offs under uneven load (MI355X_MICROARCH.md: "test every
    hand-off under uneven load"): 48 back-to-back calls per rank, each rank's
    kernels delayed by its own random 0-80 us before every call, three input
    sets in rotation, every output bit-exact vs the oracle."""
    calls = 48
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_uneven_main, args=(r, world, port, q, engine, n, calls)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, bad, err = q.get(timeout=240)
            res[r] = (bad, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        bad, err = res[r]
        assert err is None, f"rank {r}: {err}"
        assert bad == [], f"rank {r}: wrong outputs at calls {bad}"
