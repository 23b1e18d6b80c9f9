"""Reduce-scatter (gpu): inccl_reduce_scatter_f32 / _bf16 / _f16, the
allreduce's first half for sharded-gradient callers.  Rank r's result must be
bit-identical to elements [r*shard, (r+1)*shard) of the oracle's reduce of every
rank's buckets (orc_reduce_f32 / _bf16 / _f16), over every route: the fused
world-1 kernel, RCCL's ncclReduceScatter at world 1, the in-process transport
(W = 2..4, aligned and ragged shards), and one process per rank on the IPC
engines (p2p pull-reduce into the shard; a ragged shard through the int32
allreduce), with average mode and repeated calls (buffer reuse)."""
import multiprocessing as mp
import os
import socket

import numpy as np
import pytest

from conftest import ROOT
from test_gpu_comm import _run_ranks

pytestmark = pytest.mark.gpu

KINDS = ("f32", "bf16", "f16")


def _bucket(rng, n, kind):
    x = rng.standard_normal(n).astype(np.float32) * 2.0
    if kind == "f32":
        return x
    if kind == "bf16":
        return (x.view(np.uint32) >> 16).astype(np.uint16)
    return x.astype(np.float16).view(np.uint16)


def _dev(h, dev, kind):
    import torch
    if kind == "f32":
        return torch.from_numpy(h).to(dev)
    t = torch.from_numpy(h.view(np.int16)).to(dev)
    return t.view(torch.bfloat16 if kind == "bf16" else torch.float16)


def _host(t, kind):
    import torch
    if kind == "f32":
        return t.cpu().numpy()
    return t.view(torch.int16).cpu().numpy().view(np.uint16)


def _reduce(O, every, kind, k):
    return {"f32": O.reduce_f32, "bf16": O.reduce_bf16, "f16": O.reduce_f16}[kind](every, k)


def _auto_k(O, every, kind, RW):
    return O.choose_scale({"f32": O.absmax, "bf16": O.absmax_bf16, "f16": O.absmax_f16}[kind](every), RW)


@pytest.mark.parametrize("kind", KINDS)
@pytest.mark.parametrize("world,shard,R,k", [(1, 4099, 2, "auto"), (2, 4096, 2, 25), (3, 1001, 1, "auto"),
                                             (4, 65_540, 2, "auto"), (2, 262_144, 1, 23)])
def test_reduce_scatter_local(gpu, orc, kind, world, shard, R, k):
    import torch
    from container_inc_amd import inccl
    n = world * shard
    rng = np.random.default_rng(world * 100 + shard % 97 + len(kind))
    hs = [[_bucket(rng, n, kind) for _ in range(R)] for _ in range(world)]
    every = [h for per in hs for h in per]
    kk = _auto_k(orc, every, kind, world * R) if k == "auto" else k
    want = _reduce(orc, every, kind, kk)
    hub = f"rs-{kind}-{world}-{shard}-{R}"

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, hub)
        comm = inccl.inccl_communicator_create(grp, 0)
        srcs = [_dev(h, gpu, kind) for h in hs[r]]
        res = []
        for _ in range(2):   # workspace reuse
            out = comm.reduce_scatter(srcs, scale_exp=inccl.SCALE_AUTO if k == "auto" else k, stream=comm.stream)
            torch.cuda.synchronize()
            res.append(_host(out, kind))
        comm.barrier()
        comm.destroy()
        grp.destroy()
        return res

    for r, res in enumerate(_run_ranks(world, rank)):
        for got in res:
            np.testing.assert_array_equal(got, want[r * shard:(r + 1) * shard])


@pytest.mark.parametrize("world", [2, 4])
def test_reduce_scatter_average(gpu, orc, world):
    """inccl_comm_set_average: the shard of the mean, bit-identical to sum / W."""
    import torch
    from container_inc_amd import inccl
    shard = 8192
    n = world * shard
    rng = np.random.default_rng(world)
    hs = [[_bucket(rng, n, "f32")] for _ in range(world)]
    every = [h for per in hs for h in per]
    want = orc.reduce_f32(every, 25) / np.float32(world)

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, f"rs-avg-{world}")
        comm = inccl.inccl_communicator_create(grp, 0)
        comm.set_average(True)
        out = comm.reduce_scatter([_dev(hs[r][0], gpu, "f32")], scale_exp=25, stream=comm.stream)
        torch.cuda.synchronize()
        got = _host(out, "f32")
        comm.barrier()
        comm.destroy()
        grp.destroy()
        return got

    for r, got in enumerate(_run_ranks(world, rank)):
        np.testing.assert_array_equal(got.view(np.uint32), want[r * shard:(r + 1) * shard].view(np.uint32))


def test_reduce_scatter_rccl_world1(gpu, orc, monkeypatch):
    """RCCL at world 1 through the sharded route: a real ncclReduceScatter."""
    import torch
    from container_inc_amd import inccl
    monkeypatch.setenv("INCCL_FORCE_RCCL", "1")
    monkeypatch.setenv("INCCL_FORCE_SHARDED", "1")
    monkeypatch.setenv("INCCL_MASTER_PORT", "0")
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    assert grp.transport == "rccl"
    rng = np.random.default_rng(3)
    for kind in KINDS:
        hs = [_bucket(rng, 50_001, kind) for _ in range(2)]
        want = _reduce(orc, hs, kind, _auto_k(orc, hs, kind, 2))
        for eng in ("rccl", "ar"):
            comm.set_engine(eng)
            out = comm.reduce_scatter([_dev(h, gpu, kind) for h in hs], stream=comm.stream)
            torch.cuda.synchronize()
            np.testing.assert_array_equal(_host(out, kind), want, err_msg=f"{kind} {eng}")
    with pytest.raises(Exception):
        comm.reduce_scatter([torch.zeros(10, device=gpu)], out=torch.zeros(3, device=gpu))   # wrong shard size
    x = torch.zeros(128, device=gpu)
    with pytest.raises(inccl.IncclError, match="overlaps"):   # a full-size dst that overlaps the source
        comm.reduce_scatter([x[:64]], out=x[32:96])
    comm.destroy()
    grp.destroy()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _ipc_rank(rank, world, port, q, engine, mesh_rs=None, misalign=False):
    """One process of the multi-process tests.  mesh_rs: None = the default
    (the mesh engines' own route), "0" = INCCL_MESH_RS=0 (the p2p pull-reduce).
    misalign: odd ranks pass a dst one element into a buffer, so that it is not
    16-B (fp32) or 8-B (16-bit) aligned while the even ranks' is: every rank
    must still take the same route (api.c reduce_scatter_body)."""
    try:
        os.environ["INCCL_ENGINE"] = engine
        if mesh_rs is not None:
            os.environ["INCCL_MESH_RS"] = mesh_rs
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        from oracle import oracle as O
        dev = torch.device("cuda", 0)
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port, device=0)
        comm = inccl.inccl_communicator_create(grp, 0)
        ok = []
        mesh_route = engine in ("mesh", "meshw") and mesh_rs != "0"
        for kind in KINDS:
            for shard, R, seed in ((1 << 18, 2, 1), (1001, 1, 2), (4096, 2, 3)):   # 1001: the int32-allreduce route
                n = world * shard
                hs = [[_bucket(np.random.default_rng(seed * 1000 + r * 10 + j), n, kind) for j in range(R)]
                      for r in range(world)]
                every = [h for per in hs for h in per]
                want = _reduce(O, every, kind, _auto_k(O, every, kind, world * R))[rank * shard:(rank + 1) * shard]
                srcs = [_dev(h, dev, kind) for h in hs[rank]]
                for _ in range(2):
                    out = None
                    if misalign and rank % 2:
                        out = torch.empty(shard + 1, dtype=srcs[0].dtype, device=dev)[1:]
                    out = comm.reduce_scatter(srcs, out=out, stream=comm.stream)
                    torch.cuda.synchronize()
                    ok.append(bool(np.array_equal(_host(out, kind), want)))
                if engine == "ll" and kind == "f32" and shard == 4096:
                    comm.ipc_mem_kind("ll")   # raises unless the ll kernel's buffers exist: the ll route ran
                if engine in ("mesh", "meshw") and shard == 1 << 18:
                    if mesh_route:
                        comm.ipc_mem_kind("mesh")   # the persistent kernel's reduce-scatter route ran
                        if kind == "f32":   # ... and the p2p pull-reduce did not (shard 1001 comes later)
                            with pytest.raises(Exception):
                                comm.ipc_mem_kind("p2p")
                    else:
                        comm.ipc_mem_kind("p2p")    # INCCL_MESH_RS=0: the p2p pull-reduce
        if misalign:   # the 16-bit allreduce: a dst that is not 4-B aligned on odd ranks (api.c allreduce_16_body)
            for kind in ("bf16", "f16"):
                n = world * 4096 + 2
                hs = [_bucket(np.random.default_rng(77 + r), n, kind) for r in range(world)]
                want = _reduce(O, hs, kind, 20)
                src = _dev(hs[rank], dev, kind)
                out = torch.empty(n + 1, dtype=src.dtype, device=dev)
                out = out[1:] if rank % 2 else out[:n]
                fn = comm.allreduce_bf16 if kind == "bf16" else comm.allreduce_f16
                fn([src], out=out, scale_exp=20, stream=comm.stream)
                torch.cuda.synchronize()
                ok.append(bool(np.array_equal(_host(out, kind), want)))
        comm.barrier()
        comm.destroy()
        grp.destroy()
        q.put((rank, ok, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


def _run_mp(world, target, *args, timeout=240):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, ok, err = q.get(timeout=timeout)
            res[r] = (ok, err)
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    errs = {r: res[r][1] for r in range(world) if res[r][1] is not None}
    assert not errs, f"errors by rank: {errs}"   # every rank's, not only the first
    bad = {r: res[r][0] for r in range(world) if not all(res[r][0])}
    assert not bad, f"mismatches by rank: {bad}"


def _run_ipc(world, engine, mesh_rs=None, misalign=False):
    _run_mp(world, _ipc_rank, engine, mesh_rs, misalign)


@pytest.mark.parametrize("world,engine", [(2, "p2p"), (3, "p2p"), (2, "mesh"), (3, "mesh"), (4, "meshw"), (2, "ll"),
                                         (4, "ll")])
def test_reduce_scatter_ipc_multiprocess(gpu, world, engine):
    """ll: a small fp32 bucket (shard 4096) through the one-kernel ll reduce-
    scatter; mesh / meshw: their persistent kernel's own route (shards of whole
    64-element groups; the allreduce's instructions with the other ranks'
    gathers reduced to their waits, DESIGN.md "Mesh reduce-scatter route");
    the others through the p2p pull-reduce or the int32 allreduce (shard
    1001)."""
    _run_ipc(world, engine)


@pytest.mark.parametrize("world,engine", [(2, "mesh"), (3, "meshw")])
def test_reduce_scatter_mesh_route_off(gpu, world, engine):
    """INCCL_MESH_RS=0: the mesh engines reduce-scatter through the p2p
    pull-reduce instead."""
    _run_ipc(world, engine, mesh_rs="0")


@pytest.mark.parametrize("world,engine", [(2, "p2p"), (2, "mesh"), (3, "ll")])
def test_reduce_scatter_misaligned_dst_on_some_ranks(gpu, world, engine):
    """Odd ranks pass a dst that is not 16-B / 8-B aligned, even ranks an
    aligned one.  The route must not depend on it: before, the
    misaligned ranks fell back to the int32 allreduce while the others ran the
    pull-reduce or the mesh kernel -- mismatched barriers."""
    _run_ipc(world, engine, misalign=True)


def _mode_switch_rank(rank, world, port, q, shard_log2):
    """The mesh engines' kernel across mode switches on one communicator:
    allreduce <-> reduce-scatter, fp32 <-> bf16, mesh <-> meshw, and a regrow,
    with exact fixed-point data (rank r's bucket in step i is (r + 1) * m * b,
    m = 1 + i % 3 and b a multiple of 2^-12 with |b| < 1/2: every partial is
    exact at k = 20, and no step's partials equal the previous step's), so every
    call is checked exactly without the oracle."""
    where = ["setup"]
    try:
        os.environ["INCCL_ENGINE"] = "mesh"
        # the bounded wait is a liveness check, not a latency one: four ranks
        # share one GPU, and while another process held high-priority queues on
        # it they were time-sliced and a wait expired (DESIGN.md "Mesh
        # reduce-scatter route", liveness); a stall still fails, with the
        # expired wait, the ranks' progress and the raised flags in the error
        os.environ["INCCL_LL_TIMEOUT_MS"] = "30000"
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "120"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        dev = torch.device("cuda", 0)
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port, device=0)
        comm = inccl.inccl_communicator_create(grp, 0)
        ok = []
        for lg in (shard_log2 - 2, shard_log2):   # the second size regrows the buffers (beyond 2^19 elements)
            shard = 1 << lg
            n = world * shard
            i = torch.arange(n, device=dev, dtype=torch.int64)
            b = ((i % 4093) - 2046).to(torch.float32) * 2.0 ** -12
            x = b * float(rank + 1)

            def want_of(dt, m):   # the exact sum of every rank's bucket as `dt`, rounded once to `dt`
                acc = torch.zeros(n, device=dev, dtype=torch.float32)
                for r in range(world):
                    acc += (b * float((r + 1) * m)).to(dt).float()
                return acc.to(dt)

            f32, b16 = torch.float32, torch.bfloat16
            for step, (eng, op, dt) in enumerate([("mesh", "ar", f32), ("mesh", "rs", f32), ("mesh", "ar", b16),
                                                  ("mesh", "rs", b16), ("meshw", "rs", f32), ("meshw", "ar", f32),
                                                  ("mesh", "rs", f32), ("meshw", "ar", b16), ("meshw", "rs", b16),
                                                  ("mesh", "ar", f32)]):
                where[0] = f"shard 2^{lg} step {step} ({eng} {op} {dt})"
                comm.set_engine(eng)
                m = 1 + step % 3   # a bucket unlike the previous step's: a partial read stale would show
                src = (x * float(m)).to(dt)
                torch.cuda.synchronize()   # src is made on torch's stream; the library runs on comm.stream
                if op == "ar":
                    out = (comm.allreduce_f32([src], scale_exp=20, stream=comm.stream) if dt == torch.float32 else
                           comm.allreduce_bf16([src], out=torch.empty_like(src), scale_exp=20, stream=comm.stream))
                    want = want_of(dt, m)
                else:
                    out = comm.reduce_scatter([src], scale_exp=20, stream=comm.stream)
                    want = want_of(dt, m)[rank * shard:(rank + 1) * shard]
                torch.cuda.synchronize()
                ok.append(bool(torch.equal(out, want)))
            comm.ipc_mem_kind("mesh")
        comm.barrier()
        comm.destroy()
        grp.destroy()
        q.put((rank, ok, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, f"{where[0]}: {e!r}"))


@pytest.mark.parametrize("world,shard_log2", [(2, 16), (3, 14), (4, 22)])
def test_mesh_mode_switches(gpu, world, shard_log2):
    """One communicator, the mesh kernel in every mode in turn (CPU model:
    tests/test_mesh_schedule_model.py); (4, 2^22) is the configuration in
    which round 5's reduce-scatter route faulted."""
    _run_mp(world, _mode_switch_rank, shard_log2)


def test_mesh_w4_beside_a_live_communicator(gpu):
    """Liveness regression (DESIGN.md "Mesh reduce-scatter route", liveness):
    this process keeps a one-rank communicator (which holds the host paths'
    high-priority copy streams) alive while four rank processes run the
    mode-switch sequence on the same GPU.  While every communicator created
    those streams at creation, the ranks included, this took 54-93 s or timed
    out (the ranks' persistent kernels time-sliced); now a multi-rank
    communicator makes them on its first host-path call, and it takes about
    3 s."""
    import time
    from container_inc_amd import inccl
    grp = inccl.inccl_group_create_local(1, 0, "liveness")
    comm = inccl.inccl_communicator_create(grp, 0)
    try:
        t0 = time.monotonic()
        _run_mp(4, _mode_switch_rank, 22)
        took = time.monotonic() - t0
        assert took < 30, f"four ranks took {took:.1f} s beside a live communicator"
    finally:
        comm.destroy()
        grp.destroy()


def test_calls_on_alternating_streams(gpu, orc):
    """A communicator's calls share its workspaces (int32 partials, the auto
    scale's word): back-to-back calls on two streams, no host sync between them,
    inputs of different magnitude (so different scales), must each match the
    oracle -- the second call waits for the first (api.c ws_enter)."""
    import torch
    from container_inc_amd import inccl
    world, n = 2, 1 << 22
    rng = np.random.default_rng(11)
    xs = [[rng.standard_normal(n).astype(np.float32)] for _ in range(world)]
    ys = [[(rng.standard_normal(n) * 1000.0).astype(np.float32)] for _ in range(world)]
    want_x = _reduce(orc, [h for per in xs for h in per], "f32", _auto_k(orc, [h for per in xs for h in per], "f32", world))
    want_y = _reduce(orc, [h for per in ys for h in per], "f32", _auto_k(orc, [h for per in ys for h in per], "f32", world))

    def rank(r):
        grp = inccl.inccl_group_create_local(world, r, "alt-streams")
        comm = inccl.inccl_communicator_create(grp, 0)
        sa, sb = torch.cuda.Stream(device=gpu), torch.cuda.Stream(device=gpu)
        dx, dy = _dev(xs[r][0], gpu, "f32"), _dev(ys[r][0], gpu, "f32")
        torch.cuda.synchronize()
        res = []
        for _ in range(3):
            ox = comm.allreduce_f32([dx], scale_exp=inccl.SCALE_AUTO, stream=sa.cuda_stream)
            oy = comm.allreduce_f32([dy], scale_exp=inccl.SCALE_AUTO, stream=sb.cuda_stream)
            rx = comm.reduce_scatter([dx], stream=sa.cuda_stream)
            torch.cuda.synchronize()
            res.append((_host(ox, "f32"), _host(oy, "f32"), _host(rx, "f32")))
        comm.barrier()
        comm.destroy()
        grp.destroy()
        return res

    shard = n // world
    for r, res in enumerate(_run_ranks(world, rank)):
        for gx, gy, grs in res:
            np.testing.assert_array_equal(gx, want_x)
            np.testing.assert_array_equal(gy, want_y)
            np.testing.assert_array_equal(grs, want_x[r * shard:(r + 1) * shard])


@pytest.mark.parametrize("engine", ["rccl", "ar"])
def test_reduce_scatter_graph_capture_world1(gpu, orc, monkeypatch, engine):
    """inccl_reduce_scatter_f32 captured into a hipGraph on the RCCL engines
    (world 1, the sharded route forced: a real ncclReduceScatter / ncclAllReduce
    in the graph): three captured calls replayed with fresh inputs, bit-exact."""
    import torch
    from container_inc_amd import inccl
    monkeypatch.setenv("INCCL_FORCE_RCCL", "1")
    monkeypatch.setenv("INCCL_FORCE_SHARDED", "1")
    monkeypatch.setenv("INCCL_MASTER_PORT", "0")
    grp = inccl.inccl_group_create(1, 0, "127.0.0.1")
    comm = inccl.inccl_communicator_create(grp, 0)
    comm.set_engine(engine)
    n = (1 << 18) + 64
    bufs = [torch.empty(n, device=gpu) for _ in range(2)]
    outs = [torch.empty(n, device=gpu) for _ in range(3)]
    st = torch.cuda.Stream(device=gpu)
    comm.reduce_scatter(bufs, out=outs[0], scale_exp=24, stream=st.cuda_stream)   # workspaces sized eagerly
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=st):
        for o in outs:
            comm.reduce_scatter(bufs, out=o, scale_exp=24, stream=st.cuda_stream)
    rng = np.random.default_rng(79)
    for _ in range(3):
        hs = [_bucket(rng, n, "f32") for _ in range(2)]
        for b, h in zip(bufs, hs):
            b.copy_(torch.from_numpy(h).to(gpu))
        for o in outs:
            o.fill_(float("nan"))
        torch.cuda.synchronize()
        graph.replay()
        torch.cuda.synchronize()
        want = orc.reduce_f32(hs, 24)
        for o in outs:
            np.testing.assert_array_equal(_host(o, "f32"), want)
    del graph
    comm.destroy()
    grp.destroy()


def _knobs_rank(rank, world, port, q, case):
    """knobs read from each process's environment are agreed when
    the communicator is created (api.c agree_knobs)."""
    try:
        os.environ["INCCL_DEVICE"] = "0"
        os.environ["INCCL_BOOT_TIMEOUT"] = "60"
        if case == "mesh_rs":   # only rank 1 opts out of the mesh route: every rank must take the p2p route
            os.environ["INCCL_ENGINE"] = "mesh"
            if rank == 1:
                os.environ["INCCL_MESH_RS"] = "0"
        else:                   # different engines: creation fails on every rank, naming both
            os.environ["INCCL_ENGINE"] = "mesh" if rank == 0 else "p2p"
        import sys
        sys.path.insert(0, ROOT)
        import torch
        from container_inc_amd import inccl
        from oracle import oracle as O
        dev = torch.device("cuda", 0)
        grp = inccl.inccl_group_create(world, rank, "127.0.0.1", port=port, device=0)
        comm = inccl.inccl_communicator_create(grp, 0)
        if case != "mesh_rs":
            from container_inc_amd import load
            ok = [comm is None and "INCCL_ENGINE differs" in load().inccl_last_error().decode()]
            grp.destroy()
            q.put((rank, ok, None))
            return
        shard = 1 << 16
        hs = [_bucket(np.random.default_rng(40 + r), world * shard, "f32") for r in range(world)]
        want = O.reduce_f32(hs, 25)[rank * shard:(rank + 1) * shard]
        out = comm.reduce_scatter([_dev(hs[rank], dev, "f32")], scale_exp=25, stream=comm.stream)
        torch.cuda.synchronize()
        ok = [bool(np.array_equal(_host(out, "f32"), want))]
        comm.ipc_mem_kind("p2p")   # the agreed route: the p2p pull-reduce on both ranks
        comm.barrier()
        comm.destroy()
        grp.destroy()
        q.put((rank, ok, None))
    except BaseException as e:  # noqa: BLE001
        q.put((rank, None, repr(e)))


@pytest.mark.parametrize("case", ["mesh_rs", "engine"])
def test_environment_knobs_agreed_across_ranks(gpu, case):
    _run_mp(2, _knobs_rank, case, timeout=120)
