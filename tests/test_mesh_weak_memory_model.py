"""Weak-memory CPU model of the mesh engine's persistent kernel
(container_inc_amd/csrc/inccl_mesh.hip: k_mesh, do_push, do_reduce, do_gather).

tests/test_mesh_schedule_model.py checks the ticket schedule under sequentially
consistent memory, with every work item one atomic step.  This model breaks the
items into the kernel's instructions and runs them on a memory that is as weak
as the hardware the kernel is written for (the conditions of MI355X_MICROARCH.md
"Valid forms" that the kernel relies on, and nothing more):

  * every store is posted: it lands at some later, arbitrary point, and the
    stores of one workgroup land in any order -- so a flag may become visible
    before the data stored ahead of it, unless the storing workgroup waited for
    its stores (`s_waitcnt vmcnt(0)`, then the workgroup barrier) in between;
  * a load marked sc0|sc1 (system scope: every inbox / result / flag load of
    the kernel) returns the landed value; a load NOT so marked may return any
    value the location held since the reading rank's kernel started (a line
    cached and never refreshed) -- used only by the mutant below;
  * a kernel's end publishes only its own rank's stores: a rank's call ends
    when its workgroups retired and THEIR stores landed; stores that peers
    posted into this rank's memory may still be in flight;
  * memory is addressed in 2-byte units, so calls of different element widths
    (fp32 / 16-bit results), chunk lengths (buffer regrow: the chunk follows the
    shard) and modes overlap in the same bytes, as they do on the GPU.

Calls switch between allreduce and reduce-scatter, fp32 and 16-bit results,
and mesh (pull) and meshw (push_res) between calls on one communicator.  Every
load of a partial or a result asserts that it holds the current call's value;
after each call the host check reads the rank's dst.

Designs:
  "r6"    the kernel as built: reduce-scatter = the allreduce's instructions,
          gather(c, me) copying my result chunk into dst, the other gathers
          only waiting (round 6);
  "r5rs"  round 5's reduce-scatter: each reduce storing straight into dst, every
          gather only waiting.
Both hold under this model (DESIGN.md "Mesh reduce-scatter route": round 5's
failures were not a protocol error).  Mutants that drop one of the kernel's
orderings must fail -- the model has teeth.
"""
import random

import pytest


class _Violation(AssertionError):
    pass


class _Mem:
    def __init__(self, rng):
        self.rng = rng
        self.t = 0
        self.val = {}    # loc -> landed value
        self.hist = {}   # loc -> [(time, value)]

    def land(self, loc, v):
        self.t += 1
        self.val[loc] = v
        self.hist.setdefault(loc, []).append((self.t, v))

    def load_sc(self, loc):
        return self.val.get(loc)

    def load_plain(self, loc, since):
        """any value the location held at or after time `since`"""
        h = self.hist.get(loc, [])
        older = [v for t, v in h if t <= since]
        cand = ([older[-1]] if older else [None]) + [v for t, v in h if t > since]
        return self.rng.choice(cand)


class _Wg:
    def __init__(self, rank, gen_fn):
        self.rank = rank
        self.pending = []   # posted stores: (loc, value)
        self.gen = gen_fn(self)
        self.done = False
        self.item = None


def _run(W, G, calls, seed, design="r6", mutant=None):
    """calls: list of per-call dicts {mode: "ar"|"rs", es: 1|2 units per result
    element, L: elements per chunk, nchunks, lag, push_res}."""
    rng = random.Random(seed)
    mem = _Mem(rng)
    per_slot = 2 * W + 1

    class Rank:
        pass

    ranks = []
    for me in range(W):
        r = Rank()
        r.me, r.call, r.epoch_done, r.ticket, r.retired = me, 0, 0, 0, 0
        r.running, r.wgs, r.kstart = False, [], 0
        ranks.append(r)

    def waitcnt(wg):
        if mutant == "no_wait_push" and wg.item == "push":
            return
        if mutant == "no_wait_reduce" and wg.item == "reduce":
            return
        while wg.pending:
            yield "blocked"

    def wait_flag(rk, loc, e):
        while (mem.load_sc(loc) or 0) < e:
            yield "blocked"

    def units_res(cfg, c):
        L, es = cfg["L"], cfg["es"]
        return range(c * L * es, (c + 1) * L * es)

    def units_inbox(cfg, c):
        L = cfg["L"]
        return range(c * L * 2, (c + 1) * L * 2)   # int32 partials: 2 units per element

    def units_dst_ar(cfg, j, c):   # allreduce dst: the whole bucket, shard j at j * shard
        L, es, nch = cfg["L"], cfg["es"], cfg["nchunks"]
        base = j * nch * L * es
        return range(base + c * L * es, base + (c + 1) * L * es)

    def check(v, want, what):
        if v != want:
            raise _Violation(f"{what}: read {v}, want {want}")

    def wg_body(rk, cfg, e):
        mode, push_res = cfg["mode"], cfg["push_res"]
        nch, lag = cfg["nchunks"], cfg["lag"]
        total = (nch + 2 * lag) * per_slot
        rs = mode == "rs"

        def gen(wg):
            me = rk.me
            while True:
                t = rk.ticket
                rk.ticket += 1
                yield "step"
                if t >= total:
                    break
                s, pos = divmod(t, per_slot)
                if pos < W:
                    if s >= nch:
                        continue
                    c, j = s, (me + 1 + pos) % W
                    wg.item = "push"
                    for u in units_inbox(cfg, c):   # the partial, into rank j's inbox slot me
                        wg.pending.append((("inbox", j, me, u), (e, me)))
                        yield "step"
                    yield from waitcnt(wg)
                    wg.pending.append((("arrive", j, me, c), e))   # the flag: posted, not waited
                    yield "step"
                elif pos == W:
                    c = s - lag
                    if not 0 <= c < nch:
                        continue
                    wg.item = "reduce"
                    for j in range(W):
                        yield from wait_flag(rk, ("arrive", me, j, c), e)
                    for j in range(W):
                        for u in units_inbox(cfg, c):
                            loc = ("inbox", me, j, u)
                            v = mem.load_plain(loc, rk.kstart) if mutant == "plain_loads" else mem.load_sc(loc)
                            check(v, (e, j), f"rank {me} call {e} reduce({c}) inbox slot {j} unit {u}")
                        yield "step"
                    if design == "r5rs" and rs:
                        for u in units_res(cfg, c):   # round 5: straight into the caller's dst
                            wg.pending.append((("dst", me, u), e))
                    elif push_res and not rs:
                        for j in range(W):             # meshw: slot me of every rank's result inbox
                            for u in units_res(cfg, c):
                                wg.pending.append((("resin", j, me, u), e))
                    else:
                        for u in units_res(cfg, c):
                            wg.pending.append((("res", me, u), e))
                    yield "step"
                    yield from waitcnt(wg)
                    for j in range(W):
                        wg.pending.append((("ready", j, me, c), e))
                    yield "step"
                else:
                    c = s - 2 * lag
                    if not 0 <= c < nch:
                        continue
                    j = (me + pos - W) % W
                    wg.item = "gather"
                    if mutant != "rs_gather_no_wait" or not rs:
                        yield from wait_flag(rk, ("ready", me, j, c), e)
                    if rs and (design == "r5rs" or j != me):
                        continue                        # the wait alone
                    if rs:
                        src = [("res", me, u) for u in units_res(cfg, c)]
                        dst = [("dst", me, u) for u in range(c * cfg["L"] * cfg["es"], (c + 1) * cfg["L"] * cfg["es"])]
                    elif push_res:
                        src = [("resin", me, j, u) for u in units_res(cfg, c)]
                        dst = [("dst", me, u) for u in units_dst_ar(cfg, j, c)]
                    else:
                        src = [("res", j, u) for u in units_res(cfg, c)]
                        dst = [("dst", me, u) for u in units_dst_ar(cfg, j, c)]
                    for sl, dl in zip(src, dst):
                        v = mem.load_plain(sl, rk.kstart) if mutant == "plain_loads" else mem.load_sc(sl)
                        check(v, e, f"rank {me} call {e} gather({c}, {j}) {sl}")
                        wg.pending.append((dl, e))
                    yield "step"
            wg.done = True
        return gen

    def launch(rk):
        cfg = calls[rk.call]
        rk.call += 1
        rk.running = True
        rk.retired = 0
        rk.cfg = cfg
        rk.epoch = rk.epoch_done + 1
        rk.kstart = mem.t
        body = wg_body(rk, cfg, rk.epoch)
        rk.wgs = [_Wg(rk, body) for _ in range(G)]

    def host_check(rk):
        cfg, e, me = rk.cfg, rk.epoch, rk.me
        if cfg["mode"] == "rs":
            units = range(cfg["nchunks"] * cfg["L"] * cfg["es"])
        else:
            units = range(W * cfg["nchunks"] * cfg["L"] * cfg["es"])
        for u in units:
            check(mem.load_sc(("dst", me, u)), e, f"host: rank {me} call {e} dst unit {u}")

    for rk in ranks:
        launch(rk)
    steps = 0
    while True:
        steps += 1
        assert steps < 2_000_000
        acts = []
        for rk in ranks:
            for wg in rk.wgs:
                if wg.pending:
                    acts.append(("land", wg))
                if not wg.done:
                    acts.append(("run", wg))
            if rk.running and all(wg.done for wg in rk.wgs) and not any(wg.pending for wg in rk.wgs):
                acts.append(("end", rk))
            if not rk.running and rk.call < len(calls):
                acts.append(("launch", rk))
        if not acts:
            break
        rng.shuffle(acts)
        progressed = False
        for kind, x in acts:
            if kind == "land":
                loc, v = x.pending.pop(rng.randrange(len(x.pending)))   # any posted store, any order
                mem.land(loc, v)
            elif kind == "run":
                if next(x.gen, "step") == "blocked":
                    continue
            elif kind == "end":   # the last workgroup retired and its rank's stores landed
                host_check(x)
                x.epoch_done = x.epoch
                x.ticket = 0
                x.running = False
            else:
                launch(x)
            progressed = True
            break
        if not progressed:
            raise AssertionError(f"deadlock W={W} G={G} seed={seed} design={design}")
    for rk in ranks:
        assert rk.epoch_done == len(calls)


def _calls(rng, n, modes=("ar", "rs")):
    out = []
    for _ in range(n):
        nch = rng.randint(1, 3)
        out.append({"mode": rng.choice(modes), "es": rng.choice([1, 2]), "L": rng.choice([1, 2]),
                    "nchunks": nch, "lag": rng.randint(1, nch), "push_res": rng.random() < 0.5})
    return out


@pytest.mark.parametrize("design", ["r6", "r5rs"])
@pytest.mark.parametrize("W", [2, 3, 4])
def test_weak_model_holds(W, design):
    """Both designs, random mode / width / chunk / engine switches between calls,
    random interleavings and store landing orders: no stale read, no deadlock,
    every host check exact."""
    rng = random.Random(7919 * W + len(design))
    for _ in range(25):
        _run(W, rng.choice([1, 2, 3]), _calls(rng, 4), rng.randrange(1 << 30), design=design)


@pytest.mark.parametrize("mutant", ["no_wait_push", "no_wait_reduce", "plain_loads", "rs_gather_no_wait"])
def test_weak_model_mutants_fail(mutant):
    """Each ordering the kernel relies on, removed, must produce a stale read
    (or a wrong host result) in some interleaving: the model is not vacuous."""
    rng = random.Random(hash(mutant) & 0xFFFF)
    modes = ("rs",) if mutant == "rs_gather_no_wait" else ("ar", "rs")
    for _ in range(400):
        try:
            _run(rng.choice([2, 3]), rng.choice([1, 2]), _calls(rng, 3, modes), rng.randrange(1 << 30),
                 mutant=mutant)
        except _Violation:
            return
    pytest.fail(f"mutant {mutant} survived 400 runs")
