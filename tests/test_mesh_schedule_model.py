"""CPU model of the mesh engine's persistent-kernel schedule
(container_inc_amd/csrc/inccl_mesh.hip k_mesh, :407-447; do_push :147-226,
do_reduce :231-313, do_gather :318-359).

Each rank runs G workgroups that draw tickets from one counter; ticket t is
slot s = t / (2W + 1), position pos = t % (2W + 1): pos < W push(s, (me + 1 +
pos) % W), pos == W reduce(s - lag), else gather(s - 2 lag, (me + pos - W) % W)
-- the kernel's decomposition.  A push writes the rank's partial of chunk c
into rank j's inbox slot and then raises j's arrival flag; a reduce waits for
every rank's arrival flag of its chunk, reads the W inbox slots, writes its
result (own_res) and raises its ready flag at every rank; a gather waits for
rank j's ready flag and reads rank j's result chunk (reduce-scatter: only its
own, j == me; the other gathers only wait).  Flags hold the call's epoch; a wait is `flag >= epoch`.  The
last workgroup to retire resets the ticket counter and publishes the epoch;
a rank's next call starts only after every workgroup of its previous call
retired (stream order).

The model interleaves the workgroups of every rank at random (sequentially
consistent memory: it checks the schedule's logic; the memory model is
tests/test_mesh_weak_memory_model.py's) and
asserts, over many seeds, shapes and both modes:
  * no deadlock, with every rank's workgroups co-resident (the kernel's launch
    assumption, mesh.c grid sizing);
  * a reduce reads only partials of its own call (an inbox slot is never
    overwritten by the next call before it is read);
  * a gather reads only results of its own call (own_res is never overwritten
    by the next call's reduce before every peer pulled it);
  * every chunk of every rank is reduced exactly once per call.
"""
import random

import pytest


class _Rank:
    def __init__(self, me, W, G):
        self.me = me
        self.epoch_done = 0       # ctr[0]
        self.ticket = 0           # ctr[2]
        self.retired = 0          # ctr[1]
        self.call = 0             # calls launched
        self.wgs = [None] * G     # per workgroup: None (idle/retired) or a pending task
        self.running = False
        self.arrive = {}          # (j, c) -> epoch      (own sig, arrive_idx)
        self.ready = {}           # (j, c) -> epoch      (own sig, ready_idx)
        self.inbox = {}           # (j, c) -> epoch of the partial rank j pushed
        self.res = {}             # c -> epoch of own result chunk
        self.reduced = {}         # (epoch, c) -> count


def _run(W, G, nchunks, lag, calls, rs, seed):
    rng = random.Random(seed)
    ranks = [_Rank(r, W, G) for r in range(W)]
    per_slot = 2 * W + 1
    total = (nchunks + 2 * lag) * per_slot

    def launch(rk):
        rk.call += 1
        rk.running = True
        rk.retired = 0
        rk.epoch = rk.epoch_done + 1
        rk.wgs = ["fetch"] * G

    def step(rk, w):
        """One step of workgroup w of rank rk; False if it is blocked."""
        task = rk.wgs[w]
        e = rk.epoch
        if task == "fetch":
            t = rk.ticket
            rk.ticket += 1
            if t >= total:
                rk.wgs[w] = None
                rk.retired += 1
                if rk.retired == G:   # the last one resets and publishes (:439-446)
                    rk.ticket = 0
                    rk.epoch_done = e
                    rk.running = False
                return True
            s, pos = divmod(t, per_slot)
            if pos < W:
                rk.wgs[w] = ("push", s, (rk.me + 1 + pos) % W) if s < nchunks else "fetch"
            elif pos == W:
                c = s - lag
                rk.wgs[w] = ("reduce", c) if 0 <= c < nchunks else "fetch"
            else:
                c = s - 2 * lag
                rk.wgs[w] = ("gather", c, (rk.me + pos - W) % W) if 0 <= c < nchunks else "fetch"
            return True
        kind = task[0]
        if kind == "push":
            _, c, j = task
            peer = ranks[j]
            # data first, then the arrival flag (s_waitcnt(0) + barrier, :223-225)
            peer.inbox[(rk.me, c)] = e
            peer.arrive[(rk.me, c)] = e
            rk.wgs[w] = "fetch"
            return True
        if kind == "reduce":
            _, c = task
            if any(rk.arrive.get((j, c), 0) < e for j in range(W)):
                return False
            for j in range(W):
                got = rk.inbox.get((j, c))
                assert got == e, f"rank {rk.me} call {e} reduce chunk {c}: inbox slot {j} holds call {got}"
            rk.res[c] = e   # own_res in every mode (round 6; round 5's reduce-scatter wrote dst)
            rk.reduced[(e, c)] = rk.reduced.get((e, c), 0) + 1
            for j in range(W):
                ranks[j].ready[(rk.me, c)] = e
            rk.wgs[w] = "fetch"
            return True
        if kind == "gather":
            _, c, j = task
            if rk.ready.get((j, c), 0) < e:
                return False
            if not rs or j == rk.me:   # reduce-scatter: gather(c, me) copies my own result chunk into dst
                got = ranks[j].res.get(c)
                assert got == e, f"rank {rk.me} call {e} gather chunk {c} of rank {j}: result of call {got}"
            rk.wgs[w] = "fetch"
            return True
        raise AssertionError(task)

    for rk in ranks:
        launch(rk)
    while True:
        runnable = []
        for rk in ranks:
            if not rk.running:
                if rk.call < calls:
                    runnable.append((rk, None))
                continue
            for w in range(G):
                if rk.wgs[w] is not None:
                    runnable.append((rk, w))
        if not runnable:
            break
        rng.shuffle(runnable)
        progressed = False
        for rk, w in runnable:
            if w is None:
                launch(rk)
                progressed = True
                break
            if step(rk, w):
                progressed = True
                break
        assert progressed, (f"deadlock: W={W} G={G} nchunks={nchunks} lag={lag} rs={rs} seed={seed}: "
                            f"{[(rk.me, rk.call, rk.wgs) for rk in ranks]}")
    for rk in ranks:
        assert rk.epoch_done == calls
        for e in range(1, calls + 1):
            for c in range(nchunks):
                assert rk.reduced.get((e, c)) == 1, (rk.me, e, c)


@pytest.mark.parametrize("rs", [False, True], ids=["allreduce", "reduce_scatter"])
@pytest.mark.parametrize("W", [2, 3, 4, 8])
def test_mesh_schedule_model(W, rs):
    rng = random.Random(1000 * W + rs)
    for case in range(40):
        G = rng.choice([1, 2, 3, 5])
        nchunks = rng.randint(1, 6)
        lag = rng.randint(1, nchunks)
        _run(W, G, nchunks, lag, calls=3, rs=rs, seed=rng.randrange(1 << 30))


def test_mesh_schedule_model_defaults():
    """The default lag (the whole shard: every push before the first reduce,
    mesh.c mesh_piece) with one and with several workgroups per rank."""
    for W in (2, 4, 8):
        for G in (1, 4):
            for rs in (False, True):
                _run(W, G, nchunks=8, lag=8, calls=4, rs=rs, seed=W * 31 + G)
