"""Multi-process engine check at a chosen world size on ONE GPU (all ranks on
device 0), reusing the GPU test's rank body: every case of
tests/test_gpu_p2p.py bit-exact against the oracle, repeated, back to back and
(ll / mesh) hipGraph-replayed.  A rehearsal of the W = 8 code paths the 8-GPU
bench exercises; not part of the suite (8 processes on one card).

    python tools/mp_engines.py WORLD ENGINE [ENGINE ...]
"""
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


def main():
    import test_gpu_p2p as T
    world = int(sys.argv[1])
    engines = sys.argv[2:] or ["p2p", "ll", "mesh"]
    bad = 0
    for engine in engines:
        cases = {"p2p": T.P2P_CASES, "ll": T.LL_CASES, "mesh": T.MESH_CASES, "meshw": T.MESH_CASES}[engine]
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        port = T._free_port()
        t0 = time.time()
        ps = [ctx.Process(target=T._rank_main, args=(r, world, port, cases, q, engine)) for r in range(world)]
        for p in ps:
            p.start()
        res = {}
        try:
            for _ in range(world):
                r, ok, err = q.get(timeout=300)
                res[r] = (ok, err)
        finally:
            for p in ps:
                p.join(timeout=60)
                if p.is_alive():
                    p.kill()
        good = all(err is None and all(ok) for ok, err in res.values()) and len(res) == world
        bad += 0 if good else 1
        print(f"world={world} engine={engine}: {'ok' if good else 'FAIL'} ({time.time() - t0:.1f} s)", flush=True)
        if not good:
            for r in sorted(res):
                ok, err = res[r]
                print(f"  rank {r}: err={err} ok={ok}", flush=True)
    sys.exit(1 if bad else 0)


if __name__ == "__main__":
    main()
