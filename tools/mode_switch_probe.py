"""One rank of tests/test_gpu_reduce_scatter.py's mode-switch sequence
(_mode_switch_rank) started from a shell (tools/gpu_mode_switch.sh) instead of
from a pytest process that holds a GPU context of its own: the same calls, the
same checks, one JSON line per rank.

    python tools/mode_switch_probe.py RANK PORT W LOG2"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tests"))
sys.path.insert(0, ROOT)


class _Print:
    def put(self, item):
        rank, ok, err = item
        print(json.dumps({"rank": rank, "ok": ok, "error": err}), flush=True)


def main():
    rank, port, world, lg = (int(v) for v in sys.argv[1:5])
    from test_gpu_reduce_scatter import _mode_switch_rank
    _mode_switch_rank(rank, world, port, _Print(), lg)


if __name__ == "__main__":
    main()
