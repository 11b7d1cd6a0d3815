"""Step-time cost of the dropout draw (timing only, never a bench line): run bench.py's main with
pcs_dropout_bits_bounded skipped after the first step's two calls, so every later step reuses the
first step's keep bits, and compare with a normal run on the same box.

    python tools/draw_cost.py --steps 10 --warmup 3 --no-cpu-baseline"""
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import pcs_amd._lib as L  # noqa: E402

_call = L.call
_seen = [0]


def call(name, *args):
    if name == "pcs_dropout_bits_bounded":
        _seen[0] += 1
        if _seen[0] > 2:
            return 0
    return _call(name, *args)


L.call = call
import bench  # noqa: E402

if __name__ == "__main__":
    bench.main()
