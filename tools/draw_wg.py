"""bench.py with the side-stream dropout draw bounded at DRAW_WG workgroups per CU instead of the
engine's 2 (timing only, never a bench line): pcs_dropout_bits_bounded's max_workgroups is
rewritten before the call.

    DRAW_WG=3 python tools/draw_wg.py --steps 10 --warmup 3 --no-cpu-baseline"""
import os
import sys

import torch

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import pcs_amd._lib as L  # noqa: E402

_call = L.call
_per_cu = int(os.environ.get("DRAW_WG", "2"))


def call(name, *args):
    if name == "pcs_dropout_bits_bounded" and args[6] > 0:
        args = list(args)
        args[6] = _per_cu * torch.cuda.get_device_properties(0).multi_processor_count
    return _call(name, *args)


L.call = call
import bench  # noqa: E402

if __name__ == "__main__":
    bench.main()
