#!/usr/bin/env python3
"""Run ``models/train.py`` with the attention backward of another ``_fused`` build (the loss-lineage
check of a kernel change: every other kernel is this tree's).

    python bench/with_attn_bwd.py --so scratch/r04/_fused.cpython-310-x86_64-linux-gnu.so -- \\
        --model llama3-8b --batch 4 --seq 4096 --steps 5 --warmup 2

If the losses match the old tree's bit for bit with the old backward swapped in, a lineage change of
the current tree comes from the backward kernel's rounding alone.
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))  # bench/ (the repo root's bench.py shadows the dir)
from attn_step_ab import Switch, load_other  # noqa: E402
from gpu_topology_on_k8s_amd.models import train  # noqa: E402
from gpu_topology_on_k8s_amd.ops import fused  # noqa: E402


def main():
    argv = sys.argv[1:]
    if "--so" not in argv or "--" not in argv:
        raise SystemExit(__doc__)
    so = argv[argv.index("--so") + 1]
    rest = argv[argv.index("--") + 1:]
    sw = Switch(fused.hip(), load_other(so))
    sw.use_other = True
    fused.hip = lambda: sw
    return train.main(rest)


if __name__ == "__main__":
    sys.exit(main())
