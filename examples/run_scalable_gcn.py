#!/usr/bin/env python3
"""Train / evaluate / infer scalable_gcn (reference examples/*/run_*.py).  Flags: see euler_amd.tools.runner.

    python examples/run_scalable_gcn.py --run_mode train --num_epochs 10
    torchrun --nproc-per-node 8 --master-addr 127.0.0.1 examples/run_scalable_gcn.py   # data parallel over RCCL
"""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from euler_amd.tools.runner import main  # noqa: E402

if __name__ == "__main__":
    main(model="scalable_gcn")
