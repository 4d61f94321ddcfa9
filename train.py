#!/usr/bin/env python3
"""Drop-in for the reference's train.py:
    python train.py --config-file configs/default.yaml --output-dir runs
Multi-GPU (one process per GPU):
    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 \\
        train.py --config-file configs/default.yaml --output-dir runs
"""
import _rtpkg  # noqa: F401
from ppo_radiotherapy_amd.train import get_argparser, main, train  # noqa: F401

if __name__ == "__main__":
    main()
