"""Rank program for tests/test_scripts.py::test_stalled_rank_fails_within_timeout.

Both ranks join a gloo group through ``penroz.parallel.dist.init_group`` (explicit timeout from
``PENROZ_DIST_TIMEOUT``); rank 1 then stalls (never enters the collective) while rank 0 calls an
all-reduce, which must raise once the timeout expires instead of waiting forever.
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

from penroz.parallel.dist import init_group  # noqa: E402

init_group("gloo")
if dist.get_rank() == 1:
    time.sleep(120)
    sys.exit(0)
t0 = time.time()
try:
    dist.all_reduce(torch.ones(4))
except Exception as e:  # the timeout
    print(f"rank0 collective failed after {time.time() - t0:.1f}s: {type(e).__name__}", flush=True)
    sys.exit(3)
sys.exit(0)
