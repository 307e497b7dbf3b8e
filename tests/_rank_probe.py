"""Stand-in rank body for tests/test_bench.py::test_spawn_ranks_gloo: checks the env that
bench.spawn_ranks hands each rank and sums the ranks over gloo (CPU only)."""
import os
import sys

import torch
import torch.distributed as dist

rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
assert os.environ["LOCAL_RANK"] == str(rank) and os.environ["MASTER_ADDR"] == "127.0.0.1"
dist.init_process_group("gloo")
t = torch.tensor([float(rank + 1)], dtype=torch.float64)
dist.all_reduce(t)
if rank == 0:
    print("world=%d sum=%g" % (world, float(t.item())), flush=True)
dist.destroy_process_group()
sys.exit(int(os.environ.get("PROBE_EXIT_RANK", "-1")) == rank and 3 or 0)
