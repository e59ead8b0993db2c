"""Multi-rank path on CPU: world_size 2 and 3 over gloo.

Each rank renders its interleaved row blocks with the CPU oracle (as a GPU rank
renders them with the HIP path), gathers its accumulator rows to rank 0 through
`surf_amd.dist.RowGather` -- the same code bench.py runs over RCCL -- and rank 0
checks the assembled frame bit-for-bit against a single full-frame render.
"""
import os
import socket
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _rank_main(rank, world, port, width, height, row_block, frames):
    for p in (REPO, os.path.join(REPO, "surf-path-tracer_amd")):
        if p not in sys.path:
            sys.path.insert(0, p)
    import torch
    import torch.distributed as dist
    import oracle
    import surf_amd
    from surf_amd.dist import RowGather

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        scene = oracle.OracleScene()
        spec = surf_amd.ShardSpec(rank, world, row_block)
        rows = surf_amd.shard_rows(height, spec)
        # this rank's rows, rendered block by block (contiguous runs of `rows`)
        parts = []
        start = 0
        while start < len(rows):
            end = start
            while end + 1 < len(rows) and rows[end + 1] == rows[end] + 1:
                end += 1
            acc, _, _ = scene.render(width, height, frames, rows=(int(rows[start]), int(rows[end]) + 1), threads=1)
            parts.append(acc)
            start = end + 1
        mine = torch.from_numpy(np.concatenate(parts, axis=0)) if parts else torch.zeros((0, width, 4))
        g = RowGather(width, height, world, rank, row_block, torch.device("cpu"))
        g.gather(mine)
        if rank == 0:
            full = g.assemble()
            ref, _, _ = scene.render(width, height, frames, threads=1)
            assert np.array_equal(full.view(np.uint32), ref.view(np.uint32)), "assembled shards differ from the full render"
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,height,row_block", [(2, 48, 16), (3, 40, 16), (2, 37, 0)])
def test_row_shards_gather_assemble_gloo(world, height, row_block):
    import torch.multiprocessing as mp
    mp.spawn(_rank_main, args=(world, _free_port(), 24, height, row_block, 2), nprocs=world, join=True)
