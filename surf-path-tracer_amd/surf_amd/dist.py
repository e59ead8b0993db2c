"""Multi-GPU image assembly: one collective per render call.

Rows are sharded in interleaved blocks (`ShardSpec`, same rule as
`surf_create_sharded`); every (pixel, frame) sample depends only on (p, f), so
ranks render independently and the only exchange is the gather of each rank's
float accumulator rows to the destination rank, followed by a host-side row
un-permute.  Backend-agnostic: `nccl` (RCCL over xGMI) with device tensors in
bench.py, `gloo` with CPU tensors in the multi-process CPU tests.
"""
from __future__ import annotations

import numpy as np

from . import ShardSpec, assemble_slabs, shard_rows


class RowGather:
    """Preallocated buffers for gathering (rows, W, 4) accumulators to `dst`."""

    def __init__(self, width: int, height: int, world: int, rank: int, row_block: int, device, dst: int = 0):
        import torch
        self.width, self.height, self.world, self.rank, self.dst = width, height, world, rank, dst
        self.row_block = row_block
        self.specs = [ShardSpec(r, world, row_block) for r in range(world)]
        self.rows = [len(shard_rows(height, s)) for s in self.specs]
        self.max_rows = max(self.rows)
        self.send = torch.zeros((self.max_rows, width, 4), dtype=torch.float32, device=device)
        self.recv = ([torch.empty_like(self.send) for _ in range(world)] if rank == dst else None)

    def gather(self, acc_rows) -> None:
        """acc_rows: this rank's (rows, W, 4) float32 tensor on the buffers' device."""
        import torch.distributed as dist
        n = self.rows[self.rank]
        if tuple(acc_rows.shape) != (n, self.width, 4):
            raise ValueError(f"rank {self.rank}: accumulator shape {tuple(acc_rows.shape)} != {(n, self.width, 4)}")
        self.send[:n].copy_(acc_rows)
        dist.gather(self.send, self.recv, dst=self.dst)

    def assemble(self) -> np.ndarray:
        """Full (H, W, 4) frame on the destination rank: the gathered slabs
        un-permuted by libsurf_mgpu's native code (surf_mgpu_assemble, the same
        un-permute a C++ application's surf_mgpu_gather runs)."""
        if self.recv is None:
            raise RuntimeError("assemble() is only valid on the destination rank")
        import torch
        slabs = torch.stack([r.cpu() for r in self.recv]).numpy()
        return assemble_slabs(self.width, self.height, self.world, self.row_block, slabs)
