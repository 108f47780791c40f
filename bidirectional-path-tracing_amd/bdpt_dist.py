"""Multi-GPU decomposition of the BDPT frame (one process per GPU).

The image is split into interleaved row shards: rank r renders rows
r, r + N, r + 2N, ... (every camera sample of those rows). Interleaving
balances cost across ranks, because the Cornell scenes' cost varies smoothly
with the image row. Light subpaths splat onto any pixel of the image
(connectToCamera, reference bdpt.h:295-371), so each rank accumulates into its
own full-frame buffer. The frame is then the element-wise sum of the rank
buffers: one sum-reduce (RCCL over xGMI with the "nccl" backend) to the
output rank. That reduce is the path's only exchange step.
"""
from __future__ import annotations


def row_shard(rank: int, world: int) -> tuple[int, int]:
    """(row_offset, row_stride) of `rank` for bdpt_frame_params."""
    if world < 1 or not (0 <= rank < world):
        raise ValueError(f"bad shard {rank}/{world}")
    return rank, world


def shard_rows(rank: int, world: int, height: int) -> list[int]:
    off, stride = row_shard(rank, world)
    return list(range(off, height, stride))


def reduce_framebuffer(fb, dst: int = 0) -> None:
    """Sums every rank's full-frame buffer into `fb` on rank `dst` (in place)."""
    import torch.distributed as dist

    if dist.is_available() and dist.is_initialized() and dist.get_world_size() > 1:
        if dist.get_backend() == "gloo" and fb.is_cuda:  # gloo reduces host tensors
            host = fb.cpu()
            dist.reduce(host, dst=dst, op=dist.ReduceOp.SUM)
            if dist.get_rank() == dst:
                fb.copy_(host)
        else:
            dist.reduce(fb, dst=dst, op=dist.ReduceOp.SUM)
