"""N > 1 decomposition on CPU: world_size-2 gloo process group, each rank
renders its interleaved row shard (with the C oracle standing in for the GPU
renderer, as the checker), and the framebuffer sum-reduce must give the
single-process frame. Exercises bdpt_dist.row_shard / reduce_framebuffer, the
functions bench.py uses over RCCL."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import bdpt_dist
import oracle as O
import variants

NAME, W, H, SPP, RR = "hardlight", 24, 20, 3, 2


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        rows = bdpt_dist.shard_rows(rank, world, H)
        sc = O.Scene(variants.obj_path(NAME))
        fb, n = sc.render(O.make_params(variants.SCENES[NAME]["camera"], W, H, SPP, RR), rows=rows)
        t = torch.from_numpy(fb.copy())
        cnt = torch.tensor([n], dtype=torch.int64)
        bdpt_dist.reduce_framebuffer(t, dst=0)
        dist.all_reduce(cnt)
        if rank == 0:
            np.save(out_path, t.numpy())
            np.save(out_path + ".n.npy", cnt.numpy())
    finally:
        dist.destroy_process_group()


def test_row_shards_partition_the_image():
    for world in (1, 2, 3, 8):
        rows = sorted(r for k in range(world) for r in bdpt_dist.shard_rows(k, world, 37))
        assert rows == list(range(37))
    with pytest.raises(ValueError):
        bdpt_dist.row_shard(2, 2)


def test_two_rank_gloo_reduce_equals_single_process(tmp_path):
    out = str(tmp_path / "fb.npy")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    fb = np.load(out)
    n = int(np.load(out + ".n.npy")[0])
    ref, nref = O.Scene(variants.obj_path(NAME)).render(O.make_params(variants.SCENES[NAME]["camera"], W, H, SPP, RR))
    assert n == nref == W * H * SPP
    a, r = fb.reshape(-1, 3).astype(np.float64), ref.reshape(-1, 3).astype(np.float64)
    err = np.linalg.norm(a - r, axis=1) / np.maximum(np.linalg.norm(r, axis=1), 1e-8)
    assert err.max() <= 1e-5  # only splat summation order differs
