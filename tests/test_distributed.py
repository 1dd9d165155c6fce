"""Multi-rank tile sharding over torch.distributed (gloo, world_size 2, CPU): the sharded
renders summed with lumo_amd.dist.reduce_film equal the single-process render exactly.  The
per-rank renderer here is the oracle (no GPU in this container); the GPU path uses the same
shard_tasks / reduce_film code (bench.py, Renderer.render)."""
import os
import socket
import sys

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
W = H = 48
SPP = 4
SEED = 77


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _render(tasks):
    import lumo_amd as L
    import oracle_ffi as O
    sc = L.Scene.cornell_box()
    cam = L.Camera.cornell_box((W, H))
    bufs, res, _ = O.render_tasks(sc.desc(), cam.desc, tasks, O.WAVEFRONT, 2)
    film = L.Film(W, H)
    for t, b in zip(tasks, bufs):
        film.add_tile(t, b)
    return film, sum(r.num_rays for r in res)


def _worker(rank, ws, port, out_dir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    import lumo_amd as L
    from lumo_amd.dist import reduce_film, shard_tasks
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
    tasks = L.make_tasks(W, H, SPP, SEED)
    mine = shard_tasks(tasks, W, H, rank, ws)
    film, rays = _render(mine)
    total = reduce_film(film)
    np.save(os.path.join(out_dir, f"film{rank}.npy"), total.pixels)
    np.save(os.path.join(out_dir, f"rays{rank}.npy"), np.array([rays, len(mine)]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("ws", [2])
def test_sharded_render_equals_single(ws, tmp_path):
    import torch.multiprocessing as mp
    import lumo_amd as L
    port = _free_port()
    mp.start_processes(_worker, args=(ws, port, str(tmp_path)), nprocs=ws, join=True, start_method="spawn")
    tasks = L.make_tasks(W, H, SPP, SEED)
    film, rays = _render(list(tasks))
    parts = [np.load(tmp_path / f"rays{r}.npy") for r in range(ws)]
    assert sum(int(p[1]) for p in parts) == len(tasks)
    assert sum(int(p[0]) for p in parts) == rays
    for r in range(ws):
        got = np.load(tmp_path / f"film{r}.npy")
        # tiles are disjoint per rank and a pixel's splats only come from its own tile, so the
        # sum is exact
        np.testing.assert_array_equal(got, film.pixels)
