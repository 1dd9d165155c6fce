"""Multi-rank tile sharding over torch.distributed (gloo, world_size 2): the sharded renders
summed with lumo_amd.dist.reduce_film equal the single-process render.  PathTrace and BDPT
(whose light-tracing splats are full-frame, tile.rs:96-101, and are summed across ranks) run
through the oracle on the CPU; the GPU test drives Renderer.render(rank, world_size) on cuda:0
from both ranks (the one-GPU box) and compares with the single-process render."""
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


def _scene(integrator):
    import lumo_amd as L
    from lumo_amd import scenes
    if integrator == 0:
        return L.Scene.cornell_box(), L.Camera.cornell_box((W, H))
    return scenes.caustics(), scenes.caustics_camera((W, H))


def _render(tasks, integrator=0):
    import lumo_amd as L
    import oracle_ffi as O
    sc, cam = _scene(integrator)
    splats = [] if integrator else None
    bufs, res, _ = O.render_tasks(sc.build().desc(), cam.desc, tasks, O.WAVEFRONT, 2, integrator=integrator,
                                  splats_out=splats)
    film = L.Film(W, H, samples=SPP)
    for i, (t, b) in enumerate(zip(tasks, bufs)):
        film.add_tile(t, b, splats[i] if splats is not None else None)
    return film, sum(r.num_rays for r in res)


def _worker(rank, ws, port, out_dir, integrator):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    import lumo_amd as L
    from lumo_amd.dist import reduce_film, shard_tasks
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
    tasks = L.make_tasks(W, H, SPP, SEED)
    mine = shard_tasks(tasks, W, H, rank, ws)
    film, rays = _render(mine, integrator)
    total = reduce_film(film)
    np.save(os.path.join(out_dir, f"film{rank}.npy"), total.pixels)
    np.save(os.path.join(out_dir, f"splats{rank}.npy"), total.splats)
    np.save(os.path.join(out_dir, f"meta{rank}.npy"), np.array([total.splat_scale, total.color_space,
                                                                   total.filter_radius, total.filter_sigma]))
    np.save(os.path.join(out_dir, f"rays{rank}.npy"), np.array([rays, len(mine)]))
    dist.barrier()
    dist.destroy_process_group()


def _spawn(fn, ws, *args):
    import torch.multiprocessing as mp
    mp.start_processes(fn, args=(ws, _free_port()) + args, nprocs=ws, join=True, start_method="spawn")


@pytest.mark.parametrize("integrator", [0, 1], ids=["pathtrace", "bdpt"])
def test_sharded_render_equals_single(integrator, tmp_path):
    import lumo_amd as L
    ws = 2
    _spawn(_worker, ws, str(tmp_path), integrator)
    tasks = L.make_tasks(W, H, SPP, SEED)
    film, rays = _render(list(tasks), integrator)
    parts = [np.load(tmp_path / f"rays{r}.npy") for r in range(ws)]
    assert sum(int(p[1]) for p in parts) == len(tasks)
    assert sum(int(p[0]) for p in parts) == rays
    if integrator:
        assert film.splats.any()  # the caustics scene has light-tracing splats
    for r in range(ws):
        got = np.load(tmp_path / f"film{r}.npy")
        # tiles are disjoint per rank and a pixel's non-splat samples only come from its own
        # tile, so the pixel sum is exact
        np.testing.assert_array_equal(got, film.pixels)
        # splats are full-frame: summed per rank, then across ranks (a different float order)
        np.testing.assert_allclose(np.load(tmp_path / f"splats{r}.npy"), film.splats, rtol=0, atol=1e-12)
        meta = np.load(tmp_path / f"meta{r}.npy")
        np.testing.assert_array_equal(meta, [film.splat_scale, film.color_space, film.filter_radius,
                                             film.filter_sigma])


def _gpu_worker(rank, ws, port, out_dir, integrator):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    import lumo_amd as L
    from lumo_amd.dist import reduce_film
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
    sc, cam = _scene(integrator)
    r = L.Renderer(sc, cam).samples(SPP).seed(SEED).integrator(
        L.Integrator.BDPathTrace if integrator else L.Integrator.PathTrace)
    total = reduce_film(r.render(rank, ws))
    np.save(os.path.join(out_dir, f"film{rank}.npy"), total.pixels)
    np.save(os.path.join(out_dir, f"splats{rank}.npy"), total.splats)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", [0, 1], ids=["pathtrace", "bdpt"])
def test_gpu_renderer_sharded_equals_single(integrator, tmp_path):
    """Renderer.render(rank, 2) on both ranks + reduce_film == Renderer.render() in one process."""
    import lumo_amd as L
    _spawn(_gpu_worker, 2, str(tmp_path), integrator)
    sc, cam = _scene(integrator)
    single = L.Renderer(sc, cam).samples(SPP).seed(SEED).integrator(
        L.Integrator.BDPathTrace if integrator else L.Integrator.PathTrace).render()
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"film{r}.npy"), single.pixels)
        np.testing.assert_allclose(np.load(tmp_path / f"splats{r}.npy"), single.splats, rtol=0, atol=1e-12)


def test_tile_queue_hands_out_every_tile_once():
    """TileQueue over one store: interleaved claims from two queues (two ranks) cover every tile
    exactly once, in chunks, and a later queue (the next render) starts from tile 0 again."""
    import torch.distributed as dist
    from lumo_amd.dist import TileQueue, tiles_per_batch
    store = dist.HashStore()
    n = tiles_per_batch(W, H)
    qs = [TileQueue(W, H, 2, chunk=2, store=store, key="render1") for _ in range(2)]  # one render's two ranks
    got = []
    while True:
        a, b = qs[0].claim(), qs[1].claim()
        got += a + b
        if not a and not b:
            break
        assert len(a) <= 2 and len(b) <= 2
    assert sorted(got) == list(range(n))
    nxt = TileQueue(W, H, 2, chunk=5, store=store, key="render2")
    assert nxt.claim() == list(range(5))
    assert TileQueue(W, H, 2, store=store, key="render3").chunk == max(1, n // 4)
    with pytest.raises(ValueError):
        TileQueue(W, H, 2, chunk=0, store=store, key="render4")


def _dyn_worker(rank, ws, port, out_dir, integrator):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    import lumo_amd as L
    from lumo_amd.dist import TileQueue, reduce_film, tasks_of_tiles
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
    if rank == 1:  # a rank-local queue first (a preview render): must not shift the shared render's key
        store = dist.distributed_c10d._get_default_store()
        TileQueue(W, H, 1, chunk=4, store=store, key="lumo_amd/preview").claim()
    tasks = L.make_tasks(W, H, SPP, SEED)
    film = L.Film(W, H, samples=SPP)
    rays = n_tasks = 0
    for tiles in TileQueue(W, H, ws, chunk=1):
        mine = tasks_of_tiles(tasks, W, H, tiles)
        part, r = _render(mine, integrator)
        film.pixels += part.pixels
        film.splats += part.splats
        rays += r
        n_tasks += len(mine)
    total = reduce_film(film)
    np.save(os.path.join(out_dir, f"film{rank}.npy"), total.pixels)
    np.save(os.path.join(out_dir, f"splats{rank}.npy"), total.splats)
    np.save(os.path.join(out_dir, f"rays{rank}.npy"), np.array([rays, n_tasks]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("integrator", [0, 1], ids=["pathtrace", "bdpt"])
def test_dynamic_queue_render_equals_single(integrator, tmp_path):
    """Tiles claimed one at a time from the shared TileQueue by two gloo ranks, rendered through
    the oracle and summed with reduce_film: the single-process film (pixels exact)."""
    import lumo_amd as L
    ws = 2
    _spawn(_dyn_worker, ws, str(tmp_path), integrator)
    tasks = L.make_tasks(W, H, SPP, SEED)
    film, rays = _render(list(tasks), integrator)
    parts = [np.load(tmp_path / f"rays{r}.npy") for r in range(ws)]
    assert sum(int(p[1]) for p in parts) == len(tasks)
    assert sum(int(p[0]) for p in parts) == rays
    for r in range(ws):
        np.testing.assert_array_equal(np.load(tmp_path / f"film{r}.npy"), film.pixels)
        np.testing.assert_allclose(np.load(tmp_path / f"splats{r}.npy"), film.splats, rtol=0, atol=1e-12)


def _gpu_dyn_worker(rank, ws, port, out_dir, integrator):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    import lumo_amd as L
    from lumo_amd.dist import reduce_film
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
    sc, cam = _scene(integrator)
    r = L.Renderer(sc, cam).samples(SPP).seed(SEED).integrator(
        L.Integrator.BDPathTrace if integrator else L.Integrator.PathTrace)
    total = reduce_film(r.render(rank, ws, schedule="dynamic", chunk=3))
    np.save(os.path.join(out_dir, f"film{rank}.npy"), total.pixels)
    np.save(os.path.join(out_dir, f"splats{rank}.npy"), total.splats)
    np.save(os.path.join(out_dir, f"tasks{rank}.npy"), np.array([r.tasks_rendered]))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("integrator", [0, 1], ids=["pathtrace", "bdpt"])
def test_gpu_renderer_dynamic_equals_single(integrator, tmp_path):
    """Renderer.render(rank, 2, schedule="dynamic") on both ranks + reduce_film ==
    Renderer.render() in one process."""
    import lumo_amd as L
    _spawn(_gpu_dyn_worker, 2, str(tmp_path), integrator)
    sc, cam = _scene(integrator)
    single = L.Renderer(sc, cam).samples(SPP).seed(SEED).integrator(
        L.Integrator.BDPathTrace if integrator else L.Integrator.PathTrace).render()
    assert sum(int(np.load(tmp_path / f"tasks{r}.npy")[0]) for r in range(2)) == len(L.make_tasks(W, H, SPP, SEED))
    for r in range(2):
        np.testing.assert_array_equal(np.load(tmp_path / f"film{r}.npy"), single.pixels)
        np.testing.assert_allclose(np.load(tmp_path / f"splats{r}.npy"), single.splats, rtol=0, atol=1e-12)


def test_render_rejects_unknown_schedule():
    import lumo_amd as L
    r = L.Renderer(L.Scene.cornell_box(), L.Camera.cornell_box((W, H))).samples(1).seed(1)
    with pytest.raises(ValueError):
        r.render(0, 2, schedule="round-robin")


def _verify_worker(rank, ws, port, out_dir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import torch.distributed as dist
    from lumo_amd.dist import TileQueue
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
    q = TileQueue(W, H, ws, chunk=2)
    ok = 0
    if rank == 0:
        q.claim()  # a chunk handed out but never taken through the iteration: its tiles are lost
    # the lost chunk must be claimed before either rank iterates, or rank 1 may drain the queue
    # first and rank 0's claim comes back empty (nothing lost, nothing to detect)
    dist.barrier()
    try:
        for _ in q:
            pass
    except RuntimeError:
        ok = 1
    np.save(os.path.join(out_dir, f"raised{rank}.npy"), np.array([ok]))
    dist.barrier()
    dist.destroy_process_group()


def test_tile_queue_detects_lost_tiles(tmp_path):
    """A chunk claimed by rank 0 but never rendered (not taken through the iteration): the ranks'
    per-key total of tiles taken falls short of the frame's, and both ranks raise instead of
    reducing a film with missing tiles."""
    _spawn(_verify_worker, 2, str(tmp_path))
    assert [int(np.load(tmp_path / f"raised{r}.npy")[0]) for r in range(2)] == [1, 1]


def _failed_rank_worker(rank, ws, port, out_dir):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]
    import time
    import torch.distributed as dist
    from lumo_amd.dist import TileQueue
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=ws)
    q = TileQueue(W, H, ws, chunk=2, timeout=2.0)
    msg = ""
    t0 = time.monotonic()
    if rank == 0:
        try:
            for _ in q:
                pass
        except RuntimeError as e:
            msg = str(e)
    # rank 1 "fails mid-render": it never iterates to the end of the queue, so never reaches verify
    np.save(os.path.join(out_dir, f"failed{rank}.npy"), np.array([len(msg) > 0, time.monotonic() - t0]))
    with open(os.path.join(out_dir, f"msg{rank}.txt"), "w") as f:
        f.write(msg)
    dist.barrier()
    dist.destroy_process_group()


def test_tile_queue_failed_rank_raises_not_hangs(tmp_path):
    """A rank that never finishes its tiles: the others' coverage check gives up at the queue's
    deadline with an error naming the missing ranks, instead of blocking in a barrier."""
    _spawn(_failed_rank_worker, 2, str(tmp_path))
    r0 = np.load(tmp_path / "failed0.npy")
    assert bool(r0[0]) and r0[1] < 30
    assert "1 of 2 ranks" in (tmp_path / "msg0.txt").read_text()


def test_tile_queue_default_deadline_is_the_store_timeout():
    """The coverage check's deadline defaults to the store's own timeout (the process group's), not
    a fixed 300 s that a healthy slow rank could exceed (advisor, round 5)."""
    from datetime import timedelta

    import torch.distributed as dist
    from lumo_amd.dist import TileQueue
    s = dist.HashStore()
    s.set_timeout(timedelta(seconds=1234))
    q = TileQueue(64, 64, 2, store=s, key="lumo_amd/test/deadline")
    assert q.timeout == 1234.0
    assert TileQueue(64, 64, 2, store=s, key="lumo_amd/test/deadline2", timeout=7).timeout == 7.0
