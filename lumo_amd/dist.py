"""Multi-GPU tile sharding.

lumo renders independent (batch, tile) RenderTasks (renderer.rs:179-204) and merges each finished
FilmTile into the Film (film.rs:155-171).  Across GPUs the same split holds: every rank owns the
tiles with tile_index % world_size == rank for every batch (so a rank's batches of one tile stay
on one GPU), renders them with no communication, and the partial films are summed once at the
end.  The sum is the only collective and it is off the hot path.
"""
import numpy as np

from . import TILE_SIZE, Film


def tiles_per_batch(width, height):
    return ((width + TILE_SIZE - 1) // TILE_SIZE) * ((height + TILE_SIZE - 1) // TILE_SIZE)


def shard_tasks(tasks, width, height, rank, world_size):
    """This rank's tasks, in publish order."""
    if not 0 <= rank < world_size:
        raise ValueError(f"rank {rank} outside world of {world_size}")
    tpb = tiles_per_batch(width, height)
    return [t for i, t in enumerate(tasks) if (i % tpb) % world_size == rank]


def reduce_film(film, group=None, dst=None):
    """Sum partial films over the process group (all ranks, or only `dst` when given).

    Film::add_tile (film.rs:155-171) adds a tile's pixels and then its splats; across ranks the
    tiles are disjoint, so the pixel sum is exact, and the BDPT light-tracing splats
    (tile.rs:96-101, full-frame) are summed in one collective with them.  The film's colour
    space, splat scale (1 / samples, film.rs:137) and filter carry over."""
    import torch
    import torch.distributed as dist
    backend = dist.get_backend(group)
    dev = "cuda" if backend == "nccl" else "cpu"
    n_pix = film.pixels.size
    flat = np.concatenate([np.ascontiguousarray(film.pixels).ravel(), np.ascontiguousarray(film.splats).ravel()])
    t = torch.from_numpy(flat).to(dev)
    if dst is None:
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=group)
    else:
        dist.reduce(t, dst=dst, op=dist.ReduceOp.SUM, group=group)
    out = Film(film.width, film.height, film.color_space, filter_radius=film.filter_radius,
               filter_sigma=film.filter_sigma)
    out.splat_scale = film.splat_scale
    v = t.cpu().numpy()
    out.pixels[...] = v[:n_pix].reshape(out.pixels.shape)
    out.splats[...] = v[n_pix:].reshape(out.splats.shape)
    return out
