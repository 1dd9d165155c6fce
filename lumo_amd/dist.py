"""Multi-GPU tile sharding.

lumo renders independent (batch, tile) RenderTasks (renderer.rs:179-204) and merges each finished
FilmTile into the Film (film.rs:155-171).  Across GPUs the same split holds: every rank owns the
tiles with tile_index % world_size == rank for every batch (so a rank's batches of one tile stay
on one GPU), renders them with no communication, and the partial films are summed once at the
end.  The sum is the only collective and it is off the hot path.

For skewed scenes `TileQueue` hands tiles out dynamically instead (lumo's shared task receiver,
pool.rs:26); the measured `tile % 8` shares of the benchmark scenes are balanced to 1.02 max/mean
(DESIGN.md §6), so the static split stays the default.
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


def tasks_of_tiles(tasks, width, height, tiles):
    """The tasks (every batch, publish order) of the given tile indices."""
    tpb = tiles_per_batch(width, height)
    keep = set(int(t) for t in tiles)
    return [t for i, t in enumerate(tasks) if (i % tpb) in keep]


_GENERATION_KEY = "lumo_amd/tile_queue/generation"


class TileQueue:
    """Dynamic, skew-tolerant tile distribution across ranks.

    lumo's workers pop RenderTasks from one shared `Mutex<Receiver>` (pool.rs:26, 41-54; published
    by renderer.rs:179-204), so a slow tile never holds up the others.  Across GPUs the shared
    receiver is a counter in the process group's key-value store: `claim()` takes the next chunk
    of `chunk` tiles with one atomic `add` (no collective, nothing on the data path) and returns
    its tile indices, or [] once every tile has been handed out.  Every tile goes to exactly one
    rank; since each task carries its own seed (renderer.rs:196-203) the film does not depend on
    which rank renders which tile.

    The ranks' queues of one render share a store key, agreed on collectively: rank 0 draws a
    fresh generation number from the store and broadcasts it (one small collective per render,
    off the data path), so a rank that built more or fewer queues before (a preview render, a
    retry) cannot pair up with another render's queue.  When the iteration over a queue ends,
    every rank adds the tiles it took to a per-key total and, once every rank has reported (a
    count in the store, polled), checks that the total is the frame's tile count (`verify`), so a
    lost or doubled tile raises instead of silently changing the reduced film.  `key=` skips both and needs no process group (a bare
    store, single-process use); without `key=` the queue needs an initialised torch.distributed
    process group even when `store=` is given.  The coverage check waits on the store with a
    deadline rather than in a barrier, so a rank that failed mid-render turns into an error on the
    others instead of a hang.  The deadline (`timeout` seconds after this rank's last chunk)
    defaults to the store's own timeout, the process group's (30 min unless configured), because a
    healthy rank may still be rendering its last chunk long after a fast one finished.

    `chunk` defaults to half of one rank's static share: every claim is one more render call with
    fewer paths in flight and its own pipeline fill and drain (C1 1024² @ 64 spp, two ranks on one
    GPU: static 221 ms per frame; chunks of 1/2, 1/4, 1/8 share 266, 348, 435 ms; profiles/r03/dist),
    so claims stay few and large."""

    def __init__(self, width, height, world_size, chunk=None, store=None, key=None, group=None,
                 timeout=None):
        self.collective = key is None
        if store is None:
            import torch.distributed as dist
            store = dist.distributed_c10d._get_default_store()
        if timeout is None:  # the store's timeout (the process group's), else c10d's default 30 min
            t = getattr(store, "timeout", None)
            timeout = t.total_seconds() if hasattr(t, "total_seconds") else 1800.0
        self.timeout = float(timeout)
        self.n_tiles = tiles_per_batch(width, height)
        if chunk is None:
            chunk = max(1, self.n_tiles // (2 * max(1, world_size)))
        if chunk < 1:
            raise ValueError(f"chunk {chunk} < 1")
        self.chunk = int(chunk)
        self.store = store
        self.group = group
        self.claimed = 0
        if key is None:
            import torch.distributed as dist
            gen = [int(store.add(_GENERATION_KEY, 1)) if dist.get_rank(group) == 0 else 0]
            src = dist.get_global_rank(group, 0) if group is not None else 0
            dist.broadcast_object_list(gen, src=src, group=group)
            key = f"lumo_amd/tile_queue/{gen[0]}"
        self.key = key

    def claim(self):
        # store.add returns the counter after the increment: this claim owns [end - chunk, end)
        end = int(self.store.add(self.key, self.chunk))
        lo = end - self.chunk
        if lo >= self.n_tiles:
            return []
        return list(range(lo, min(end, self.n_tiles)))

    def verify(self):
        """Collective, after this rank's last chunk: the chunks the ranks iterated over cover the
        frame (claims are disjoint by construction; this catches tiles claimed but not taken
        through the iteration, or a rank on another frame size)."""
        import time
        import torch.distributed as dist
        self.store.add(self.key + "/done", self.claimed)
        self.store.add(self.key + "/ranks", 1)
        ws = dist.get_world_size(self.group)
        deadline = time.monotonic() + self.timeout
        while int(self.store.add(self.key + "/ranks", 0)) < ws:
            if time.monotonic() > deadline:
                arrived = int(self.store.add(self.key + "/ranks", 0))
                raise RuntimeError(f"tile queue {self.key}: only {arrived} of {ws} ranks finished their "
                                   f"tiles within {self.timeout:.0f} s (a rank failed mid-render?)")
            time.sleep(0.005)
        total = int(self.store.add(self.key + "/done", 0))
        if total != self.n_tiles:
            raise RuntimeError(f"tile queue {self.key}: {total} tiles handed out, the frame has {self.n_tiles}")

    def __iter__(self):
        while True:
            tiles = self.claim()
            if not tiles:
                break
            self.claimed += len(tiles)
            yield tiles
        if self.collective:
            self.verify()


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
