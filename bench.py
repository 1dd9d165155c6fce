#!/usr/bin/env python3
"""Benchmark: lumo's Cornell box, PathTrace, 1024x1024 @ 1024 spp (BASELINE.json configs[1]).

One "step" = the full C1 render: every (256-spp batch, 16x16 tile) RenderTask of the frame
(renderer.rs:179-204), 4 batches x 4096 tiles = 1.07e9 camera paths.  With N ranks (one per GPU,
launched by torch.distributed.run) the tasks are sharded by tile index (tile % N == rank), the
scene is replicated, and no collective touches the data path; only the timing barrier and the
final max/sum reductions use the process group.

Prints ONE JSON line (rank 0).  `value` is whole-job Mrays/s = (closest-hit + shadow-visibility
queries of all ranks) / max-over-ranks wall time of the K timed steps.  Also reported:
Msamples/s (camera paths), lumo's own "total rays" rate (sum of path depths, task.rs:65), the
roofline of the dominant kernel (algorithmic bytes from the kernels' own traversal counters over
live HIP-event kernel time), and the CPU baseline (the f64 oracle in lumo's tile-serial order on
this host's cores, on a bounded sample of the same frame).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E peak (MI355X_MICROARCH.md, chip-level parameters)
SEED = 0x5EED_1234
# Algorithmic bytes per unit: f64 data touched by the algorithm.
B_AABB, B_KD, B_TRI = 48, 16, 84           # slab test bounds; kd split node; 3 vertices + indices
B_CLOSEST_IO = 48 + 20  # ray in + hit out
B_RECORD, B_FOLD = 104, 104  # shadow record in; per path: gathered + pdf_light + radiance read/write
STAGES = ["camera", "closest", "shade", "shadow", "resolve", "finish", "film", "ring"]


def dist_env():
    ws = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", str(rank)))
    return ws, rank, local


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="c1", choices=["c1", "c2", "c3", "c4"],
                    help="c1 Cornell 1024^2@1024 (BASELINE configs[1]); c2 dragon.rs 1920x1080@256 with the "
                         "871k-triangle stand-in (configs[2]); c3 Bistro stand-in 1920x1080@256 (configs[3]); "
                         "c4 caustics.rs BDPT 1024^2@4096 (configs[4])")
    ap.add_argument("--res", type=int, default=None, help="square resolution override")
    ap.add_argument("--spp", type=int, default=None)
    ap.add_argument("--max-paths", type=int, default=1 << 23, help="paths in flight per wavefront")
    ap.add_argument("--max-vertices", type=int, default=0, help="BDPT vertex storage per subpath (0 = 128)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle on the host (rank 0, N=1)")
    ap.add_argument("--cpu-tile-stride", type=int, default=32, help="CPU sample: every k-th tile of each batch")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    import lumo_amd as L
    from lumo_amd import _ffi

    pg = None
    if ws > 1:
        import torch
        import torch.distributed as dist
        backend = "nccl" if torch.cuda.is_available() else "gloo"
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
        pg = dist

    scene, cam, (W, H), spp, wl = build_config(args)
    tasks = L.make_tasks(W, H, spp, SEED)
    from lumo_amd.dist import shard_tasks, tiles_per_batch
    tiles = tiles_per_batch(W, H)
    mine = shard_tasks(tasks, W, H, rank, ws)
    mine_arr = (_ffi.TileTask * len(mine))(*mine)

    splat_film = np.zeros((H, W, 3)) if wl.get("integrator") == L.Integrator.BDPathTrace else None
    dev = L.Device(local)
    dev.upload(scene, cam)
    lib = _ffi.load()

    def step():
        if wl.get("integrator") == L.Integrator.BDPathTrace:
            splat_film[:] = 0.0
            bufs, res = dev.render_tasks(mine_arr, max_paths=args.max_paths, integrator=L.Integrator.BDPathTrace,
                                         splat_film=splat_film, max_vertices=args.max_vertices)
        else:
            bufs, res = dev.render_tasks(mine_arr, max_paths=args.max_paths)
        return sum(r.num_queries for r in res), sum(r.num_camera_rays for r in res), sum(r.num_rays for r in res)

    def barrier():
        if pg is not None:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            pg.barrier()

    for _ in range(args.warmup):
        step()
    lib.lumo_set_timing(1)
    lib.lumo_stats_reset(dev.ctx)
    barrier()
    t0 = time.perf_counter()
    q = cams = rays = 0
    for _ in range(args.steps):
        a, b, c = step()
        q, cams, rays = q + a, cams + b, rays + c
    barrier()  # lumo_render_tiles returns only after its stream has drained
    elapsed = time.perf_counter() - t0
    lib.lumo_set_timing(0)
    st = dev.stats()

    if pg is not None:
        import torch
        dev_t = "cuda" if torch.cuda.is_available() else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev_t)
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([q, cams, rays], dtype=torch.float64, device=dev_t)
        pg.all_reduce(s, op=pg.ReduceOp.SUM)
        q, cams, rays = (float(x) for x in s.tolist())

    if rank == 0:
        roof = roofline(st, n_shadow_rays(scene), bdpt=wl.get("integrator") == L.Integrator.BDPathTrace,
                        workload=args.config)
        cpu = cpu_baseline(scene, cam, tasks, tiles, args, W, H, spp, wl) if (args.cpu_baseline and ws == 1) else None
        value = q / elapsed / 1e6
        out = {
            "metric": "Mrays/s",
            "value": round(value, 3),
            "unit": "Mrays/s",
            "n_gpus": ws,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": wl["data"],
            "config": {
                "workload": f"{wl['name']}_{W}x{H}_{spp}spp_{wl.get('tag', 'pathtrace')}",
                "scene": wl["scene"],
                "camera": wl["camera"],
                "resolution": [W, H],
                "spp": spp,
                "integrator": wl.get("integrator_name", "PathTrace (NEE + MIS + RR)"),
                "seed": SEED,
                "rng_mode": "wavefront (per-path Xorshiftr128+ streams; DESIGN.md §RNG)",
                "parallelism": f"tiles sharded tile%{ws}",
            },
            "msamples_per_s": round(cams / elapsed / 1e6, 3),
            "lumo_total_rays_per_s_M": round(rays / elapsed / 1e6, 3),
            "queries_per_step": q / args.steps,
            "scene_build_s": wl["scene_build_s"],
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        print(json.dumps(out))
    dev.close()
    if pg is not None:
        pg.destroy_process_group()


def build_config(args):
    """(scene, camera, (W, H), spp, labels) of BASELINE.json's configs, built with lumo's API."""
    import lumo_amd as L
    from lumo_amd import scenes
    t0 = time.perf_counter()
    if args.config == "c1":
        W = H = args.res or 1024
        spp = args.spp or 1024
        scene, cam = scenes.cornell(), L.Camera.cornell_box((W, H))
        wl = {"name": "cornell", "scene": "Scene::cornell_box (32 triangles, 1 rectangle light)",
              "camera": "Camera::cornell_box", "data": "synthetic (Scene::cornell_box defined in code; no assets)"}
    elif args.config == "c2":
        W, H = (args.res, args.res) if args.res else (1920, 1080)
        spp = args.spp or 256
        scene, cam = scenes.dragon(), scenes.default_camera((W, H))
        wl = {"name": "dragon", "scene": "examples/dragon.rs: empty_box + 871414-triangle procedural stand-in "
                                         "(transparent MfDielectric 0.03, eta 1.5 glass curve) as an Instance",
              "camera": "Camera::builder() default", "data": "synthetic (procedural stand-in for dragon.obj)"}
    elif args.config == "c4":
        W = H = args.res or 1024
        spp = args.spp or 4096
        scene, cam = scenes.caustics(), scenes.caustics_camera((W, H))
        wl = {"name": "caustics", "scene": "examples/caustics.rs: empty_box MAGENTA/CYAN + mirror and glass "
                                           "instances of a 968-triangle suzanne stand-in",
              "camera": "origin (0,0,2), zoom 3 (caustics.rs:7-10)",
              "data": "synthetic (procedural stand-in for suzanne.obj)", "integrator": L.Integrator.BDPathTrace,
              "integrator_name": "BDPathTrace (all (s,t) strategies, MIS, light-tracing splats)", "tag": "bdpt",
              "cpu_tile_stride": 512, "cpu_batches": 1}
    else:
        W, H = (args.res, args.res) if args.res else (1920, 1080)
        spp = args.spp or 256
        scene, cam = scenes.bistro(), scenes.bistro_camera((W, H))
        wl = {"name": "bistro", "scene": "procedural Bistro stand-in: ~2.8M triangles in 400 material groups, "
                                         "2048 emissive triangles, environment light",
              "camera": "origin (-16,5,-1) towards (0,0,0) (bistro.rs:15-18)",
              "data": "synthetic (procedural stand-in for Bistro exterior)"}
    scene.build()
    wl["scene_build_s"] = round(time.perf_counter() - t0, 2)
    return scene, cam, (W, H), spp, wl


def roofline(st, n_shadow, bdpt=False, workload="c1"):
    """Dominant-kernel roofline from live per-launch HIP-event times and traversal counters."""
    ms = list(st.kernel_ms)
    launches = list(st.launches)
    per_stage = {STAGES[i]: {"ms": round(ms[i], 3), "launches": int(launches[i])} for i in range(8)}
    dom = max(range(8), key=lambda i: ms[i])
    name = STAGES[dom]
    if bdpt:
        nbytes = None  # BDPT: no algorithmic byte model yet
    elif name == "closest":
        nbytes = (st.closest_queries * B_CLOSEST_IO + st.aabb_tests[0] * B_AABB + st.kd_nodes[0] * B_KD +
                  st.tri_tests[0] * B_TRI)
    elif name == "shadow":
        # k_shadow folds a path's 2 n_shadow records into its radiance: B_FOLD is amortised per query
        b_io = B_RECORD + B_FOLD / (2 * n_shadow)
        nbytes = (st.shadow_queries * b_io + st.aabb_tests[1] * B_AABB + st.kd_nodes[1] * B_KD +
                  st.tri_tests[1] * B_TRI)
    else:
        nbytes = None
    # BDPT stage slots: walk traces = closest (k_closest), walk steps = shade (k_bdpt_step),
    # connections = shadow (k_bdpt_conn_a + k_bdpt_vis + k_bdpt_paths), re-runs + fold = resolve
    bd_names = {"closest": "bdpt_walk_trace", "shade": "bdpt_walk_step", "shadow": "bdpt_connections",
                "resolve": "bdpt_redo_fold"}
    if bdpt:
        per_stage = {bd_names.get(k, k): v for k, v in per_stage.items()}
    kname = {"closest": "k_closest", "shade": "k_bdpt_step", "shadow": "k_bdpt_vis",
             "resolve": "k_bdpt_redo"}.get(name, f"k_{name}") if bdpt else f"k_{name}"
    pmc = pmc_traffic(kname[2:]) if workload == "c1" else {}  # the committed PMC table profiles C1
    out = {"bound": "hbm", "kernel": kname, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "traffic": pmc.get("hbm_bytes_per_launch"), "traffic_raw": pmc.get("hbm_bytes_per_launch_raw"),
           "traffic_source": "profiles/pmc_traffic.json" if pmc else None, "stages": per_stage}
    cq, sq = max(st.closest_queries, 1), max(st.shadow_queries, 1)
    out["per_query"] = {
        "closest": {"aabb": st.aabb_tests[0] / cq, "kd": st.kd_nodes[0] / cq, "tri": st.tri_tests[0] / cq},
        "shadow": {"aabb": st.aabb_tests[1] / sq, "kd": st.kd_nodes[1] / sq, "tri": st.tri_tests[1] / sq}}
    if nbytes is not None and ms[dom] > 0 and launches[dom] > 0:
        achieved = nbytes / (ms[dom] * 1e-3) / 1e9
        avg_s = ms[dom] * 1e-3 / launches[dom]
        out.update({"achieved": round(achieved, 2), "frac": round(achieved / HBM_PEAK_GBS, 5),
                    "bytes_per_launch": nbytes / launches[dom], "avg_launch_us": avg_s * 1e6})
        if out["traffic"]:
            # measured DRAM-side rate of the same kernel: PMC bytes per launch over live launch time
            out["hbm_gbs_measured"] = round(out["traffic"] / avg_s / 1e9, 2)
    else:
        out.update({"achieved": None, "frac": None})
    return out


def n_shadow_rays(scene):
    """Scene::num_shadow_rays (scene.rs:90-92): max(ilog2(#lights), 1)."""
    n = scene.desc().num_lights
    return max(n.bit_length() - 1, 1)


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC summary, if present."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get(f"k_{kernel}", {})
    except (OSError, ValueError):
        return {}


def cpu_baseline(scene, cam, tasks, tiles, args, W, H, spp, wl):
    """The oracle (f64 restatement of lumo's CPU path, lumo's own tile-serial RNG order) on this
    host: every k-th tile of every batch of the same frame, all spp; Mrays/s of that sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    try:
        import oracle_ffi as O
        O.load()
    except OSError:
        return None
    integrator = wl.get("integrator", 0)
    stride = wl.get("cpu_tile_stride", args.cpu_tile_stride)
    batches = wl.get("cpu_batches", None)  # BDPT: the first batch only (CPU BDPT is ~100x slower)
    sample = [t for i, t in enumerate(tasks) if (i % tiles) % stride == 0 and (batches is None or i // tiles < batches)]
    threads = min(16, os.cpu_count() or 1)
    t0 = time.perf_counter()
    bufs, res, cnt = O.render_tasks(scene.desc(), cam.desc, sample, O.LUMO_ORDER, threads, integrator=integrator,
                                    splats_out=[] if integrator else None)
    dt = time.perf_counter() - t0
    q = sum(r.num_queries for r in res)
    paths = sum(r.num_camera_rays for r in res)
    return {"value": round(q / dt / 1e6, 4), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "msamples_per_s": round(paths / dt / 1e6, 4), "seconds": round(dt, 2),
            "sample": f"{len(sample)} tasks = every {stride}th 16x16 tile of "
                      f"{'each' if batches is None else f'the first {batches}'} 256-spp batch(es) of "
                      f"the {W}x{H} @ {spp} spp frame ({paths} paths), lumo tile-serial RNG order"}


if __name__ == "__main__":
    main()
