#!/usr/bin/env python3
"""Benchmark: BASELINE.json's metric, "Mrays/sec + Msamples/sec ... Cornell 1024spp and Bistro 256spp".

Default run (the driver's `python bench.py --gpus N --steps K --warmup W`):
  * C1 = BASELINE configs[1]: lumo's Cornell box, PathTrace, 1024x1024 @ 1024 spp.  One "step" is
    the whole frame: every (256-spp batch, 16x16 tile) RenderTask (renderer.rs:179-204),
    4 batches x 4096 tiles = 1.07e9 camera paths.  W warmup frames, then K timed frames.  These
    are the top-level fields of the JSON line.
  * C3 = BASELINE configs[3]: the Bistro stand-in, PathTrace, 1920x1080 @ 256 spp, one timed
    frame after a 1-spp warmup frame (`--bistro-frames`, 0 disables).  Reported under "c3" with
    its own ms_per_step, roofline and CPU baseline.
  * C2 = BASELINE configs[2]: the dragon stand-in, PathTrace, 1920x1080 @ 256 spp, one timed frame
    after a 1-spp warmup frame (`--dragon-frames`, 0 disables), under "c2".
  * C4 = BASELINE configs[4] (caustics.rs, BDPT, 1024x1024 @ 4096 spp, quoted on 8 GPUs): one
    rank's share of the 8-GPU run (the tiles with tile % 8 == 0, `--c4-share`, "" disables), timed
    on this GPU after a 1-spp warmup, under "c4_share" with "share": "0/8".
With N ranks (one per GPU, launched by torch.distributed.run) the tasks are sharded by tile index
(tile % N == rank, all batches of a tile on one rank), the scene is replicated, and no collective
touches the data path; only the timing barriers and the final max/sum of scalars use the group.

`value` is whole-job Mrays/s = (closest-hit + shadow-visibility queries of all ranks) / max-over-
ranks wall time of the timed frames: lumo's Scene::hit / hit_light calls for the frame, including
the shadow records the device answers without a traversal because their contribution is 0
whatever the visibility (`shadow_resolved_per_step`; `mrays_traversed_per_s` excludes them).
Also reported: Msamples/s (camera paths), lumo's own "total
rays" rate (sum of path depths, task.rs:65), the roofline of the dominant kernel (algorithmic
bytes from the kernels' own traversal counters over live HIP-event kernel time, DESIGN.md
§Roofline), and the CPU baseline (the f64 oracle in lumo's tile-serial order on this host's
cores, on a bounded sample of the same frame, at all usable cores and at lumo's default 4).
"""
import argparse
import json
import math
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
B_CONN_IO = 104  # BDPT connection query: the two vertices' position / error / normal in, result out
# wide accel (LUMO_OPT_ACCEL = 1): its counters are child boxes tested (aabb), nodes
# visited (kd) and triangles tested; a node visit reads its 128-B node (four f32 boxes, refs), a
# triangle test its 80-B leaf record (three f64 vertices + ids)
B_WNODE, B_WTRI = 128, 80
# acceleration structure per workload (--accel auto): the wide BVH where it measured faster
ACCEL_AUTO = {"c1": 0, "c2": 1, "c3": 1, "c4": 1}
LUMO_DEFAULT_THREADS = 4  # renderer.rs:21
CPU_REPEATS = 3  # CPU baseline: median of this many runs per thread count
# f64 VALU peak in lane-operations per second (an FMA counts once): 256 CUs x 4 SIMDs x 16 f64
# lanes per cycle x 2.4 GHz = 78.6 TFLOP/s / 2 (MI355X FP64 vector rate).  The VALU bound prices
# every VALU lane-operation at this rate (integer / f32 ops issue at twice it, so the fraction is
# an upper bound on how busy the f64 pipe is).
VALU_PEAK_LANE_OPS = 256 * 4 * 16 * 2.4e9
# timed stages (lumo_amd._ffi.STAGES indices) of each roofline unit
UNIT_STAGES = {"k_bounce_q+k_bounce_tail": [1, 4], "k_closest": [1], "k_shadow": [3],
               "k_bdpt_trace_a+k_bdpt_vis": [8, 10], "frame": list(range(12))}


def progress(msg):
    """A progress line on stderr (long default runs: the C4 share and the CPU baselines)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


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
    ap.add_argument("--bistro-frames", type=int, default=1,
                    help="with --config c1: also time this many C3 Bistro frames at 1920x1080@256 (0: skip)")
    ap.add_argument("--bistro-spp", type=int, default=256)
    ap.add_argument("--dragon-frames", type=int, default=1,
                    help="with --config c1: also time this many C2 dragon frames at 1920x1080@256 (0: skip)")
    ap.add_argument("--c4-share", default="0/8",
                    help="with --config c1: also time this rank share R/N of the C4 caustics BDPT frame "
                         "(1024^2@4096) on this GPU (empty: skip)")
    ap.add_argument("--max-paths", type=int, default=1 << 23, help="paths in flight per wavefront")
    ap.add_argument("--max-vertices", type=int, default=0, help="BDPT vertex storage per subpath (0 = 128)")
    ap.add_argument("--cpu-baseline", type=int, default=1, help="time the oracle on the host (rank 0, N=1)")
    ap.add_argument("--cpu-seconds", type=float, default=4.0, help="target CPU work per baseline run (x3 repeats)")
    ap.add_argument("--share", default=None,
                    help="R/N: render only rank R's share of an N-rank run (tile %% N == R) in this single "
                         "process, to time one rank's load of a multi-GPU run on one GPU")
    ap.add_argument("--schedule", default="static", choices=["static", "dynamic"],
                    help="multi-GPU tile distribution: tile %% N (static) or chunks claimed from a shared "
                         "queue in the process group's store (dynamic, lumo_amd.dist.TileQueue)")
    ap.add_argument("--chunk", type=int, default=None, help="tiles per claim of the dynamic schedule")
    ap.add_argument("--accel", default="auto", choices=["auto", "lumo", "wide"],
                    help="walks over lumo's BVHs + kd-trees (bit-exact with the reference) or the wide BVH "
                         "(LUMO_OPT_ACCEL, DESIGN.md 4b); auto: per workload, ACCEL_AUTO")
    args = ap.parse_args()

    ws, rank, local = dist_env()
    pg = None
    if ws > 1:
        import torch
        import torch.distributed as dist
        # LUMO_BENCH_BACKEND=gloo with more ranks than GPUs rehearses the multi-rank path on one
        # GPU (RCCL refuses two ranks on one device); the driver's runs use RCCL, one GPU per rank
        backend = os.environ.get("LUMO_BENCH_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        n_dev = torch.cuda.device_count()
        if n_dev > 0:
            local = local % n_dev
        if backend == "nccl":
            torch.cuda.set_device(local)
        dist.init_process_group(backend=backend)
        pg = dist

    main_res = run(args.config, args, ws, rank, local, pg, steps=args.steps, warmup=args.warmup,
                   res=args.res, spp=args.spp, share=args.share)
    extra = {}
    if args.config == "c1" and args.bistro_frames > 0:
        extra["c3"] = run("c3", args, ws, rank, local, pg, steps=args.bistro_frames, warmup=1, spp=args.bistro_spp,
                          warm_spp=1)
    if args.config == "c1" and args.dragon_frames > 0:
        extra["c2"] = run("c2", args, ws, rank, local, pg, steps=args.dragon_frames, warmup=1, warm_spp=1)
    if args.config == "c1" and args.c4_share and ws == 1:
        # one rank's load of the 8-GPU C4 run (BASELINE configs[4] is quoted on 8 GPUs), on this GPU
        extra["c4_share"] = run("c4", args, ws, rank, local, pg, steps=1, warmup=1, warm_spp=1, share=args.c4_share)
    if rank == 0:
        out = main_res
        keys = ("metric", "value", "unit", "steps", "warmup", "ms_per_step", "dtype", "data", "config",
                "msamples_per_s", "lumo_total_rays_per_s_M", "queries_per_step", "shadow_resolved_per_step",
                "mrays_traversed_per_s", "mrays_lumo_equivalent_per_s", "scene_build_s", "sample_checks", "roofline",
                "cpu_baseline", "warmup_spp", "share")
        for name, rec in extra.items():
            out[name] = {k: rec[k] for k in keys if k in rec}
        print(json.dumps(out))
    if pg is not None:
        pg.destroy_process_group()


def run(config, args, ws, rank, local, pg, steps, warmup, res=None, spp=None, warm_spp=None, share=None):
    """Render `steps` timed frames of `config` (after `warmup` frames, at `warm_spp` if given) and
    return the JSON record (rank 0 fields complete).  `share` "R/N": only the tiles with
    tile % N == R (one rank's load of an N-rank run), in this process."""
    import lumo_amd as L
    from lumo_amd import _ffi
    from lumo_amd.dist import TileQueue, shard_tasks, tasks_of_tiles, tiles_per_batch

    progress(f"{config}: building the scene")
    scene, cam, (W, H), spp, wl = build_config(config, res, spp)
    progress(f"{config}: {W}x{H} @ {spp} spp{' share ' + share if share else ''}, scene built in {wl['scene_build_s']} s")
    bdpt = wl.get("integrator") == L.Integrator.BDPathTrace
    tasks = L.make_tasks(W, H, spp, SEED)
    tiles = tiles_per_batch(W, H)
    if share:
        sr, sn = (int(x) for x in share.split("/"))
        mine = shard_tasks(tasks, W, H, sr, sn)
    else:
        mine = shard_tasks(tasks, W, H, rank, ws)
    mine_arr = (_ffi.TileTask * len(mine))(*mine)
    warm_arr = mine_arr
    if warm_spp is not None:
        wr, wn = (int(x) for x in share.split("/")) if share else (rank, ws)
        wt = shard_tasks(L.make_tasks(W, H, warm_spp, SEED), W, H, wr, wn)
        warm_arr = (_ffi.TileTask * len(wt))(*wt)

    splat_film = np.zeros((H, W, 3)) if bdpt else None
    accel = ACCEL_AUTO[config] if args.accel == "auto" else int(args.accel == "wide")
    dev = L.Device(local, accel=accel)
    dev.upload(scene, cam)
    accel = dev.scene_info().accel  # 0 when the build refused the scene
    lib = _ffi.load()

    def step(arr):
        if bdpt:
            splat_film[:] = 0.0
            bufs, res_ = dev.render_tasks(arr, max_paths=args.max_paths, integrator=L.Integrator.BDPathTrace,
                                          splat_film=splat_film, max_vertices=args.max_vertices)
        else:
            bufs, res_ = dev.render_tasks(arr, max_paths=args.max_paths)
        return sum(r.num_queries for r in res_), sum(r.num_camera_rays for r in res_), sum(r.num_rays for r in res_)

    def barrier():
        if pg is not None:
            import torch
            if torch.cuda.is_available():
                torch.cuda.synchronize()
            pg.barrier()

    for _ in range(warmup):
        step(warm_arr)
    progress(f"{config}: warmup done, timing {steps} step(s)")
    dev.set_option("timing", 1)
    lib.lumo_stats_reset(dev.ctx)
    barrier()
    t0 = time.perf_counter()
    q = cams = rays = 0
    dynamic = getattr(args, "schedule", "static") == "dynamic" and ws > 1 and not share
    for _ in range(steps):
        if dynamic:
            # every rank builds one queue per timed frame, in the same order (TileQueue keys)
            for tl in TileQueue(W, H, ws, chunk=args.chunk):
                part = tasks_of_tiles(tasks, W, H, tl)
                a, b, c = step((_ffi.TileTask * len(part))(*part))
                q, cams, rays = q + a, cams + b, rays + c
            continue
        a, b, c = step(mine_arr)
        q, cams, rays = q + a, cams + b, rays + c
    barrier()  # lumo_render_tiles returns only after its stream has drained
    elapsed = time.perf_counter() - t0
    progress(f"{config}: {elapsed / steps * 1e3:.1f} ms per step")
    dev.set_option("timing", 0)
    st = dev.stats()
    # busy time (union of launch intervals) of every stage and of the roofline units
    busy = {name: dev.busy_ms(stages) for name, stages in UNIT_STAGES.items()}
    busy["_stages"] = [dev.busy_ms([k]) for k in range(len(_ffi.STAGES))]
    checks = [st.samples_nan, st.samples_neg, st.samples_large]
    resolved = st.shadow_resolved

    if pg is not None:
        import torch
        dev_t = "cuda" if pg.get_backend() == "nccl" else "cpu"
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev_t)
        pg.all_reduce(t, op=pg.ReduceOp.MAX)
        elapsed = float(t.item())
        s = torch.tensor([q, cams, rays, resolved] + checks, dtype=torch.float64, device=dev_t)
        pg.all_reduce(s, op=pg.ReduceOp.SUM)
        q, cams, rays, resolved = (float(x) for x in s.tolist()[:4])
        checks = [int(x) for x in s.tolist()[4:]]
    dev.close()

    out = None
    if rank == 0:
        # a rank's share launches fewer paths per pass: its own PMC entry when one was profiled
        wkey = f"{config}_share" if share and pmc_traffic(f"{config}_share", "source") else config
        roof = roofline(st, n_shadow_rays(scene), bdpt=bdpt, workload=wkey, elapsed=elapsed, busy=busy, accel=accel)
        cpu = cpu_baseline(scene, cam, tasks, tiles, args, W, H, spp, wl, repeats=wl.get("cpu_repeats", CPU_REPEATS)) \
            if (args.cpu_baseline and ws == 1) else None
        out = {
            "metric": "Mrays/s",
            # traversed queries only: the shadow records answered without a traversal (their BSDF
            # pdf is 0, integrator.rs:146) are in the lumo-equivalent rate below, not here
            "value": round((q - resolved) / elapsed / 1e6, 3),
            "unit": "Mrays/s",
            "n_gpus": ws,
            "steps": steps,
            "warmup": warmup,
            "ms_per_step": round(elapsed / steps * 1e3, 3),
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
                "parallelism": (f"tiles from a shared queue, {ws} ranks" if dynamic else f"tiles sharded tile%{ws}"),
                "accel": ("wide (4-wide SAH BVH, LUMO_OPT_ACCEL=1; DESIGN.md 4b)" if accel else
                          "lumo (objects/lights BVH + per-mesh kd-trees, bit-exact with the reference)"),
            },
            "msamples_per_s": round(cams / elapsed / 1e6, 3),
            "lumo_total_rays_per_s_M": round(rays / elapsed / 1e6, 3),
            "queries_per_step": q / steps,
            # of which shadow records answered without a traversal (their BSDF pdf is 0, so
            # mis_sample returns 0 whatever the visibility, integrator.rs:146)
            "shadow_resolved_per_step": resolved / steps,
            "mrays_traversed_per_s": round((q - resolved) / elapsed / 1e6, 3),
            # every Scene::hit / hit_light call lumo would make for the frame (the traversed ones +
            # the shadow records the device resolves without traversal)
            "mrays_lumo_equivalent_per_s": round(q / elapsed / 1e6, 3),
            "scene_build_s": wl["scene_build_s"],
            # tone_mapping.rs:42-56 debug checks over the timed camera samples: NaN, negative, > 1000
            "sample_checks": {"nan": checks[0], "negative": checks[1], "large": checks[2]},
            "roofline": roof,
            "cpu_baseline": cpu,
        }
        if warm_spp is not None:
            out["warmup_spp"] = warm_spp
        if share:
            out["share"] = share  # one rank's load of an N-rank run, timed on this one GPU
    del scene
    return out


def build_config(name, res=None, spp_override=None):
    """(scene, camera, (W, H), spp, labels) of BASELINE.json's configs, built with lumo's API."""
    import lumo_amd as L
    from lumo_amd import scenes
    t0 = time.perf_counter()
    if name == "c1":
        W = H = res or 1024
        spp = spp_override or 1024
        scene, cam = scenes.cornell(), L.Camera.cornell_box((W, H))
        wl = {"name": "cornell", "scene": "Scene::cornell_box (32 triangles, 1 rectangle light)",
              "camera": "Camera::cornell_box", "data": "synthetic (Scene::cornell_box defined in code; no assets)",
              "cpu_tile_stride": 32}
    elif name == "c2":
        W, H = (res, res) if res else (1920, 1080)
        spp = spp_override or 256
        scene, cam = scenes.dragon(), scenes.default_camera((W, H))
        wl = {"name": "dragon", "scene": "examples/dragon.rs: empty_box + 871414-triangle procedural stand-in "
                                         "(transparent MfDielectric 0.03, eta 1.5 glass curve) as an Instance",
              "camera": "Camera::builder() default", "data": "synthetic (procedural stand-in for dragon.obj)",
              "cpu_tile_stride": 256}
    elif name == "c4":
        W = H = res or 1024
        spp = spp_override or 4096
        scene, cam = scenes.caustics(), scenes.caustics_camera((W, H))
        wl = {"name": "caustics", "scene": "examples/caustics.rs: empty_box MAGENTA/CYAN + mirror and glass "
                                           "instances of a 968-triangle suzanne stand-in",
              "camera": "origin (0,0,2), zoom 3 (caustics.rs:7-10)",
              "data": "synthetic (procedural stand-in for suzanne.obj)", "integrator": L.Integrator.BDPathTrace,
              "integrator_name": "BDPathTrace (all (s,t) strategies, MIS, light-tracing splats)", "tag": "bdpt",
              "cpu_tile_stride": 512, "cpu_batches": 1}
    else:
        W, H = (res, res) if res else (1920, 1080)
        spp = spp_override or 256
        scene, cam = scenes.bistro(), scenes.bistro_camera((W, H))
        wl = {"name": "bistro", "scene": "procedural Bistro stand-in: ~2.8M triangles in 400 material groups, "
                                         "2048 emissive triangles, environment light",
              "camera": "origin (-16,5,-1) towards (0,0,0) (bistro.rs:15-18)",
              "data": "synthetic (procedural stand-in for Bistro exterior)", "cpu_tile_stride": 512}
    scene.build()
    wl["scene_build_s"] = round(time.perf_counter() - t0, 2)
    return scene, cam, (W, H), spp, wl


def roofline(st, n_shadow, bdpt=False, workload="c1", elapsed=None, busy=None, accel=0):
    """Dominant-kernel roofline from live HIP-event launch intervals and traversal counters.

    Unit = one ray query; bytes = IO + 48 per AABB test + 16 per kd split visit + 84 per triangle
    test (f64), the counters being the kernels' own (identical to the oracle's on the same rays).
    PathTrace: k_closest (closest IO) or k_shadow (shadow record + the per-path fold amortised
    over its 2 n_shadow queries), or, with fused bounces, k_bounce_q + its tail kernel as one unit.
    BDPT: the walk traces (k_closest) or the connection traversals (k_bdpt_trace_a + k_bdpt_vis).

    Time base: the unit's BUSY time, the union of its launches' [start, end] intervals (HIP events
    on the streams they run on).  With pipelined passes launches of the unit overlap on several
    streams, so the sum of launch durations exceeds the time the unit occupied the GPU (it can
    exceed the frame time); the union never does.  `achieved` = algorithmic bytes / busy time.
    The per-launch view (bytes per launch / average launch duration, what rocprofv3's average
    duration checks) is reported beside it as `achieved_per_launch`."""
    from lumo_amd._ffi import STAGES
    ms = list(st.kernel_ms)
    launches = list(st.launches)
    busy = busy or {}
    bst = busy.get("_stages", [None] * len(STAGES))
    per_stage = {STAGES[i]: {"ms": round(ms[i], 3), "busy_ms": None if bst[i] is None else round(bst[i], 3),
                             "launches": int(launches[i])} for i in range(len(STAGES))}
    cq = max(st.closest_queries, 1)
    # shadow records resolved without traversal (p_sct == 0) read only their pdf
    traversed = st.shadow_queries - st.shadow_resolved
    sq = max(traversed, 1)
    if accel:  # wide walks: 128 B per node visited, 80 B per triangle record (boxes are in the node)
        closest_bytes = st.closest_queries * B_CLOSEST_IO + st.kd_nodes[0] * B_WNODE + st.tri_tests[0] * B_WTRI
        trav1 = st.kd_nodes[1] * B_WNODE + st.tri_tests[1] * B_WTRI
    else:
        closest_bytes = (st.closest_queries * B_CLOSEST_IO + st.aabb_tests[0] * B_AABB + st.kd_nodes[0] * B_KD +
                         st.tri_tests[0] * B_TRI)
        trav1 = st.aabb_tests[1] * B_AABB + st.kd_nodes[1] * B_KD + st.tri_tests[1] * B_TRI

    def unit(name, stages, nbytes):
        return (sum(ms[i] for i in stages), sum(launches[i] for i in stages), nbytes, busy.get(name))

    if bdpt:
        cands = {"k_closest": unit("k_closest", [1], closest_bytes),
                 "k_bdpt_trace_a+k_bdpt_vis": unit("k_bdpt_trace_a+k_bdpt_vis", [8, 10],
                                                   st.shadow_queries * B_CONN_IO + trav1)}
    else:
        b_io = B_RECORD + B_FOLD / (2 * n_shadow)
        shadow_bytes = traversed * b_io + st.shadow_resolved * 8 + trav1
        if n_shadow == 1 and ms[1] > 0 and ms[2] == 0:
            # fused bounce (k_bounce_q: closest hit + shading + the NEE pair, 'closest' stage) and
            # its tail kernel ('resolve' stage for n_shadow == 1): one unit carrying every query
            cands = {"k_bounce_q+k_bounce_tail": unit("k_bounce_q+k_bounce_tail", [1, 4], closest_bytes + shadow_bytes)}
        else:
            cands = {"k_closest": unit("k_closest", [1], closest_bytes), "k_shadow": unit("k_shadow", [3], shadow_bytes)}
    dom_stage = STAGES[max(range(len(STAGES)), key=lambda i: ms[i])]
    kname = max(cands, key=lambda k: cands[k][3] if cands[k][3] is not None else cands[k][0])
    kms, kl, nbytes, kbusy = cands[kname]
    pmc = pmc_traffic(workload, kname)
    out = {"bound": "hbm", "kernel": kname, "longest_stage": dom_stage, "peak": HBM_PEAK_GBS, "unit": "GB/s",
           "traffic": pmc.get("hbm_bytes_per_launch"), "traffic_raw": pmc.get("hbm_bytes_per_launch_raw"),
           "traffic_source": f"profiles/pmc_traffic.json[{workload}]" if pmc else None, "stages": per_stage}
    ka, kk = ("boxes", "nodes") if accel else ("aabb", "kd")
    out["per_query"] = {
        "closest": {ka: st.aabb_tests[0] / cq, kk: st.kd_nodes[0] / cq, "tri": st.tri_tests[0] / cq},
        ("connection" if bdpt else "shadow"): {ka: st.aabb_tests[1] / sq, kk: st.kd_nodes[1] / sq,
                                               "tri": st.tri_tests[1] / sq}}
    out["byte_model"] = ("query IO + 128 B per wide node visited + 80 B per triangle record" if accel else
                         "query IO + 48 B per AABB test + 16 B per kd node + 84 B per triangle test")
    if kms > 0 and kl > 0:
        t_busy = (kbusy if kbusy else kms) * 1e-3
        achieved = nbytes / t_busy / 1e9
        avg_s = kms * 1e-3 / kl
        out.update({"achieved": round(achieved, 2), "frac": round(achieved / HBM_PEAK_GBS, 5),
                    "bytes_per_launch": nbytes / kl, "launches": kl, "busy_ms": round(t_busy * 1e3, 3),
                    "launch_ms_sum": round(kms, 3), "avg_launch_us": avg_s * 1e6,
                    "achieved_per_launch": round(nbytes / (kms * 1e-3) / 1e9, 2),
                    "frac_per_launch": round(nbytes / (kms * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)})
        if elapsed:
            out["busy_over_wall"] = round(t_busy / elapsed, 4)
        if out["traffic"]:
            # measured DRAM bytes of the same launches over the unit's busy time
            out["hbm_gbs_measured"] = round(out["traffic"] * kl / t_busy / 1e9, 2)
            out["traffic_over_algorithmic"] = round(out["traffic"] / (nbytes / kl), 3)
        lane_ops = pmc.get("valu_lane_ops_per_launch")
        if lane_ops:
            va = lane_ops * kl / t_busy
            out["valu"] = {"bound": "valu", "achieved": round(va / 1e12, 3), "peak": round(VALU_PEAK_LANE_OPS / 1e12, 3),
                           "unit": "T lane-op/s (f64 rate)", "frac": round(va / VALU_PEAK_LANE_OPS, 5),
                           "lanes_active_per_valu_inst": pmc.get("lanes_active_per_valu_inst"),
                           "source": out["traffic_source"]}
    else:
        out.update({"achieved": None, "frac": None})
    return out


def n_shadow_rays(scene):
    """Scene::num_shadow_rays (scene.rs:90-92): max(ilog2(#lights), 1)."""
    n = scene.desc().num_lights
    return max(n.bit_length() - 1, 1)


def pmc_traffic(workload, kernel):
    """HBM bytes per launch of `kernel` for `workload` from the committed rocprofv3 PMC summary
    (kernel "source": the entry's provenance string, i.e. whether the workload was profiled)."""
    p = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        with open(p) as f:
            d = json.load(f)
        return d.get(workload, {}).get(kernel, {})
    except (OSError, ValueError):
        return {}


def host_cpus():
    """Cores this process may use: the affinity mask, capped by a cgroup v2 CPU quota if one is
    set (on the GPU box os.cpu_count() reports the whole machine), and the CPU model."""
    n_aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    try:
        q, period = open("/sys/fs/cgroup/cpu.max").read().split()[:2]
        if q != "max":
            quota = int(q) / int(period)
    except (OSError, ValueError):
        pass
    usable = min(n_aff, max(1, math.floor(quota))) if quota else n_aff
    model = None
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return {"usable": usable, "os_cpu_count": os.cpu_count(), "affinity": n_aff,
            "cgroup_quota_cpus": quota, "model": model}


def cpu_baseline(scene, cam, tasks, tiles, args, W, H, spp, wl, repeats=CPU_REPEATS):
    """The oracle (f64 restatement of lumo's CPU path, lumo's own tile-serial RNG order) on this
    host, BASELINE.md §5: once with every usable core and once with lumo's default 4 threads
    (renderer.rs:21).  Each run renders every k-th tile of the frame's batches at the frame's spp,
    with k scaled to the thread count so each run is ~--cpu-seconds of work; the rate is per query
    (and per camera sample) of that sample."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    try:
        import oracle_ffi as O
        O.load()
    except OSError:
        return None
    integrator = wl.get("integrator", 0)
    batches = wl.get("cpu_batches", None)  # BDPT: the first batch only (CPU BDPT is ~100x slower)
    info = host_cpus()
    runs = []
    # stride for 16 threads at ~8 s (measured per config), scaled to the thread count
    base_stride = wl.get("cpu_tile_stride", 32)
    space = [i for i in range(len(tasks)) if batches is None or i // tiles < batches]
    for threads in sorted({info["usable"], LUMO_DEFAULT_THREADS}, reverse=True):
        stride = max(1, int(round(base_stride * 16 / threads * 8.0 / args.cpu_seconds))) | 1
        # a whole number of tasks per thread (at least one each: a thread without a tile would
        # understate the host), evenly spaced over the frame's tiles
        n = max(threads, -(-(-(-len(space) // stride)) // threads) * threads)
        n = min(n, len(space))
        sample = [tasks[space[(k * len(space)) // n]] for k in range(n)]
        times = []
        progress(f"cpu baseline: {len(sample)} tiles at {threads} threads x {repeats}")
        for _ in range(repeats):  # the host is shared: the median of repeated runs, with their spread
            t0 = time.perf_counter()
            bufs, res, cnt = O.render_tasks(scene.desc(), cam.desc, sample, O.LUMO_ORDER, threads,
                                            integrator=integrator, splats_out=[] if integrator else None)
            times.append(time.perf_counter() - t0)
        dt = sorted(times)[len(times) // 2]
        q = sum(r.num_queries for r in res)
        paths = sum(r.num_camera_rays for r in res)
        runs.append({"threads": threads, "value": round(q / dt / 1e6, 4), "msamples_per_s": round(paths / dt / 1e6, 4),
                     "seconds": round(dt, 2), "repeats": len(times),
                     "value_min": round(q / max(times) / 1e6, 4), "value_max": round(q / min(times) / 1e6, 4),
                     "sample": f"{len(sample)} 16x16 tiles evenly spaced over "
                               f"{'all' if batches is None else f'the first {batches}'} 256-spp batch(es) of "
                               f"the {W}x{H} @ {spp} spp frame ({paths} paths), lumo tile-serial RNG order"})
    best = runs[0]
    return {"value": best["value"], "unit": "Mrays/s", "cores": best["threads"], "kind": "port",
            "statistic": f"median of {repeats} runs", "value_min": best["value_min"],
            "value_max": best["value_max"],
            "msamples_per_s": best["msamples_per_s"], "seconds": best["seconds"], "sample": best["sample"],
            "cpu_model": info["model"], "host": info, "runs": runs}


if __name__ == "__main__":
    main()
