"""Per-rank load of an N-rank run, timed on one GPU: every share (tile % N == R) of a bench config
rendered in turn in this process (scene built and uploaded once), wall time per share, the
max/mean imbalance and each share's rate relative to the full frame's.
Usage: python tools/share_times.py <config> <N> [spp] > gpurun_out/shares_<config>.json"""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
import lumo_amd as L  # noqa: E402
from lumo_amd import _ffi  # noqa: E402
from lumo_amd.dist import shard_tasks  # noqa: E402


def main():
    config, n = sys.argv[1], int(sys.argv[2])
    spp = int(sys.argv[3]) if len(sys.argv) > 3 else None
    scene, cam, (W, H), spp, wl = bench.build_config(config, None, spp)
    tasks = L.make_tasks(W, H, spp, bench.SEED)
    dev = L.Device(0)
    dev.upload(scene, cam)
    lib = _ffi.load()

    def render(ts):
        arr = (_ffi.TileTask * len(ts))(*ts)
        t0 = time.perf_counter()
        _, res = dev.render_tasks(arr, max_paths=1 << 23)
        dt = time.perf_counter() - t0
        return dt, sum(r.num_queries for r in res), sum(r.num_camera_rays for r in res)

    render(shard_tasks(tasks, W, H, 0, n))  # warm-up
    out = {"config": config, "n": n, "spp": spp, "resolution": [W, H], "shares": []}
    lib.lumo_stats_reset(dev.ctx)
    full_t, full_q, _ = render(tasks)
    st = dev.stats()
    out["full"] = {"s": round(full_t, 4), "mrays_per_s": round((full_q - st.shadow_resolved) / full_t / 1e6, 2)}
    for r in range(n):
        lib.lumo_stats_reset(dev.ctx)
        dt, q, cams = render(shard_tasks(tasks, W, H, r, n))
        st = dev.stats()
        out["shares"].append({"rank": r, "s": round(dt, 4), "paths": cams,
                              "mrays_per_s": round((q - st.shadow_resolved) / dt / 1e6, 2)})
        print(f"share {r}/{n}: {dt:.3f} s", file=sys.stderr, flush=True)
    ts = [s["s"] for s in out["shares"]]
    out["max_over_mean"] = round(max(ts) / (sum(ts) / n), 4)
    out["sum_of_shares_s"] = round(sum(ts), 4)
    # rate of a rank at its share relative to the whole frame on one GPU (1.0 = no strong-scaling loss)
    out["share_rate_over_full"] = round(out["full"]["s"] / (sum(ts) / n) / n, 4)
    out["projected_n_gpu_speedup"] = round(full_t / max(ts), 3)
    dev.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
