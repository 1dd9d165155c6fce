"""Procedural stand-ins for the reference's downloaded benchmark assets:
the assets (Stanford dragon, Amazon Bistro) are fetched from URLs by lumo's parser and are not
available offline, so the benchmark configurations use seeded procedural meshes with the same
triangle counts and the same scene structure."""
import numpy as np

DRAGON_TRIANGLES = 871_414  # dragon.obj as loaded by lumo


def torus_knot_tube(n_along, n_around, p=3, q=7, R=1.0, r_knot=0.42, r_tube=0.13, noise=0.02, seed=1):
    """Closed tube around a (p, q) torus knot: n_along x n_around quads -> 2 * n_along * n_around
    triangles, with seeded low-frequency radial noise so the surface is not trivially regular."""
    rng = np.random.default_rng(seed)
    t = np.arange(n_along) * (2 * np.pi / n_along)
    u = np.arange(n_around) * (2 * np.pi / n_around)

    def curve(tt):
        rr = R + r_knot * np.cos(q * tt)
        return np.stack([rr * np.cos(p * tt), r_knot * np.sin(q * tt), rr * np.sin(p * tt)], -1)

    c = curve(t)
    tang = curve(t + 1e-4) - curve(t - 1e-4)
    tang /= np.linalg.norm(tang, axis=1, keepdims=True)
    ref = np.array([0.0, 1.0, 0.0])
    n1 = np.cross(tang, ref)
    n1 /= np.linalg.norm(n1, axis=1, keepdims=True)
    n2 = np.cross(tang, n1)
    # seeded smooth radial modulation: a few random harmonics along and around the tube
    k = rng.integers(1, 40, size=(6, 2))
    ph = rng.uniform(0, 2 * np.pi, size=6)
    amp = rng.uniform(0.3, 1.0, size=6)
    T, U = np.meshgrid(t, u, indexing="ij")
    mod = sum(a * np.sin(kk[0] * T + kk[1] * U + f) for a, kk, f in zip(amp, k, ph)) / amp.sum()
    rad = r_tube * (1.0 + noise / r_tube * mod)
    v = (c[:, None, :] + rad[..., None] * (np.cos(U)[..., None] * n1[:, None, :] +
                                           np.sin(U)[..., None] * n2[:, None, :]))
    v = v.reshape(-1, 3)
    i = np.arange(n_along)[:, None]
    j = np.arange(n_around)[None, :]
    a = i * n_around + j
    b = ((i + 1) % n_along) * n_around + j
    c2 = ((i + 1) % n_along) * n_around + (j + 1) % n_around
    d = i * n_around + (j + 1) % n_around
    faces = np.stack([a, b, c2, d], -1).reshape(-1, 4)
    return v, faces


def dragon_standin(seed=1):
    """871 414-triangle closed mesh: (3, 7) torus-knot tube with 10 627 x 41 quads."""
    return torus_knot_tube(10627, 41, seed=seed)


BISTRO_GROUPS = 400        # ~ number of usemtl groups (one kd-tree each, parser/obj.rs:85-108)
BISTRO_LAMPS = 1024        # emissive quads -> 2048 Triangle lights (num_shadow_rays = 11)


def _box_grid(center, size, n, rng, jitter=0.0):
    """Axis-aligned box with each face split into n x n quads (outward winding)."""
    cx, cy, cz = center
    sx, sy, sz = size
    g = np.linspace(0.0, 1.0, n + 1)
    U, V = np.meshgrid(g, g, indexing="ij")
    faces_v, faces_f, base = [], [], 0
    # (origin, edge u, edge v) per face, u x v pointing outwards
    lo = np.array([cx - sx / 2, cy, cz - sz / 2])
    E = [np.array([sx, 0, 0]), np.array([0, sy, 0]), np.array([0, 0, sz])]
    specs = [(lo, E[2], E[1]), (lo + E[0], E[1], E[2]),  # -x, +x
             (lo, E[0], E[2]), (lo + E[1], E[2], E[0]),  # -y, +y
             (lo, E[1], E[0]), (lo + E[2], E[0], E[1])]  # -z, +z
    for o, eu, ev in specs:
        P = o + U[..., None] * eu + V[..., None] * ev
        if jitter:
            nrm = np.cross(eu, ev)
            nrm = nrm / np.linalg.norm(nrm)
            inner = np.zeros_like(U, dtype=bool)
            inner[1:-1, 1:-1] = True
            P = P + (jitter * rng.standard_normal(U.shape) * inner)[..., None] * nrm
        faces_v.append(P.reshape(-1, 3))
        i = np.arange(n)[:, None] * (n + 1) + np.arange(n)[None, :]
        q = np.stack([i, i + n + 1, i + n + 2, i + 1], -1).reshape(-1, 4) + base
        faces_f.append(q)
        base += (n + 1) * (n + 1)
    return np.concatenate(faces_v), np.concatenate(faces_f)


def bistro_standin(seed=7, groups=BISTRO_GROUPS, lamps=BISTRO_LAMPS, n=24):
    """Procedural stand-in for the Bistro exterior: a ground plane and (groups - 1) buildings,
    each its own mesh (material group), ~6 900 triangles per group (~2.8 M total), plus `lamps`
    small emissive quads on the facades.  Returns (groups: [(v, f, kind, rgb)], lamps: [(v, f)])."""
    rng = np.random.default_rng(seed)
    cam = np.array([-16.0, 5.0, -1.0])
    # candidate building sites on a street grid, keeping the camera's line of sight to the origin open
    xs = np.arange(-30.0, 30.1, 2.4)
    cand = []
    for x in xs:
        for z in xs:
            p = np.array([x, 0.0, z])
            d = p[[0, 2]]
            seg = cam[[0, 2]]
            t = np.clip(np.dot(d, seg) / np.dot(seg, seg), 0.0, 1.0)
            if np.linalg.norm(d - t * seg) < 2.6 or np.linalg.norm(d) < 3.0:
                continue
            cand.append(p)
    cand.sort(key=lambda p: np.linalg.norm(p))
    sites = cand[:groups - 1]
    out = []
    ground_n = int(round(np.sqrt(6912 / 2)))
    gv, gf = _box_grid((0.0, -0.05, 0.0), (64.0, 0.05, 64.0), 1, rng)  # thin slab under the streets
    # replace the slab top with a finely split ground plane
    g = np.linspace(-32.0, 32.0, ground_n + 1)
    X, Z = np.meshgrid(g, g, indexing="ij")
    gv = np.stack([X, np.zeros_like(X), Z], -1).reshape(-1, 3)
    i = np.arange(ground_n)[:, None] * (ground_n + 1) + np.arange(ground_n)[None, :]
    gf = np.stack([i, i + 1, i + ground_n + 2, i + ground_n + 1], -1).reshape(-1, 4)
    out.append((gv, gf, "diffuse", (0.35, 0.33, 0.3)))
    facade = []
    for k, p in enumerate(sites):
        h = rng.uniform(1.5, 7.0)
        w = rng.uniform(1.2, 1.9)
        d = rng.uniform(1.2, 1.9)
        v, f = _box_grid((p[0], 0.0, p[2]), (w, h, d), n, rng, jitter=0.004)
        kind = "metal" if rng.uniform() < 0.1 else "diffuse"
        out.append((v, f, kind, tuple(rng.uniform(0.2, 0.9, 3))))
        facade.append((p, w, h, d))
    lamps_out = []
    for k in range(lamps):
        p, w, h, d = facade[k % len(facade)]
        side = rng.integers(4)
        y = rng.uniform(0.8, min(h - 0.3, 3.0))
        s = 0.08
        off = 0.02
        if side == 0:
            c, eu, ev = np.array([p[0] - w / 2 - off, y, p[2] + rng.uniform(-d, d) * 0.4]), [0, 0, s], [0, s, 0]
        elif side == 1:
            c, eu, ev = np.array([p[0] + w / 2 + off, y, p[2] + rng.uniform(-d, d) * 0.4]), [0, s, 0], [0, 0, s]
        elif side == 2:
            c, eu, ev = np.array([p[0] + rng.uniform(-w, w) * 0.4, y, p[2] - d / 2 - off]), [s, 0, 0], [0, s, 0]
        else:
            c, eu, ev = np.array([p[0] + rng.uniform(-w, w) * 0.4, y, p[2] + d / 2 + off]), [0, s, 0], [s, 0, 0]
        eu, ev = np.array(eu, dtype=float), np.array(ev, dtype=float)
        v = np.array([c - eu - ev, c + eu - ev, c + eu + ev, c - eu + ev])
        lamps_out.append((v, np.array([[0, 1, 2, 3]])))
    return out, lamps_out


SUZANNE_TRIANGLES = 968  # suzanne.obj (examples/caustics.rs) triangulated


def suzanne_standin(seed=3):
    """Closed ~1k-triangle head-like blob in place of suzanne.obj: a UV sphere (22 x 22 quads,
    fan-capped poles -> 968 triangles) squashed and given two seeded 'ear' bulges and low-frequency
    bumps, so that mirror / glass caustics come from a curved, non-convex-looking surface."""
    rng = np.random.default_rng(seed)
    n_lat, n_lon = 23, 22
    th = np.arange(1, n_lat) * (np.pi / n_lat)      # interior latitude rings
    ph = np.arange(n_lon) * (2 * np.pi / n_lon)
    T, P = np.meshgrid(th, ph, indexing="ij")
    d = np.stack([np.sin(T) * np.cos(P), np.cos(T), np.sin(T) * np.sin(P)], -1)
    k = rng.integers(1, 5, size=(4, 2))
    phase = rng.uniform(0, 2 * np.pi, size=4)
    bump = sum(np.sin(kk[0] * T + kk[1] * P + f) for kk, f in zip(k, phase)) * 0.04
    ears = 0.35 * (np.exp(-((d[..., 0] - 0.8) ** 2 + (d[..., 1] - 0.4) ** 2) * 12.0) +
                   np.exp(-((d[..., 0] + 0.8) ** 2 + (d[..., 1] - 0.4) ** 2) * 12.0))
    r = (1.0 + bump + ears)[..., None]
    v = (d * r * np.array([1.0, 0.85, 0.9])).reshape(-1, 3)
    top, bot = len(v), len(v) + 1
    v = np.vstack([v, [[0.0, 0.85, 0.0], [0.0, -0.85, 0.0]]])
    faces = []
    for i in range(n_lat - 2):
        for j in range(n_lon):
            a, b = i * n_lon + j, i * n_lon + (j + 1) % n_lon
            c, e = (i + 1) * n_lon + (j + 1) % n_lon, (i + 1) * n_lon + j
            faces += [(a, b, c), (a, c, e)]
    last = (n_lat - 2) * n_lon
    for j in range(n_lon):
        faces.append((top, (j + 1) % n_lon, j))
        faces.append((bot, last + j, last + (j + 1) % n_lon))
    return v, np.asarray(faces, dtype=np.int64)
