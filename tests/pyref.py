"""Independent pure-Python restatements of small integer/f64 pieces of lumo, used to pin the
C++ host code and the oracle (test infrastructure only)."""
import math

M64 = (1 << 64) - 1
EPSILON = 1e-10


class Xorshift:
    """Xorshiftr128+ (lumo src/rng.rs:24-117)."""

    def __init__(self, seed):
        s = max(seed, 1)
        self.lo = s
        self.hi = s
        for _ in range(3):  # rng.rs:46
            self.step()

    def step(self):
        lo, hi = self.lo, self.hi
        self.hi = lo
        hi ^= (hi << 23) & M64
        hi ^= hi >> 17
        hi ^= lo
        self.lo = (hi + lo) & M64
        return hi

    def gen_u64(self):
        return self.step()

    def gen_float(self):  # rng.rs:71-75
        return min(float(self.step()) * 2.0 ** -64, 1.0 - EPSILON)

    def gen_vec2(self):
        x = self.gen_float()
        return x, self.gen_float()

    def gen_perm(self, n):  # rng.rs:104-116
        perm = list(range(n))
        for i in range(n - 1):
            j = i + self.gen_u64() % (n - i)
            perm[i], perm[j] = perm[j], perm[i]
        return perm


def mj_offsets(batch, total_samples, seed, count):
    """MultiJitteredSampler (samplers.rs:135-193) via SamplerType::new (samplers.rs:26-37)."""
    rng = Xorshift(seed)
    dim = math.ceil(math.sqrt(float(total_samples)))
    s0 = batch * 256
    s1 = min((batch + 1) * 256, total_samples)
    sc0 = (1.0 / dim, dim / total_samples)
    sc1 = (sc0[0] / dim, sc0[1] / dim)
    px, py = rng.gen_perm(dim), rng.gen_perm(dim)
    out = []
    for state in range(s0, min(s1, s0 + count)):
        x0, y0 = state % dim, state // dim
        o0 = (sc0[0] * x0, sc0[1] * y0)
        o1 = (sc1[0] * px[y0], sc1[1] * py[x0])
        u = rng.gen_vec2()
        r = (sc1[0] * u[0], sc1[1] * u[1])
        out.append((o0[0] + o1[0] + r[0], o0[1] + o1[1] + r[1]))
    return out


def splitmix64(z):
    z = (z + 0x9E3779B97F4A7C15) & M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & M64
    return z ^ (z >> 31)


def sampler_points(kind, batch, total_samples, seed):
    """SamplerType::new(batch, samples, seed) (samplers.rs:26-37) and every point it yields:
    kind 1 Uniform (:56-85), 2 Jittered (:87-132), 3 Sobol (:195-248 with sobol_seq.rs);
    0 MultiJittered is mj_offsets."""
    s0 = batch * 256
    s1 = min((batch + 1) * 256, total_samples)
    if kind == 0:
        return mj_offsets(batch, total_samples, seed, s1 - s0)
    if kind == 1:
        rng = Xorshift(seed)
        return [rng.gen_vec2() for _ in range(s1 - s0)]
    if kind == 2:
        rng = Xorshift(seed)
        dim = math.ceil(math.sqrt(float(total_samples)))
        sc = (1.0 / dim, dim / total_samples)
        out = []
        for state in range(s0, s1):
            off = (sc[0] * (state % dim), sc[1] * (state // dim))
            u = rng.gen_vec2()
            out.append((sc[0] * u[0] + off[0], sc[1] * u[1] + off[1]))
        return out
    # Sobol: sobol_seq.rs, written out as the const fns iterate
    deg = 10
    vs1 = [(m << (64 - i - 1)) & M64 for i, m in enumerate([1, 1, 7, 15, 5, 19, 69, 51, 121, 695])]
    vs2 = [(m << (64 - i - 1)) & M64 for i, m in enumerate([1, 1, 7, 7, 7, 53, 57, 229, 473, 533])]
    max_len = (1 << deg) - 1
    batch_states = [(0, 0)] * (1 + max_len // 256)
    state, prev = 0, (0, 0)
    while state < max_len:
        if state % 256 == 0:
            batch_states[state // 256] = prev
        state += 1
        tz = (state & -state).bit_length() - 1
        prev = (prev[0] ^ vs1[tz], prev[1] ^ vs2[tz])
    state, prev = s0, batch_states[batch]
    out = []
    while state != s1:
        state += 1
        tz = (state & -state).bit_length() - 1
        prev = (prev[0] ^ vs1[tz], prev[1] ^ vs2[tz])
        out.append((float(prev[0] ^ seed) * 2.0 ** -64, float(prev[1] ^ seed) * 2.0 ** -64))
    return out
