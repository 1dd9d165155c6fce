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
