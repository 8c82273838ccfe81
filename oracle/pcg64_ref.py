"""Pure-Python restatement of numpy's default_rng(seed).choice(n, size, replace=True) — the
replay sampling stream of the reference (src/replaybuffer.py:101-130). TEST INFRASTRUCTURE
ONLY (the checker of graph-marl_amd/csrc/gm_replay.hip).

numpy is a dependency of the reference (pyproject.toml, unpinned), not vendored in it; its
algorithm is restated from numpy/random: bit_generator.pyx (SeedSequence: hashmix / mix over a
4-word pool, generate_state), _pcg64.pyx + pcg64.h (PCG64 = 128-bit LCG with XSL-RR 64-bit
output, seeded by pcg_setseq_128_srandom_r; 32-bit draws take the low half of an output and
buffer the high half), distributions.c (random_bounded_uint64_fill ->
buffered_bounded_lemire_uint32 for n - 1 < 2^32 - 1). Pinned against the numpy of this image
by tests/test_replay_rng.py.
"""
M32 = 0xFFFFFFFF
M64 = (1 << 64) - 1
M128 = (1 << 128) - 1
MULT = (2549297995355413924 << 64) | 4865540595714422341
INIT_A, MULT_A, INIT_B, MULT_B = 0x43B0D7E5, 0x931E8875, 0x8B51F9DD, 0x58F38DED
MIX_L, MIX_R = 0xCA01F9DD, 0x4973F715


def entropy_words(seed):
    """An integer seed as little-endian 32-bit words (at least one)."""
    w = []
    while True:
        w.append(seed & M32)
        seed >>= 32
        if seed == 0:
            return w


def seedseq_state(seed, n_words64=4):
    """SeedSequence(seed).generate_state(n_words64, np.uint64)."""
    ent = entropy_words(seed)
    hc = [INIT_A]

    def hashmix(v):
        v ^= hc[0]
        hc[0] = (hc[0] * MULT_A) & M32
        v = (v * hc[0]) & M32
        return v ^ (v >> 16)

    def mix(x, y):
        r = (MIX_L * x - MIX_R * y) & M32
        return r ^ (r >> 16)

    pool = [hashmix(ent[i] if i < len(ent) else 0) for i in range(4)]
    for s in range(4):
        for d in range(4):
            if s != d:
                pool[d] = mix(pool[d], hashmix(pool[s]))
    for s in range(4, len(ent)):
        for d in range(4):
            pool[d] = mix(pool[d], hashmix(ent[s]))
    out, hb = [], INIT_B
    for i in range(2 * n_words64):
        v = pool[i % 4] ^ hb
        hb = (hb * MULT_B) & M32
        v = (v * hb) & M32
        out.append(v ^ (v >> 16))
    return [out[2 * i] | (out[2 * i + 1] << 32) for i in range(n_words64)]


class PCG:
    """numpy.random.PCG64 seeded like default_rng(seed)."""

    def __init__(self, seed):
        v = seedseq_state(seed)
        s, seq = (v[0] << 64) | v[1], (v[2] << 64) | v[3]
        self.inc = ((seq << 1) | 1) & M128
        self.state = 0
        self._step()
        self.state = (self.state + s) & M128
        self._step()
        self.has, self.u = 0, 0

    def _step(self):
        self.state = (self.state * MULT + self.inc) & M128

    def next64(self):
        self._step()
        x = ((self.state >> 64) ^ self.state) & M64
        r = self.state >> 122
        return ((x >> r) | (x << ((64 - r) & 63))) & M64

    def next32(self):
        if self.has:
            self.has = 0
            return self.u
        n = self.next64()
        self.has, self.u = 1, n >> 32
        return n & M32

    def bounded(self, n):
        """integers(0, n) for n - 1 < 2^32 - 1 (Lemire, numpy's rejection rule)."""
        rng = n - 1
        if rng == 0:
            return 0
        m = self.next32() * n
        left = m & M32
        if left < n:
            th = (M32 - rng) % n
            while left < th:
                m = self.next32() * n
                left = m & M32
        return m >> 32


def choice(p, n, k):
    """Generator.choice(n, k, replace=True) continuing PCG p."""
    return [p.bounded(n) for _ in range(k)]


def numpy_state(p):
    return {"state": p.state, "inc": p.inc, "has_uint32": p.has, "uinteger": p.u}
