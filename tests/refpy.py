"""Independent pure-Python/numpy restatements used to pin the C++ oracle.

* libstdc++ 11 pieces the reference calls: mt19937, uniform_int_distribution
  (Lemire nearly-divisionless, bits/uniform_int_dist.h), generate_canonical
  <float,24> (random.tcc:3348), std::shuffle (stl_algo.h:3729, pairwise form
  for n <= 65535). Checked against tests/golden/libstdcxx_golden.json.
* The reference's float arithmetic for make_table (Word2Vec.cpp:81-113) and
  precalc_sampling (:115-130), in numpy float32.
* The reference's draw ORDER for one training pass (Word2Vec.cpp:273-353,
  :251-257), to check the stream the oracle records.
"""
from __future__ import annotations

import numpy as np

M32 = 0xFFFFFFFF


class MT19937:
    def __init__(self, seed: int = 5489):
        self.mt = [0] * 624
        self.mt[0] = seed & M32
        for i in range(1, 624):
            self.mt[i] = (1812433253 * (self.mt[i - 1] ^ (self.mt[i - 1] >> 30)) + i) & M32
        self.idx = 624

    def _twist(self):
        mt = self.mt
        for i in range(624):
            y = (mt[i] & 0x80000000) | (mt[(i + 1) % 624] & 0x7FFFFFFF)
            mt[i] = mt[(i + 397) % 624] ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)
        self.idx = 0

    def __call__(self) -> int:
        if self.idx >= 624:
            self._twist()
        y = self.mt[self.idx]
        self.idx += 1
        y ^= y >> 11
        y ^= (y << 7) & 0x9D2C5680
        y ^= (y << 15) & 0xEFC60000
        y ^= y >> 18
        return y & M32


def canonical_float(x: int) -> np.float32:
    """generate_canonical<float,24> from one 32-bit draw."""
    r = np.float32(np.float32(x) / np.float32(4294967296.0))
    if r >= np.float32(1.0):
        r = np.nextafter(np.float32(1.0), np.float32(0.0))
    return np.float32(r)


def uniform_real(g, a: float, b: float) -> np.float32:
    return np.float32(canonical_float(g()) * np.float32(np.float32(b) - np.float32(a)) + np.float32(a))


def uniform_int(g, a: int, b: int) -> int:
    """uniform_int_distribution on [a, b] with a 32-bit URNG (Lemire, 64-bit product)."""
    urange = b - a
    if urange == M32:
        return g() + a
    assert urange < M32
    er = urange + 1
    prod = g() * er
    low = prod & M32
    if low < er:
        thr = ((1 << 32) - er) % er
        while low < thr:
            prod = g() * er
            low = prod & M32
    return (prod >> 32) + a


def shuffle(seq: list, g) -> list:
    """std::shuffle (libstdc++ 11) on a random-access sequence, 32-bit URNG."""
    a = list(seq)
    n = len(a)
    if n == 0:
        return a
    if M32 // n >= n:
        i = 1
        if n % 2 == 0:
            j = uniform_int(g, 0, 1)
            a[i], a[j] = a[j], a[i]
            i += 1
        while i != n:
            r = i + 1
            x = uniform_int(g, 0, r * (r + 1) - 1)
            p0, p1 = x // (r + 1), x % (r + 1)
            a[i], a[p0] = a[p0], a[i]
            i += 1
            a[i], a[p1] = a[p1], a[i]
            i += 1
        return a
    for i in range(1, n):
        j = uniform_int(g, 0, i)
        a[i], a[j] = a[j], a[i]
    return a


def make_table(counts, table_size: int) -> np.ndarray:
    """make_table (Word2Vec.cpp:81-113) in float32, sequential (small sizes only)."""
    f32 = np.float32
    V = len(counts)
    wr = [f32(np.power(f32(c), f32(0.75))) for c in counts]
    total = f32(0)
    for w in wr:
        total = f32(total + w)
    table = np.zeros(table_size, np.uint32)
    idx = 0
    d1 = f32(wr[0] / total)
    scope = f32(f32(table_size) * d1)
    i = 0
    while i < table_size:
        table[i] = idx
        if f32(i) > scope and idx < V - 1:
            idx += 1
            d1 = f32(d1 + f32(wr[idx] / total))
            scope = f32(f32(table_size) * d1)
        elif idx == V - 1:
            table[i:] = idx
            break
        i += 1
    return table


def sample_probs(counts, t: float) -> np.ndarray:
    """precalc_sampling (Word2Vec.cpp:115-130) in float32."""
    f32 = np.float32
    total = int(np.sum(np.asarray(counts, np.int64)))
    thr = f32(f32(t) * f32(total))
    out = np.ones(len(counts), np.float32)
    if not (t > 0):
        return out
    for i, c in enumerate(counts):
        cf = f32(c)
        p = f32(f32(f32(np.sqrt(f32(cf / thr))) + f32(1)) * thr)
        p = f32(p / cf)
        out[i] = min(p, f32(1.0))
    return out


def reference_draws(ids, off, keep, order, window: int, negative: int, table_size: int, model: str,
                    g) -> list:
    """Every draw the reference makes for one pass, in its order, with values:
    ('u', float bits) per token; ('w', shrink) per kept token; ('t', pos) per
    negative. SG: Word2Vec.cpp:325-349; CBOW: :279-310 (a CBOW center with
    neu1_num <= 0 draws no negatives)."""
    out = []
    for s in order:
        sent = ids[off[s]:off[s + 1]]
        L = len(sent)
        for i, c in enumerate(sent):
            u = uniform_real(g, 0.0, 1.0)
            out.append(("u", int(np.float32(u).view(np.uint32))))
            if keep[c] < u:
                continue
            rw = uniform_int(g, 0, max(window - 1, 0))
            out.append(("w", rw))
            lo, hi = max(0, i - window + rw), min(L, i + window + 1 - rw)
            if model == "cbow":
                if hi - lo - 1 <= 0:
                    continue
                for _ in range(negative):
                    out.append(("t", uniform_int(g, 0, table_size - 1)))
            else:
                for j in range(lo, hi):
                    if j == i:
                        continue
                    for _ in range(negative):
                        out.append(("t", uniform_int(g, 0, table_size - 1)))
    return out


# Philox4x32-10 known-answer vectors (Random123 kat_vectors: ctr, key, out)
PHILOX_KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


def philox4x32_10(ctr, key):
    c0, c1, c2, c3 = ctr
    k0, k1 = key
    for _ in range(10):
        p0 = 0xD2511F53 * c0
        p1 = 0xCD9E8D57 * c2
        c0, c1, c2, c3 = ((p1 >> 32) ^ c1 ^ k0) & M32, p1 & M32, ((p0 >> 32) ^ c3 ^ k1) & M32, p0 & M32
        k0 = (k0 + 0x9E3779B9) & M32
        k1 = (k1 + 0xBB67AE85) & M32
    return c0, c1, c2, c3
