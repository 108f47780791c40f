"""The generator ring's batched refill (bdpt_device.hpp mt_ring_ahead_wave): a wave
computes outputs g .. g + 63 of std::mt19937 at once, every lane reading its three
ring words before any lane writes. Checked here on the CPU against numpy's MT19937
(the same engine as std::mt19937, seeded with std::mt19937's recurrence): the
batched ring's outputs equal the engine's, and the one-at-a-time order
(mt_ring_ahead) gives the same words — fewer than 227 consecutive outputs never read
one another (output n reads n - 624, n - 623 and n - 227)."""
import numpy as np

M = 0xFFFFFFFF


def seed_words(seed):
    x = [seed & M]
    for i in range(1, 624):
        x.append((1812433253 * (x[-1] ^ (x[-1] >> 30)) + i) & M)
    return x


def twist(a, b, c):
    y = (a & 0x80000000) | (b & 0x7FFFFFFF)
    return c ^ (y >> 1) ^ (0x9908B0DF if y & 1 else 0)


def temper(v):
    v ^= v >> 11
    v ^= (v << 7) & 0x9D2C5680
    v ^= (v << 15) & 0xEFC60000
    v ^= v >> 18
    return v & M


def first_624(x):
    """outputs 0..623 (untempered), as mt_ring_ahead builds them from the seeding values"""
    u = []
    for n in range(624):
        if n < 227:
            u.append(twist(x[n], x[n + 1], x[n + 397]))
        elif n < 623:
            u.append(twist(x[n], x[n + 1], u[n - 227]))
        else:
            u.append(twist(x[623], u[0], u[396]))
    return u


def refill(ring, g, want, batched):
    if batched:  # every read, then every write (the wave)
        vals = [twist(ring[(j - 624) % 624], ring[(j - 623) % 624], ring[(j - 227) % 624]) for j in range(g, want)]
        for j, v in zip(range(g, want), vals):
            ring[j % 624] = v
    else:  # one at a time (mt_ring_ahead)
        for j in range(g, want):
            ring[j % 624] = twist(ring[(j - 624) % 624], ring[(j - 623) % 624], ring[(j - 227) % 624])


def test_batched_ring_matches_mt19937():
    for seed in (5489, 1, 0xDEADBEEF):
        x = seed_words(seed)
        bg = np.random.MT19937()
        bg.state = {"bit_generator": "MT19937", "state": {"key": np.array(x, dtype=np.uint32), "pos": 624}}
        n_out = 624 + 64 * 40 + 17
        ref = [int(v) for v in bg.random_raw(n_out)]
        u = first_624(x)
        assert [temper(v) for v in u] == ref[:624]
        rb, rs = list(u), list(u)
        out_b, g = [], 624
        # the chain's refills: 64 ahead of a draw position that advances by a few per bounce
        n, rng = 624, np.random.default_rng(seed)
        while g < n_out:
            want = min(n + 64, n_out)
            if want > g:
                refill(rb, g, want, True)
                refill(rs, g, want, False)
                assert rb == rs
                out_b += [temper(rb[j % 624]) for j in range(g, want)]
                g = want
            n += int(rng.integers(1, 40))
        assert out_b == ref[624:]
