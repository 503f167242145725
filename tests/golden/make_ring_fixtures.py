"""Generates tests/golden/ring_fixtures.json (committed).  Run from the repo root:

    python tests/golden/make_ring_fixtures.py

Directed streams for the static decoder's code ring (rc_decode.inc):
a small model (total 2^16) whose symbols 1..255 have c = 1, so one of them narrows the range by
2^16 and settles 2-3 bytes; after a range_reduction_expansion (range_coder.rs:126-135) such
symbols can settle up to 3 bytes each for the rest of an 8-symbol ring-check span, while the
rare path of the round-3 decoder staged only 12 bytes after it.

The streams are steered against tests/ring_sim.py's replay of the decoder's ring schedule: for
each 8-symbol span the search tries short symbol sequences (a few symbols that drain the ring,
then a symbol whose step ends in a range_reduction_expansion at a chosen span offset, then the
symbols that settle the most bytes) and keeps one that under-runs the round-3 schedule (rare
need 12) if it finds one.  The coder state comes from a u64 restatement of param_update
(range_coder.rs:53-92) checked byte for byte against the C oracle below.  Every chunk records
where the round-3 schedule under-ran; the round-4 schedule (need 3 * DEC_CHECK_SPAN = 24) must
under-run and over-write nowhere.  Code streams sit at several alignments mod 64 (the decoder's
load bursts start on 64-B boundaries) and the decoded output at offset 0 mod 64 (no head).
"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

from oracle import cpu  # noqa: E402
import ring_sim  # noqa: E402

M64 = (1 << 64) - 1
TOP8 = 1 << 56
TOP16 = 1 << 48
HERE = os.path.dirname(os.path.abspath(__file__))
TRIALS = 12
TOTAL = 65536
C = [TOTAL - 255] + [1] * 255
CUM = [0] + [TOTAL - 255 + i for i in range(255)]


def step(low, rng, s):
    """param_update (range_coder.rs:53-92) for symbol s: (low, range, k no-carry bytes, m rare
    bytes)."""
    r = rng // TOTAL
    rng = r * C[s]
    low = low + r * CUM[s]
    assert low <= M64
    k = 0
    while (low ^ (low + rng)) < TOP8:
        low = (low << 8) & M64
        rng = (rng << 8) & M64
        k += 1
    m = 0
    while rng < TOP16:
        rng = (~low & M64) & (TOP16 - 1)
        low = (low << 8) & M64
        rng = (rng << 8) & M64
        m += 1
    return low, rng, k, m


# ring schedules replayed, as (rare-path need, span need): round 3 and round 4
SCHEDULES = {"r3": (12, ring_sim.NEED_SPAN), "r4": (ring_sim.NEED_SPAN, ring_sim.NEED_SPAN)}


class Stream:
    """Coder state plus the ring schedules of SCHEDULES."""

    def __init__(self, n, align):
        self.low, self.rng = 0, M64
        self.syms, self.km = [], []
        self.rings = [ring_sim.Replay(n, align, 0, *q) for q in SCHEDULES.values()]

    def clone(self):
        t = Stream.__new__(Stream)
        t.low, t.rng = self.low, self.rng
        t.syms, t.km = list(self.syms), list(self.km)
        t.rings = [g.clone() for g in self.rings]
        return t

    def push(self, s):
        self.low, self.rng, k, m = step(self.low, self.rng, s)
        self.syms.append(s)
        self.km.append((k, m))
        for g in self.rings:
            g.step(k, m)
        return k, m


U64 = np.uint64
C_V = np.array(C, np.uint64)
CUM_V = np.array(CUM, np.uint64)


def vstep(low, rng):
    """step() for all 256 symbols at once (numpy u64, wrapping like the reference's u64):
    (low, range, k, m) arrays."""
    r = U64(rng // TOTAL)
    R = r * C_V
    L = U64(low) + r * CUM_V
    k = np.zeros(256, np.int64)
    m = np.zeros(256, np.int64)
    for _ in range(8):
        sh = (L ^ (L + R)) < U64(TOP8)
        k += sh
        L = np.where(sh, L << U64(8), L)
        R = np.where(sh, R << U64(8), R)
    for _ in range(8):
        sh = R < U64(TOP16)
        m += sh
        R2 = (~L) & U64(TOP16 - 1)
        L = np.where(sh, L << U64(8), L)
        R = np.where(sh, R2 << U64(8), R)
    return L, R, k, m


def most_bytes(st, rs):
    """The symbol that settles the most bytes from this state, preferring one that leaves
    range < 2^56 (so the next c = 1 symbol settles 3 bytes); ties at random."""
    _, R, k, m = vstep(st.low, st.rng)
    score = 4 * (k + m) + ((R < U64(TOP8)) & (m == 0))
    best = np.flatnonzero(score == score.max())
    return int(rs.choice(best))


def rare_now(st):
    _, _, _, m = vstep(st.low, st.rng)
    return int(np.argmax(m)) if m.max() > 0 else None


def trial(st, rs, left):
    """One candidate continuation: drain d symbols, a symbol whose step ends in a
    range_reduction_expansion (looking one symbol ahead for it), then the most bytes until the
    span after it ends.  Returns the advanced stream or None."""
    t = st.clone()
    for g in t.rings:
        g.min_slack = 1 << 30
    d = int(rs.integers(0, 12))
    for _ in range(min(d, left)):
        t.push(most_bytes(t, rs) if rs.random() < 0.7 else 0)
    if len(t.syms) - len(st.syms) >= left - 1:
        return None
    s = rare_now(t)
    if s is None:  # one symbol ahead: a first symbol after which some symbol is rare
        for s1 in rs.permutation(256)[:24]:
            low, rng, _, _ = step(t.low, t.rng, int(s1))
            _, _, _, m2 = vstep(low, rng)
            if m2.max() > 0:
                t.push(int(s1))
                s = int(np.argmax(m2))
                break
        if s is None:
            return None
    t.push(s)
    while (t.rings[0].span_offset() or 0) != 0 and len(t.syms) - len(st.syms) < left:
        t.push(most_bytes(t, rs))
    return t


def chunk(seed, n, align):
    """A stream steered to the tightest ring the round-3 schedule (need 12) allows after its
    rare events: of TRIALS continuations, the one whose bytes come closest to the staged end."""
    rs = np.random.default_rng(seed)
    st = Stream(n, align)
    while len(st.syms) < n:
        left = n - len(st.syms)
        best = None
        for _ in range(TRIALS):
            t = trial(st, rs, left)
            if t is not None and (best is None or t.rings[0].min_slack < best.rings[0].min_slack):
                best = t
        if best is not None:
            st = best
        else:  # move on: a few symbols of the usual mix
            for _ in range(min(int(rs.integers(1, 9)), left)):
                st.push(0 if rs.random() < 0.5 else int(rs.integers(1, 256)))
    return st


def main():
    n = 512
    aligns = [0, 1, 5, 8, 13, 17, 31, 33, 47, 63]
    chunks = []
    tot = {q: 0 for q in SCHEDULES}
    slack = {q: 1 << 30 for q in SCHEDULES}
    offsets = set()
    for ci, a in enumerate(aligns * 2):
        st = chunk(1000 + ci, n, a)
        syms, km = st.syms[:n], st.km[:n]
        f, code, L = cpu.encode(C, CUM, TOTAL, syms)
        assert f == 0 and L == 8 + sum(k + m for k, m in km)
        rec = dict(align=a, symbols=syms, encoded_hex=code.hex(),
                   rare_at=[i for i, (k, m) in enumerate(km) if m])
        offsets.update(i % ring_sim.DEC_CHECK_SPAN for i in rec["rare_at"])
        for (name, q), g in zip(SCHEDULES.items(), st.rings):
            u, o = ring_sim.replay(km, a, 0, *q)
            assert (u, o) == (g.under, g.over) and not o
            rec["underruns_" + name] = u
            rec["min_slack_" + name] = g.min_slack
            tot[name] += len(u)
            slack[name] = min(slack[name], g.min_slack)
        assert not rec["underruns_r4"]
        chunks.append(rec)
        print(f"chunk {ci}: align {a}, {len(code)} B, rare events {len(rec['rare_at'])}, "
              f"under-runs {[len(rec['underruns_' + q]) for q in SCHEDULES]}, "
              f"min slack {[g.min_slack for g in st.rings]}")
    assert tot["r4"] == 0
    out = dict(c=C, cum=CUM, total=TOTAL, n=n, schedules=SCHEDULES, chunks=chunks)
    with open(os.path.join(HERE, "ring_fixtures.json"), "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("under-runs by schedule:", tot, "min slack:", slack,
          "rare span offsets:", sorted(offsets))


if __name__ == "__main__":
    main()
