"""A host model of the static decoder's code-ring schedule (test infrastructure).

k_decode_static (range_coder_rust_amd/csrc/rc_decode.inc) stages each lane's code stream
through a 64-B LDS ring: 64-B load bursts, committed 32 B at a time at phase boundaries and on
demand (dec_sync), with ring checks every DEC_CHECK_SPAN symbols.  This module replays that
schedule (positions only, no data) for one chunk, given each symbol's settled bytes split into
no_carry_expansion bytes k and range_reduction_expansion bytes m (range_coder.rs:83-89), and
reports the two ways the ring can go wrong:

* under-run: a symbol reads a code byte at or past the staged end (fillb).  The ring slot then
  holds bytes from 64 B earlier: wrong symbols, no flag;
* over-write: a commit overwrites bytes not yet consumed.

The constants mirror rc_static.h / rc_decode.inc for small (SM) models; `need_rare` is the
rare path's DEC_NEED_SM (12 before round 4, 3 * DEC_CHECK_SPAN = 24 after) and `need_span` the
in-phase checks' DEC_NEED_SPAN (24; scratch guard builds lower it to provoke under-runs).  `Replay` steps
one symbol at a time (so a search can steer a stream against it); `replay` runs a whole chunk.
"""
import copy

DEC_RING = 16        # dwords
DEC_PF = 2           # 16-B blocks per commit
DEC_LD = 4           # 16-B blocks per load burst
DEC_CHECK_SPAN = 8
NEED_HEAD = 12       # head and tail: a check after every symbol for the next 4
NEED_SPAN = 3 * DEC_CHECK_SPAN


class Replay:
    """The ring schedule of one chunk of n symbols whose code starts at `align` mod 64 and whose
    output needs `head` single symbols before it is 64-B aligned (rc_decode.inc:575-637)."""

    def __init__(self, n, align=0, head=0, need_rare=NEED_SPAN, need_span=NEED_SPAN):
        self.n = n
        self.need_span = need_span
        self.head = min(head, n)
        self.nph = (n - self.head) >> 4      # 16-symbol phases after the head
        self.need_rare = need_rare
        self.fillb = 0
        self.pend_ok = 0
        self.bpos = 8 * (align + 8)          # Decoder::new primes 8 bytes
        self.under = []   # symbol indices that read unstaged bytes
        self.over = []    # symbols after which a commit overwrote unread bytes
        self.i = 0        # symbols decoded so far
        self.min_slack = 1 << 30  # fewest staged-but-unread bytes left after a symbol's reads
        for _ in range(DEC_RING // (4 * DEC_PF)):
            if not self.pend_ok:
                self._issue()
            self._commit()
        while self.fillb - self.bpos < 8 * NEED_HEAD:
            if not self.pend_ok:
                self._issue()
            self._commit()
        if not self.pend_ok:
            self._issue()
        self._check(NEED_HEAD)
        if self.head == 0:
            self._check(need_span)

    def clone(self):
        return copy.deepcopy(self)

    def unread(self):
        """Staged bytes not yet consumed."""
        return (self.fillb - self.bpos) // 8

    def span_offset(self):
        """The next symbol's offset in its ring-check span (None in the head and tail, where
        every symbol is followed by a check)."""
        j = self.i - self.head
        if j < 0 or j >= 16 * self.nph:
            return None
        return j % DEC_CHECK_SPAN

    def _issue(self):
        self.pend_ok = DEC_LD // DEC_PF

    def _commit(self):
        if self.fillb - self.bpos > 32 * DEC_RING - 128 * DEC_PF:
            self.over.append(self.i - 1)
        self.fillb += 128 * DEC_PF
        self.pend_ok -= 1

    def _sync(self, need):
        while self.fillb - self.bpos < 8 * need:
            if not self.pend_ok:
                self._issue()
            self._commit()

    def _check(self, need):
        if self.fillb - self.bpos < 8 * need:
            self._sync(need)

    def _phase(self):
        if self.pend_ok and self.fillb - self.bpos <= 32 * DEC_RING - 128 * DEC_PF:
            self._commit()
        if not self.pend_ok:
            self._issue()

    def step(self, k, m):
        """One symbol that settles k no-carry bytes and m range-reduction bytes, then the
        checks the kernel runs after it."""
        i = self.i
        if self.bpos + 8 * k > self.fillb:
            self.under.append(i)
        self.bpos += 8 * k
        if m:
            self._sync(m + self.need_rare)
            for _ in range(m):
                if self.bpos + 8 > self.fillb:
                    self.under.append(i)
                self.bpos += 8
        self.min_slack = min(self.min_slack, (self.fillb - self.bpos) // 8)
        self.i = i + 1
        j = self.i - self.head     # symbols of the body decoded so far
        if i < self.head:
            self._check(NEED_HEAD)
            if self.i == self.head:
                self._check(self.need_span)
        elif j <= 16 * self.nph:
            if j % 16 == 0:
                self._phase()
                self._check(self.need_span)
            elif j % DEC_CHECK_SPAN == 0:
                self._check(self.need_span)
        else:
            self._check(NEED_HEAD)


def replay(km, align=0, head=0, need_rare=NEED_SPAN, need_span=NEED_SPAN):
    """Replay the decoder's ring schedule over one chunk.  km: [(k, m)] per symbol; align: the
    code stream's address mod 64; head: symbols decoded singly before the output is 64-B
    aligned.  Returns (under-run symbol indices, over-write symbol indices)."""
    g = Replay(len(km), align, head, need_rare, need_span)
    for k, m in km:
        g.step(k, m)
    return g.under, g.over


M64 = (1 << 64) - 1


def settle(c, cum, total, syms):
    """[(k, m)] per symbol of an encoder run: the bytes no_carry_expansion (range_coder.rs:110-116)
    and range_reduction_expansion (:126-135) settle in param_update (:53-92), from a u64
    restatement of the coder (the decoder's state follows the encoder's exactly)."""
    low, rng = 0, M64
    out = []
    for s in syms:
        r = rng // total
        rng = r * int(c[s])
        low = low + r * int(cum[s])
        k = 0
        while (low ^ (low + rng)) < 1 << 56:
            low, rng, k = (low << 8) & M64, (rng << 8) & M64, k + 1
        m = 0
        while rng < 1 << 48:
            rng = (~low & M64) & ((1 << 48) - 1)
            low, rng, m = (low << 8) & M64, (rng << 8) & M64, m + 1
        out.append((k, m))
    return out
