"""Helpers shared by the GPU parity tests: device upload and encode/decode through the C ABI
with ragged, optionally misaligned chunk layouts and sentinel checks around the slots."""
import numpy as np
import torch

import range_coder_rust_amd as rc


def dev(a, dtype=None):
    t = torch.from_numpy(np.ascontiguousarray(a))
    if dtype is not None:
        t = t.to(dtype)
    return t.to("cuda")


def cum_of(c):
    c = np.asarray(c, dtype=np.uint64)
    return np.concatenate([[0], np.cumsum(c)[:-1]]).astype(np.uint32)


def run_encode(model, chunks, caps, misalign=False, seed=0):
    """Encode with chunks at contiguous ragged offsets.  If misalign, prefix the arena with a
    random number of bytes so every chunk (and slot) starts at an arbitrary alignment."""
    rng = np.random.default_rng(seed)
    n = len(chunks)
    lens = np.array([len(c) for c in chunks], np.int64)
    base_s = int(rng.integers(0, 16)) if misalign else 0
    sym_off = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64) + base_s
    syms = np.concatenate([rng.integers(0, 256, base_s).astype(np.uint8)] +
                          [np.asarray(c, np.uint8) for c in chunks] + [np.zeros(1, np.uint8)])
    caps = np.asarray(caps, np.int64)
    base_o = int(rng.integers(0, 16)) if misalign else 0
    out_off = np.concatenate([[0], np.cumsum(caps)]).astype(np.int64) + base_o
    out = torch.full((int(out_off[-1]) + 64,), 0xEE, dtype=torch.uint8, device="cuda")
    out_len, flags = rc.encode_batch(model, dev(syms), dev(sym_off), out, dev(out_off))
    torch.cuda.synchronize()
    h = out.cpu().numpy()
    # nothing is written outside the slots (bytes past out_len inside a slot are unspecified)
    assert (h[:base_o] == 0xEE).all() and (h[out_off[-1]:] == 0xEE).all()
    return h, out_off, out_len.cpu().numpy(), flags.cpu().numpy()


def run_decode(model, codes, counts, misalign=False, seed=0, code_lens=None):
    rng = np.random.default_rng(seed)
    n = len(codes)
    clen = np.array([len(c) for c in codes], np.int64) if code_lens is None else code_lens
    gaps = rng.integers(0, 16, n) if misalign else np.zeros(n, np.int64)
    coff = np.zeros(n, np.int64)
    parts = []
    pos = 0
    for k, c in enumerate(codes):
        parts.append(rng.integers(0, 256, int(gaps[k])).astype(np.uint8))
        pos += int(gaps[k])
        coff[k] = pos
        parts.append(np.frombuffer(bytes(c), np.uint8))
        pos += len(c)
    parts.append(np.zeros(16, np.uint8))
    blob = np.concatenate(parts)
    counts = np.asarray(counts, np.int64)
    base = int(rng.integers(0, 16)) if misalign else 0
    sym_off = np.concatenate([[0], np.cumsum(counts)]).astype(np.int64) + base
    syms = torch.full((int(sym_off[-1]) + 16,), 0xEE, dtype=torch.uint8, device="cuda")
    flags = rc.decode_batch(model, dev(blob), dev(coff), dev(clen), syms, dev(sym_off))
    torch.cuda.synchronize()
    s = syms.cpu().numpy()
    return [s[sym_off[k]:sym_off[k + 1]] for k in range(n)], flags.cpu().numpy()

