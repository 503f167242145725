"""CPU restatement of the RCB1 container (TEST INFRASTRUCTURE ONLY; layout in
include/range_coder.h).  Builds container bytes from oracle encodings (oracle/cpu.py) so the
GPU container can be compared byte for byte.  The framing is not in the reference (its stream
has no length or model: examples/sample_impl.rs:113-120, decoder.rs:38); only the chunk
streams inside follow the reference (src/encoder.rs:24-46)."""
import struct

import numpy as np

from . import cpu

HEADER = 64


def pad16(v):
    return (v + 15) & ~15


def build(kind, n_symbols, chunks, codes, c=None, total=0, adaptive=(0, 0, 0)):
    """chunks: list of symbol byte strings; codes: their chunk streams."""
    inc, lim, per = adaptive if kind == 1 else (0, 0, 0)
    n = len(chunks)
    n_syms = sum(len(x) for x in chunks)
    payload = b"".join(bytes(cd) + b"\0" * (pad16(len(cd)) - len(cd)) for cd in codes)
    head = b"RCB1" + struct.pack("<IIIIIII", 1 | (HEADER << 16), kind, n_symbols,
                                 total if kind == 0 else 0, inc, lim, per)
    head += struct.pack("<QQQQ", n, n_syms, len(payload), 0)
    assert len(head) == HEADER
    table = b""
    if kind == 0:
        table = np.asarray(c, dtype="<u4").tobytes()
        table += b"\0" * (pad16(len(table)) - len(table))
    index = b"".join(struct.pack("<QQ", len(x), len(cd)) for x, cd in zip(chunks, codes))
    return head + table + index + payload


def compress_static(c, cum, total, data, chunk_size):
    chunks = [bytes(data[i:i + chunk_size]) for i in range(0, len(data), chunk_size)]
    codes = []
    for ch in chunks:
        f, b, _ = cpu.encode(c, cum, total, ch)
        assert f == 0
        codes.append(b)
    return build(0, len(c), chunks, codes, c=c, total=total)


def parse(blob):
    """-> (kind, n_symbols, total, c, [(symbols count, code bytes)])"""
    assert blob[:4] == b"RCB1"
    vh, kind, ns, total, inc, lim, per = struct.unpack_from("<IIIIIII", blob, 4)
    n, n_syms, pay, _ = struct.unpack_from("<QQQQ", blob, 32)
    off = HEADER
    c = None
    if kind == 0:
        c = list(struct.unpack_from(f"<{ns}I", blob, off))
        off += pad16(4 * ns)
    idx = [struct.unpack_from("<QQ", blob, off + 16 * k) for k in range(n)]
    off += 16 * n
    out = []
    for sc, ln in idx:
        out.append((sc, bytes(blob[off:off + ln])))
        off += pad16(ln)
    return kind, ns, total, c, out
