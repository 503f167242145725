"""CPU tests of the RCB1 container: the library's header parser
(rc_container_info_parse, host code through the C ABI) on containers built by the oracle
restatement (oracle/container.py), and its rejection of malformed headers."""
import ctypes
import struct

import numpy as np
import pytest

from oracle import container as OC
from oracle import cpu
from range_coder_rust_amd import _native as N

SAMPLE = [2, 1, 1, 4, 1, 4, 2, 1, 0, 1, 5, 9, 8, 7, 6, 5]
C = [1, 5, 2, 0, 2, 2, 1, 1, 1, 1]
CUM = [0, 1, 6, 8, 8, 10, 12, 13, 14, 15]


def parse(blob):
    inf = N.ContainerInfo()
    rc = N.load().rc_container_info_parse(ctypes.c_char_p(bytes(blob)), len(blob),
                                          ctypes.byref(inf))
    return rc, inf


def test_oracle_container_of_the_sample():
    blob = OC.compress_static(C, CUM, 16, bytes(SAMPLE), 16)
    rc, inf = parse(blob)
    assert rc == N.RC_OK
    assert (inf.kind, inf.n_symbols, inf.total_freq, inf.n_chunks, inf.n_syms) == (0, 10, 16, 1, 16)
    assert inf.table_off == 64 and inf.index_off == 64 + 48 and inf.payload_off == 112 + 16
    assert inf.payload_bytes == 16 and inf.container_bytes == len(blob)
    # the payload is K1's 13-byte stream, zero padded
    assert blob[inf.payload_off:inf.payload_off + 13].hex() == "64475f8970365a2f83b20246c0"
    kind, ns, total, c, chunks = OC.parse(blob)
    assert c == C and chunks[0][0] == 16
    f, dec = cpu.decode(C, CUM, 16, chunks[0][1], chunks[0][0])
    assert f == 0 and list(dec) == SAMPLE


def test_ragged_chunks_layout():
    rng = np.random.default_rng(1)
    data = rng.integers(0, 10, 10000).astype(np.uint8)
    data[data == 3] = 4  # c[3] == 0
    blob = OC.compress_static(C, CUM, 16, data, 3000)
    rc, inf = parse(blob)
    assert rc == N.RC_OK and inf.n_chunks == 4 and inf.n_syms == 10000
    assert inf.container_bytes == len(blob) and inf.payload_bytes % 16 == 0
    _, _, _, _, chunks = OC.parse(blob)
    assert [k for k, _ in chunks] == [3000, 3000, 3000, 1000]


@pytest.mark.parametrize("field,value", [
    ("magic", b"RCB2"), ("version", 2), ("header", 32), ("kind", 2), ("n_symbols", 0),
    ("n_symbols", 257), ("payload", 17), ("short", None)])
def test_malformed_headers_rejected(field, value):
    blob = bytearray(OC.compress_static(C, CUM, 16, bytes(SAMPLE), 16))
    if field == "magic":
        blob[:4] = value
    elif field == "version":
        blob[4:8] = struct.pack("<I", value | (64 << 16))
    elif field == "header":
        blob[4:8] = struct.pack("<I", 1 | (value << 16))
    elif field == "kind":
        blob[8:12] = struct.pack("<I", value)
    elif field == "n_symbols":
        blob[12:16] = struct.pack("<I", value)
    elif field == "payload":
        blob[48:56] = struct.pack("<Q", value)
    elif field == "short":
        blob = blob[:40]
    rc, _ = parse(blob)
    assert rc == N.RC_E_BAD_CONTAINER
