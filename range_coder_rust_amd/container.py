"""The chunked container "RCB1" (layout in include/range_coder.h).

The reference's stream holds neither its symbol count (examples/sample_impl.rs:113-120) nor
its model (decoder.rs:38); the container frames a batch of chunk streams with both, so

    blob = compress(data)          # data: uint8 HIP tensor -> container (uint8 HIP tensor)
    data == decompress(blob)

is a complete codec.  compress = GPU histogram + table (model_build) -> encode_batch ->
rc_container_pack; decompress = rc_container_info_parse -> model from the table ->
rc_container_offsets -> decode_batch, reading the payload in place.
"""
import ctypes
import math

import numpy as np

from . import _native as N
from .api import (AdaptiveModel, RangeCoderError, StaticModel, _check_dev, _ptr, _raise_for_flag,
                  _torch, decode_batch, default_context, encode_batch, slot_capacity)
from .model_build import build_model


class ContainerError(RangeCoderError):
    """A malformed or inconsistent container (RC_E_BAD_CONTAINER)."""


def pack(model, slots, slot_off, code_len, sym_off):
    """rc_container_pack: encoder slots -> a new container tensor (uint8, same device)."""
    torch = _torch()
    _check_dev(slots, "slots", (torch.uint8,))
    for name, t in (("slot_off", slot_off), ("code_len", code_len), ("sym_off", sym_off)):
        _check_dev(t, name, (torch.int64, torch.uint64))
    n = sym_off.numel() - 1
    ctx = model.ctx
    ctx.bind_stream()
    size = ctypes.c_uint64()
    rc = ctx._lib.rc_container_pack(ctx.handle, model.handle, _ptr(slots), _ptr(slot_off),
                                    _ptr(code_len), _ptr(sym_off), n, None, 0, ctypes.byref(size))
    if rc != N.RC_E_CAPACITY:
        N.check(rc, "rc_container_pack (size)")
    dst = torch.empty(size.value, dtype=torch.uint8, device=slots.device)
    N.check(ctx._lib.rc_container_pack(ctx.handle, model.handle, _ptr(slots), _ptr(slot_off),
                                       _ptr(code_len), _ptr(sym_off), n, _ptr(dst), dst.numel(),
                                       ctypes.byref(size)), "rc_container_pack")
    return dst


def info(container):
    """rc_container_info_parse of a container (tensor or bytes)."""
    if isinstance(container, (bytes, bytearray, memoryview)):
        head = bytes(container[:N.CONTAINER_HEADER_BYTES])
    else:
        head = bytes(container[:N.CONTAINER_HEADER_BYTES].cpu().numpy())
    inf = N.ContainerInfo()
    rc = N.load().rc_container_info_parse(ctypes.c_char_p(head), len(head), ctypes.byref(inf))
    if rc == N.RC_E_BAD_CONTAINER:
        raise ContainerError("not an RCB1 container header")
    N.check(rc, "rc_container_info_parse")
    return inf


def model_of(container, inf=None, ctx=None):
    """The container's model: a StaticModel from its c_freq table (cum by calc_cum) or an
    AdaptiveModel from its parameters."""
    inf = inf or info(container)
    ctx = ctx or default_context(container.device.index)
    if inf.kind == 1:
        return AdaptiveModel(inf.n_symbols, inf.increment, inf.limit, inf.period, ctx=ctx)
    tab = container[inf.table_off: inf.table_off + 4 * inf.n_symbols].cpu().numpy()
    c = tab.view(np.uint32).copy()
    if int(c.sum(dtype=np.uint64)) != inf.total_freq:
        raise ContainerError("table does not sum to the header's total_freq")
    try:
        return StaticModel(c, None, inf.total_freq, ctx=ctx)
    except ValueError as e:
        raise ContainerError(str(e)) from None


def offsets(container, inf=None, ctx=None):
    """rc_container_offsets: (code_off, code_len, sym_off) device tensors for decode_batch."""
    torch = _torch()
    _check_dev(container, "container", (torch.uint8,))
    inf = inf or info(container)
    if container.numel() < inf.container_bytes:
        raise ContainerError(f"container truncated: {container.numel()} of "
                             f"{inf.container_bytes} bytes")
    ctx = ctx or default_context(container.device.index)
    n = inf.n_chunks
    dev = container.device
    code_off = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    code_len = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    sym_off = torch.empty(n + 1, dtype=torch.int64, device=dev)
    ctx.bind_stream()
    rc = ctx._lib.rc_container_offsets(ctx.handle, _ptr(container), ctypes.byref(inf),
                                       _ptr(code_off), _ptr(code_len), _ptr(sym_off))
    if rc == N.RC_E_BAD_CONTAINER:
        raise ContainerError("container index inconsistent with its header")
    N.check(rc, "rc_container_offsets")
    return code_off[:n], code_len[:n], sym_off


def compress(data, chunk_size=65536, model=None, target_total=1 << 16, ctx=None):
    """uint8 HIP tensor -> RCB1 container (uint8 HIP tensor).  model None: built on the GPU
    from the data's histogram, scaled to target_total with every symbol encodable."""
    torch = _torch()
    _check_dev(data, "data", (torch.uint8,))
    ctx = ctx or default_context(data.device.index)
    n_sym = data.numel()
    n = (n_sym + chunk_size - 1) // chunk_size
    dev = data.device
    sym_off = torch.arange(n + 1, dtype=torch.int64, device=dev) * chunk_size
    sym_off[-1] = n_sym
    if model is None:
        model = build_model(data, sym_off, target_total=target_total, all_symbols=True, ctx=ctx)
    cap = slot_capacity(chunk_size, model.max_bits_per_symbol())
    slot_off = torch.arange(n + 1, dtype=torch.int64, device=dev) * cap
    slots = torch.empty(max(n * cap, 16), dtype=torch.uint8, device=dev)
    out_len, flags = encode_batch(model, data, sym_off, slots, slot_off)
    if n:
        bad = flags[flags != 0]
        if bad.numel():
            _raise_for_flag(int(bad[0].item()), "compress")
    return pack(model, slots, slot_off, out_len, sym_off)


def decompress(container, ctx=None):
    """RCB1 container (uint8 HIP tensor) -> the original uint8 tensor."""
    torch = _torch()
    _check_dev(container, "container", (torch.uint8,))
    ctx = ctx or default_context(container.device.index)
    inf = info(container)
    model = model_of(container, inf, ctx)
    code_off, code_len, sym_off = offsets(container, inf, ctx)
    out = torch.empty(max(inf.n_syms, 1), dtype=torch.uint8, device=container.device)
    flags = decode_batch(model, container, code_off, code_len, out, sym_off)
    if inf.n_chunks:
        bad = flags[flags != 0]
        if bad.numel():
            _raise_for_flag(int(bad[0].item()), "decompress")
    return out[:inf.n_syms]
