"""Does the adaptive (C4) decoder speed up with more waves per SIMD?  (VERDICT r04 next #2.)

The C4 decoder keeps a 255-node u16 tree per lane (32 KiB per wave), so LDS holds 5 waves per
CU (1.25 per SIMD).  The lever DESIGN.md §5.1 names is a smaller model per lane.  This probe
measures the lever with the decoder's own instruction stream: a 128-symbol adaptive model
(Zipf(1.2) over 128 symbols, the C4 rule otherwise) leaves nodes 129..255 at zero, so the
decoder can run with only the 128 rows of nodes 1..128 in LDS (RC_ADAPT_DEC_LDS=16384: reads
past the allocation return 0, writes there are dropped).  Same data, same code, decoded with
the full 32 KiB per wave and with 16 KiB per wave; both outputs checked against the input.

    python tools/adapt_occ_probe.py [n_chunks] [reps]   -> one JSON line
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import torch  # noqa: E402

import range_coder_rust_amd as rc  # noqa: E402
from range_coder_rust_amd import synth  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 1 << 20
    reps = int(sys.argv[2]) if len(sys.argv) > 2 else 3
    L = 16384
    ctx = rc.default_context(0)
    c, _, _ = synth.zipf_table(n=128)
    inv = synth.inverse_cdf(c)
    syms = torch.empty(n * L, dtype=torch.uint8, device="cuda")
    synth.fill(ctx, 0x5EED0005, inv, syms, L, n)
    m = rc.AdaptiveModel(128, 32, 57343, 256, ctx=ctx)
    cap = rc.slot_capacity(L, 8.0)
    so = torch.arange(n + 1, dtype=torch.int64, device="cuda") * L
    oo = torch.arange(n + 1, dtype=torch.int64, device="cuda") * cap
    out = torch.empty(n * cap, dtype=torch.uint8, device="cuda")
    dec = torch.empty_like(syms)
    ol, fl = rc.encode_batch(m, syms, so, out, oo)
    torch.cuda.synchronize()
    assert int(fl.abs().sum()) == 0
    res = {"workload": f"{n} x 16 KiB chunks, adaptive order-0 over 128 symbols (Zipf(1.2)), "
                       f"the C4 rule (increment 32, limit 57343, period 256)",
           "bytes_per_symbol": round(float(ol.sum()) / (n * L), 5)}
    for tag, lds in (("tree_32k", None), ("tree_16k", "16384"), ("tree_32k_again", None)):
        if lds is None:
            os.environ.pop("RC_ADAPT_DEC_LDS", None)
        else:
            os.environ["RC_ADAPT_DEC_LDS"] = lds
        ms = []
        for _ in range(reps):
            dec.zero_()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fd = rc.decode_batch(m, out, oo[:-1].contiguous(), ol, dec, so)
            e1.record()
            torch.cuda.synchronize()
            ms.append(e0.elapsed_time(e1))
            assert int(fd.abs().sum()) == 0 and torch.equal(dec, syms), tag
        best = min(ms)
        res[tag] = {"decode_ms": round(best, 3), "decode_gsym_s": round(n * L / best / 1e6, 2),
                    "all_ms": [round(x, 3) for x in ms], "bit_exact": True}
    os.environ.pop("RC_ADAPT_DEC_LDS", None)
    res["speedup_16k_over_32k"] = round(res["tree_32k"]["decode_ms"] / res["tree_16k"]["decode_ms"], 3)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
