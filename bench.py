#!/usr/bin/env python3
"""Benchmark of the batched range coder hot path (BASELINE.json metric).

Headline, the same workload at every N (BASELINE.json configs[4]; at N = 1 it is configs[2]'s
encode+decode at full size): one fixed stream of 2^20 independent 64 KiB chunks, Zipf(1.2)
256-symbol static PModel (total 2^16), synthetic symbols generated in HBM, split into contiguous
shards over the N ranks (strong scaling).  One step = encode every chunk of the shard (reference:
Encoder::new + 65,536 x encode + finish, encoder.rs:14-46) then decode every chunk
(Decoder::new + 65,536 x decode, decoder.rs:14-54), all inputs resident in HBM.
value = symbols round-tripped / second over all ranks = 2^36 / max-over-ranks step time.

Chunks are independent streams (encoder.rs:48-55), so the shards need no data-path collective:
the process group (RCCL) carries only the barriers, the max-over-ranks of the timed region and
the all-ranks-bit-exact flag (range_coder_rust_amd/shard.py).  `bench.py --gpus N` launches its
N ranks itself (torch.distributed.run on 127.0.0.1, before any GPU call), or runs as one rank of
an external torchrun whose WORLD_SIZE must equal N.

Extras at every N: the uniform configs[1] load (2^20 chunks per GPU, c = 1, total 256; weak
scaling) and the adaptive configs[3] model (over 256 and over 128 symbols).  At N = 1 also: the
histogram / entropy report on the headline's buffers, the container and the host-resident
(PCIe) legs on the uniform leg's buffers, and a CPU baseline (the C oracle on the host cores,
rank 0, on a bounded sample of the headline's chunks).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
CTRL_DEVICE = "cuda"  # where the barrier / max-over-ranks tensors live (RCCL)
SEED = 0x5EED0001


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=None,
                   help="GPUs (ranks) of this node; default WORLD_SIZE or 1")
    p.add_argument("--steps", type=int, default=5)
    p.add_argument("--warmup", type=int, default=2)
    p.add_argument("--chunks", type=int, default=1 << 20,
                   help="uniform extra (configs[1], weak): chunks per GPU")
    p.add_argument("--global-chunks", type=int, default=1 << 20,
                   help="headline (configs[4], strong): chunks sharded over the ranks")
    p.add_argument("--chunk-bytes", type=int, default=65536)
    p.add_argument("--no-uniform", action="store_true", help="skip the uniform configs[1] leg")
    p.add_argument("--no-adaptive", action="store_true", help="skip the adaptive (C4) leg")
    p.add_argument("--no-model-build", action="store_true",
                   help="skip the histogram / entropy-report leg (on the Zipf inputs)")
    p.add_argument("--no-container", action="store_true",
                   help="skip the container pack / unpack leg (on the uniform leg's code)")
    p.add_argument("--no-host-stream", action="store_true",
                   help="skip the host-resident (PCIe) encode/decode leg")
    p.add_argument("--no-cpu-baseline", action="store_true")
    p.add_argument("--cpu-seconds", type=float, default=8.0, help="target CPU sample wall time")
    p.add_argument("--cpu-threads", type=int, default=0,
                   help="0 = every CPU this process may run on (affinity and cgroup quota)")
    p.add_argument("--traffic", default=os.path.join(ROOT, "profiles", "traffic.json"),
                   help="PMC-derived HBM bytes per launch (written by tools/pmc_traffic.py)")
    return p.parse_args()


def table(cfg):
    """The static model of cfg, or for "adaptive" / "adaptive128" the Zipf table its data is
    drawn from (over 256 / 128 symbols)."""
    from range_coder_rust_amd import synth
    if cfg == "uniform":
        return synth.uniform_table()
    return synth.zipf_table(n=128) if cfg == "adaptive128" else synth.zipf_table()


class Leg:
    """One configuration resident in HBM: inputs, code slots, decoded output."""

    def __init__(self, torch, rc, synth, ctx, cfg, n, L, first_chunk, bufs=None):
        c, cum, total = table(cfg)
        self.cfg, self.n, self.L = cfg, n, L
        if cfg.startswith("adaptive"):  # configs[3]: the C4 model over Zipf(1.2) data
            self.model = rc.AdaptiveModel(len(c), **rc.ADAPTIVE_DEFAULTS, ctx=ctx)
            cap = rc.slot_capacity(L, 6.0, slack=1.02)  # Zipf(1.2) codes at ~5.4 bits/symbol
        else:
            self.model = rc.StaticModel(c, cum, total, ctx=ctx)
            cap = rc.slot_capacity(L, 8.0, slack=1.02)  # >= the uniform model's 8 bits/symbol
        self.c, self.cum, self.total = c, cum, total
        dev = torch.device("cuda", ctx.device)
        self.cap = cap
        if bufs is None:
            bufs = Leg.alloc(torch, dev, n, L)
        if n * L > bufs["syms"].numel() or n * cap > bufs["out"].numel():
            raise ValueError("leg does not fit the shared arena")
        self.bufs = bufs
        self.syms, self.out = bufs["syms"][: n * L], bufs["out"][: n * cap]
        self.dec = bufs["dec"][: n * L]
        self.inv = synth.inverse_cdf(c)
        from range_coder_rust_amd import shard
        self.seed = shard.synth_seed(SEED, first_chunk)  # this rank's slice of one global stream
        synth.fill(ctx, self.seed, self.inv, self.syms, L, n)
        self.sym_off = torch.arange(n + 1, dtype=torch.int64, device=dev) * L
        self.out_off = torch.arange(n + 1, dtype=torch.int64, device=dev) * cap
        self.code_off = self.out_off[:-1].contiguous()
        self.out_len = torch.zeros(n, dtype=torch.int64, device=dev)
        self.fenc = torch.zeros(n, dtype=torch.int32, device=dev)
        self.fdec = torch.zeros(n, dtype=torch.int32, device=dev)
        self.rc = rc

    @staticmethod
    def alloc(torch, dev, n, L):
        """Symbols, code slots (at the uniform model's 8 bits/symbol) and decoded symbols for
        n chunks of L symbols; every leg takes prefixes of these."""
        from range_coder_rust_amd import api
        cap = api.slot_capacity(L, 8.0, slack=1.02)
        return dict(syms=torch.empty(n * L, dtype=torch.uint8, device=dev),
                    out=torch.empty(n * cap, dtype=torch.uint8, device=dev),
                    dec=torch.empty(n * L, dtype=torch.uint8, device=dev))

    def encode(self):
        self.rc.encode_batch(self.model, self.syms, self.sym_off, self.out, self.out_off,
                             self.out_len, self.fenc)

    def decode(self):
        self.rc.decode_batch(self.model, self.out, self.code_off, self.out_len, self.dec,
                             self.sym_off, self.fdec)


def equal_chunked(torch, a, b, step=1 << 30):
    """torch.equal without a full-size temporary (the tensors are 64 GiB each)."""
    if a.numel() != b.numel():
        return False
    for i in range(0, a.numel(), step):
        if not torch.equal(a[i:i + step], b[i:i + step]):
            return False
    return True


def lib_sha256(path):
    """sha256 of a built library (keys profiles/traffic.json entries to the build they measured)"""
    import hashlib
    h = hashlib.sha256()
    with open(path, "rb") as f:
        for blk in iter(lambda: f.read(1 << 20), b""):
            h.update(blk)
    return h.hexdigest()


def run_leg(torch, dist, leg, steps, warmup, world):
    """W untimed steps, then exactly K timed steps bracketed by barrier + synchronize."""
    for _ in range(warmup):
        leg.encode()
        leg.decode()
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True),
           torch.cuda.Event(enable_timing=True)) for _ in range(steps)]
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for e0, e1, e2 in ev:
        e0.record()
        leg.encode()
        e1.record()
        leg.decode()
        e2.record()
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t = time.perf_counter() - t0
    enc_ms = float(np.mean([a.elapsed_time(b) for a, b, _ in ev]))
    dec_ms = float(np.mean([b.elapsed_time(c) for _, b, c in ev]))
    from range_coder_rust_amd import shard
    t = shard.max_over_ranks(t, dist if world > 1 else None, device=CTRL_DEVICE)
    # correctness of the timed work: no chunk flagged, decode(encode(x)) == x
    ok = (int(leg.fenc.abs().sum()) == 0 and int(leg.fdec.abs().sum()) == 0
          and equal_chunked(torch, leg.dec, leg.syms))
    ok = shard.all_ranks_true(ok, dist if world > 1 else None, device=CTRL_DEVICE)
    code_bytes = int(leg.out_len.sum())
    return dict(t=t, enc_ms=enc_ms, dec_ms=dec_ms, ok=ok, code_bytes=code_bytes)


def model_build_leg(torch, rc, leg, code_bytes, reps=3):
    """SURVEY.md §8f rows 2 and 4 on the leg's inputs: GPU histogram (batch + per-chunk rows),
    its HBM roofline (reads 1 B/symbol, writes 1 KiB per chunk), the table it yields, and the
    entropy report: ideal code length of the leg's model against the coded bytes."""
    n, L = leg.n, leg.L
    _, ch = rc.histogram(leg.syms, leg.sym_off, per_chunk=True)  # warm-up
    ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
          for _ in range(reps)]
    hist = None
    for e0, e1 in ev:
        e0.record()
        hist, ch = rc.histogram(leg.syms, leg.sym_off, per_chunk=True)
        e1.record()
    torch.cuda.synchronize()
    ms = float(np.mean([a.elapsed_time(b) for a, b in ev]))
    alg = n * L + n * 256 * 4
    t0 = torch.cuda.Event(enable_timing=True)
    t1 = torch.cuda.Event(enable_timing=True)
    t0.record()
    bits = rc.ideal_bits(leg.model, ch)
    t1.record()
    torch.cuda.synchronize()
    counts = hist.cpu().numpy().astype(np.uint64)
    c, cum, total = rc.quantize_counts(counts, 1 << 16, all_symbols=True)
    ideal = float(bits.sum().item())
    return dict(
        histogram_ms=round(ms, 3), histogram_gbps=round(alg / ms / 1e6, 1),
        histogram_roofline_frac=round(alg / ms / 1e6 / HBM_PEAK_GBPS, 4),
        ideal_bits_ms=round(t0.elapsed_time(t1), 3),
        ideal_bits_per_symbol=round(ideal / (n * L), 5),
        coded_bits_per_symbol=round(code_bytes * 8 / (n * L), 5),
        coding_overhead_bits_per_symbol=round((code_bytes * 8 - ideal) / (n * L), 6),
        built_table_total=total, built_table_max_c=int(c.max()), built_table_min_c=int(c.min()))


def container_leg(torch, rc, leg):
    """SURVEY.md §8f row 1 on the leg's encoded slots: rc_container_pack (scans + the payload
    gather: reads the code, writes the container; HBM-bound) and rc_container_offsets (the
    decode side's index scan), then a decode straight from the container, checked."""
    t0, t1, t2 = (torch.cuda.Event(enable_timing=True) for _ in range(3))
    blob = rc.container.pack(leg.model, leg.out, leg.out_off, leg.out_len, leg.sym_off)  # warm
    del blob
    torch.cuda.synchronize()
    t0.record()
    blob = rc.container.pack(leg.model, leg.out, leg.out_off, leg.out_len, leg.sym_off)
    t1.record()
    inf = rc.container.info(blob)
    code_off, code_len, sym_off = rc.container.offsets(blob, inf)
    t2.record()
    torch.cuda.synchronize()
    pack_ms = t0.elapsed_time(t1)
    code = int(leg.out_len.sum())
    moved = code + int(inf.container_bytes)
    leg.dec.zero_()
    fl = rc.decode_batch(leg.model, blob, code_off, code_len, leg.dec, sym_off)
    ok = int(fl.abs().sum()) == 0 and equal_chunked(torch, leg.dec, leg.syms)
    del blob
    return dict(container_bytes=int(inf.container_bytes),
                framing_overhead=round(int(inf.container_bytes) / code - 1, 6),
                pack_ms=round(pack_ms, 3), pack_gbps=round(moved / pack_ms / 1e6, 1),
                pack_roofline_frac=round(moved / pack_ms / 1e6 / HBM_PEAK_GBPS, 4),
                offsets_ms=round(t1.elapsed_time(t2), 3), decode_from_container_ok=ok)


def host_stream_leg(torch, rc, leg, n_chunks):
    """host-resident chunks through rc_encode_host / rc_decode_host
    (pipelined H2D / kernel / D2H over 3 streams).  "pinned": every host buffer is pinned
    memory (torch pin_memory) — the pipeline's own rate; "pageable": fresh numpy buffers, which
    the call page-locks in place (first-touch + pinning cost included).  Rates are symbol bytes
    per second end to end (PCIe-inclusive); never the headline value."""
    L = leg.L
    n = min(n_chunks, leg.n)
    soff = np.arange(n + 1, dtype=np.uint64) * L
    ooff = np.arange(n + 1, dtype=np.uint64) * leg.cap
    res = {}
    for kind in ("pinned", "pageable"):
        if kind == "pinned":
            hs = torch.empty(n * L, dtype=torch.uint8, pin_memory=True)
            hs.copy_(leg.syms[: n * L])
            syms = hs.numpy()
            out = torch.empty(n * leg.cap, dtype=torch.uint8, pin_memory=True).numpy()
            dec = torch.empty(n * L, dtype=torch.uint8, pin_memory=True).numpy()
        else:
            syms = leg.syms[: n * L].cpu().numpy()
            out = dec = None
        times = []
        for rep in range(2 if kind == "pinned" else 1):
            t0 = time.perf_counter()
            out, ol, fl = rc.encode_host(leg.model, syms, soff, ooff, out=out)
            t1 = time.perf_counter()
            dec, fd = rc.decode_host(leg.model, out, ooff[:-1], ol, soff, out=dec)
            t2 = time.perf_counter()
            times.append((t1 - t0, t2 - t1))
        te, td = times[-1]
        ok = bool((fl == 0).all() and (fd == 0).all() and np.array_equal(dec, syms))
        res[kind] = dict(encode_gbps=round(n * L / te / 1e9, 2),
                         decode_gbps=round(n * L / td / 1e9, 2), round_trip_ok=ok)
        del out, dec, syms
    res["sample"] = f"{n} x {L // 1024} KiB chunks ({n * L / 2**30:.1f} GiB) host-resident"
    # the bound of this leg: plain pinned copies of 1 GiB each way on this box
    hb = torch.empty(1 << 30, dtype=torch.uint8, pin_memory=True)
    db = torch.empty(1 << 30, dtype=torch.uint8, device=leg.syms.device)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
    db.copy_(hb, non_blocking=True)
    ev[0].record()
    db.copy_(hb, non_blocking=True)
    ev[1].record()
    hb.copy_(db, non_blocking=True)
    ev[2].record()
    torch.cuda.synchronize()
    res["pcie_h2d_gbps"] = round((1 << 30) / ev[0].elapsed_time(ev[1]) / 1e6, 2)
    res["pcie_d2h_gbps"] = round((1 << 30) / ev[1].elapsed_time(ev[2]) / 1e6, 2)
    del hb, db
    return res


def host_cpus():
    """(nproc, usable): os.cpu_count(), and the CPUs this process may actually run on — its
    affinity mask, capped by a cgroup v2 CPU quota (a GPU box's share of a larger host)."""
    nproc = os.cpu_count() or 1
    try:
        usable = len(os.sched_getaffinity(0))
    except (AttributeError, OSError):
        usable = nproc
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            quota, period = f.read().split()[:2]
        if quota != "max":
            usable = min(usable, max(1, int(-(-int(quota) // int(period)))))
    except (OSError, ValueError):
        pass
    return nproc, usable


def cpu_baseline(torch, leg, seconds, threads):
    """The C oracle (a bit-exact restatement of the Rust reference; no rustc here) on the host,
    on bounded samples of the same chunks (copied from HBM), encode + decode, Gsymbols/s round
    trip: on every usable CPU (one chunk per task, as independent Encoders would run), and on
    one core."""
    from oracle import cpu
    L = leg.L

    def run(S, th, check):
        syms = leg.syms[: S * L].cpu().numpy()
        so = (np.arange(S + 1) * L).astype(np.uint64)
        oo = (np.arange(S + 1) * leg.cap).astype(np.uint64)
        t0 = time.perf_counter()
        out, ol, fl = cpu.encode_batch(leg.c, leg.cum, leg.total, syms, so, oo, th)
        t1 = time.perf_counter()
        dec, fd = cpu.decode_batch(leg.c, leg.cum, leg.total, out, oo[:-1], ol, so, th)
        t2 = time.perf_counter()
        assert (fl == 0).all() and (fd == 0).all() and (dec == syms).all()
        if check:  # the CPU stream equals the GPU stream byte for byte on the first chunks
            g = leg.out[: leg.cap * min(S, 8)].cpu().numpy()
            for k in range(min(S, 8)):
                assert bytes(g[k * leg.cap: k * leg.cap + int(ol[k])]) == \
                    bytes(out[k * leg.cap: k * leg.cap + int(ol[k])])
        return t1 - t0, t2 - t1

    nproc, usable = host_cpus()
    threads = threads or usable
    S0 = max(threads, 16)
    te, td = run(S0, threads, True)
    S = int(min(leg.n, max(S0, min(65536, S0 * seconds / max(te + td, 1e-6)))))
    S = max(threads, S // threads * threads)
    te, td = run(S, threads, False)
    n_sym = S * L
    # one core: a smaller sample (~1/4 of the time budget)
    te1, td1 = run(2, 1, False)
    S1 = int(max(2, min(256, 2 * seconds / 4 / max(te1 + td1, 1e-6))))
    te1, td1 = run(S1, 1, False)
    return dict(value=n_sym / (te + td) / 1e9, unit="Gsymbols/s", cores=threads, kind="port",
                nproc=nproc, usable_cpus=usable,
                sample=f"{S} of the {leg.n} 64 KiB chunks ({n_sym} symbols), encode+decode by "
                       f"the C oracle on {threads} host threads (nproc {nproc}, {usable} usable "
                       f"by this job): enc {n_sym / te / 1e9:.4f} Gsym/s, dec "
                       f"{n_sym / td / 1e9:.4f} Gsym/s",
                encode=n_sym / te / 1e9, decode=n_sym / td / 1e9,
                single_core=dict(value=S1 * L / (te1 + td1) / 1e9, encode=S1 * L / te1 / 1e9,
                                 decode=S1 * L / td1 / 1e9, sample=f"{S1} chunks, 1 thread"))


def resolve_world(args):
    """(world, rank, local_rank) of this process.  With --gpus N > 1 and no WORLD_SIZE in the
    environment, launch the N ranks (this process then only waits for them: it exits here)."""
    env_world = os.environ.get("WORLD_SIZE")
    if env_world is None:
        n = args.gpus or 1
        if n > 1:
            import torch  # device_count() does not initialise the GPU
            have = torch.cuda.device_count()
            if have < n and os.environ.get("RC_BENCH_ONE_DEVICE") != "1":
                sys.stderr.write(f"bench.py: --gpus {n} but {have} GPU(s) visible\n")
                sys.exit(2)
            from range_coder_rust_amd import shard
            sys.exit(shard.launch_ranks(os.path.abspath(__file__), sys.argv[1:], n))
        return 1, 0, 0
    world = int(env_world)
    if args.gpus is not None and args.gpus != world:
        sys.stderr.write(f"bench.py: --gpus {args.gpus} disagrees with WORLD_SIZE={world}\n")
        sys.exit(2)
    return world, int(os.environ.get("RANK", "0")), int(os.environ.get("LOCAL_RANK", "0"))


HEADLINE_MODEL = "Zipf(1.2) static (total 2^16)"


def plan(world, rank, global_chunks=1 << 20, chunks_per_gpu=1 << 20, L=65536, uniform=True):
    """What each rank runs.  The headline is ONE workload at every N (configs[4]; at N = 1 it is
    configs[2]'s encode+decode at full size): the 2^20 x 64 KiB Zipf(1.2) stream, split into
    contiguous shards over the ranks (strong scaling: the job's symbols are fixed, so a 1/2/4/8
    curve of `value` is a speed-up curve).  The uniform configs[1] load (chunks_per_gpu per rank,
    weak scaling) is an extra at every N, N = 1 included."""
    from range_coder_rust_amd import shard
    lo, hi = shard.shard_range(global_chunks, world, rank)
    workload = (f"configs[4]: {global_chunks} x {L // 1024} KiB chunks sharded over {world} "
                f"GPU(s), {HEADLINE_MODEL}, encode then decode, inputs resident in HBM")
    return dict(lo=lo, n=hi - lo, n_all=global_chunks, scaling="strong", workload=workload,
                weak_n=chunks_per_gpu if uniform else 0, weak_lo=rank * chunks_per_gpu)


def kernel_stats(n_sym, code_bytes, ms):
    """Gsym/s, algorithmic GB/s and HBM fraction of one kernel: encode reads the symbols and
    writes the code, decode reads the code and writes the symbols."""
    alg = n_sym + code_bytes
    return dict(ms=ms, gsym_s=n_sym / ms / 1e6, gbps=alg / ms / 1e6,
                frac=alg / ms / 1e6 / HBM_PEAK_GBPS, alg_bytes=alg)


def traffic_for(path, key):
    """(counted bytes per launch, note, HBM-side estimate) from tools/pmc_traffic.py's file, only
    when the entry was profiled on this exact librc_amd.so (keyed by its sha256).  Counted =
    the TCC->EA request bytes (Infinity-Cache hits included: no counter separates them on this
    stack); the estimate takes the read side at its first touches."""
    note = "no profile of this workload in " + os.path.relpath(path, ROOT)
    try:
        with open(path) as f:
            tr = json.load(f)
    except (OSError, ValueError):
        return None, note, None
    if key not in tr:
        return None, note, None
    from range_coder_rust_amd import _native
    e = tr[key]
    if e.get("lib_sha256") != lib_sha256(_native.LIB_PATH):
        return (None, f"stale: {e.get('round')} profiled another build of librc_amd.so; "
                      f"not reported", None)
    return (e["hbm_bytes_per_launch"],
            f"PMC TCC->EA request bytes, this build ({e.get('round')})",
            e.get("hbm_estimate_per_launch"))


def main():
    args = parse()
    world, rank, local = resolve_world(args)
    P = plan(world, rank, args.global_chunks, args.chunks, args.chunk_bytes,
             uniform=not args.no_uniform)
    import torch
    import torch.distributed as dist

    # RC_BENCH_ONE_DEVICE=1 (rehearsal of the N-rank path on a one-GPU box): every rank on
    # device 0, control messages over gloo
    global CTRL_DEVICE
    one_dev = os.environ.get("RC_BENCH_ONE_DEVICE") == "1"
    gpu = 0 if one_dev else local
    torch.cuda.set_device(gpu)
    if world > 1:
        if one_dev:
            dist.init_process_group("gloo")
            CTRL_DEVICE = "cpu"
        else:
            dist.init_process_group("nccl", device_id=torch.device("cuda", gpu))
    dd = dist if world > 1 else None

    import range_coder_rust_amd as rc
    from range_coder_rust_amd import shard, synth
    ctx = rc.default_context(gpu)

    L, n, lo, n_all = args.chunk_bytes, P["n"], P["lo"], P["n_all"]
    # one arena for every leg (each takes prefixes): the headline shard and the weak uniform load
    bufs = Leg.alloc(torch, torch.device("cuda", gpu), max(n, P["weak_n"]), L)
    leg = Leg(torch, rc, synth, ctx, "zipf", n, L, lo, bufs=bufs)
    res = run_leg(torch, dist, leg, args.steps, args.warmup, world)
    value = n_all * L * args.steps / res["t"] / 1e9

    kern = {"encode": kernel_stats(n * L, res["code_bytes"], res["enc_ms"]),
            "decode": kernel_stats(n * L, res["code_bytes"], res["dec_ms"])}
    dom = "decode" if res["dec_ms"] >= res["enc_ms"] else "encode"
    # roofline.traffic: PMC-measured HBM bytes of this exact library build only
    traffic, traffic_note, traffic_est = traffic_for(args.traffic, f"zipf:{n}:{L}:{dom}")
    achieved = kern[dom]["gbps"]
    roofline = dict(bound="hbm", achieved=round(achieved, 2), peak=HBM_PEAK_GBPS, unit="GB/s",
                    frac=round(achieved / HBM_PEAK_GBPS, 4), traffic=traffic,
                    traffic_source=traffic_note, traffic_hbm_estimate=traffic_est,
                    kernel=f"{dom} (Zipf(1.2), LUT 4)",
                    alg_bytes_per_launch=kern[dom]["alg_bytes"])
    # N > 1: achieved / peak above is one rank's kernel against one GPU; the aggregate is every
    # rank's algorithmic bytes over the slowest rank's kernel time against N GPUs' peak
    alg_all = shard.sum_over_ranks(kern[dom]["alg_bytes"], dd, device=CTRL_DEVICE)
    ms_max = shard.max_over_ranks(kern[dom]["ms"], dd, device=CTRL_DEVICE)
    roofline["scope"] = "per GPU (rank 0's kernel vs one GPU's peak)"
    roofline["aggregate"] = dict(achieved=round(alg_all / ms_max / 1e6, 2),
                                 peak=HBM_PEAK_GBPS * world,
                                 frac=round(alg_all / ms_max / 1e6 / (HBM_PEAK_GBPS * world), 4),
                                 n_gpus=world)

    extras = {}

    def io_legs(on):
        """The container and host-path legs (§8f rows 1 and 3) on a measured leg's buffers.  They
        decode through that leg's kernel again, so they run on the uniform leg when there is
        one: the headline kernel's rocprofv3 --stats average is then its own launches only."""
        if world == 1 and not args.no_container:
            extras["container"] = container_leg(torch, rc, on)
        if world == 1 and not args.no_host_stream:
            extras["host_stream"] = host_stream_leg(torch, rc, on, 131072)

    # the N = 1 legs on the headline's own buffers first: every later leg takes prefixes of the
    # same arena and overwrites the headline's symbols and code
    if world == 1 and not args.no_model_build:
        extras["model_build"] = model_build_leg(torch, rc, leg, res["code_bytes"])
    if not P["weak_n"]:
        io_legs(leg)
    if P["weak_n"]:  # configs[1]: the uniform model, 2^20 chunks on every rank
        wn = P["weak_n"]
        u = Leg(torch, rc, synth, ctx, "uniform", wn, L, P["weak_lo"], bufs=bufs)
        us = max(2, args.steps // 2)
        ur = run_leg(torch, dist, u, us, 1, world)
        ue = kernel_stats(wn * L, ur["code_bytes"], ur["enc_ms"])
        ud = kernel_stats(wn * L, ur["code_bytes"], ur["dec_ms"])
        utr, utr_note, utr_est = traffic_for(args.traffic, f"uniform:{wn}:{L}:decode")
        extras["uniform_weak"] = dict(
            workload=f"configs[1] on every rank: {wn} x {L // 1024} KiB chunks per GPU, "
                     f"uniform-256 static model (c = 1, total 256; weak scaling)",
            value=round(wn * world * L * us / ur["t"] / 1e9, 3),
            encode_gsym_s=round(ue["gsym_s"], 3), decode_gsym_s=round(ud["gsym_s"], 3),
            encode_ms=round(ue["ms"], 3), decode_ms=round(ud["ms"], 3),
            bytes_per_symbol=round(ur["code_bytes"] / (wn * L), 5),
            roofline_frac_encode=round(ue["frac"], 4), roofline_frac_decode=round(ud["frac"], 4),
            decode_traffic=utr, decode_traffic_source=utr_note,
            decode_traffic_hbm_estimate=utr_est,
            bit_exact_round_trip=ur["ok"])
        io_legs(u)
    if not args.no_adaptive and L % 16384 == 0:
        La = 16384
        na = n * (L // La)
        a = Leg(torch, rc, synth, ctx, "adaptive", na, La, lo * (L // La), bufs=bufs)
        ar = run_leg(torch, dist, a, max(2, args.steps // 2), 1, world)
        extras["adaptive_c4"] = dict(
            workload=f"configs[3]: {na} x 16 KiB chunks per GPU, adaptive order-0 "
                     f"(increment 32, limit 57343, period 256) over Zipf(1.2) data",
            value=round(n_all * L * max(2, args.steps // 2) / ar["t"] / 1e9, 3),
            encode_gsym_s=round(na * La / ar["enc_ms"] / 1e6, 3),
            decode_gsym_s=round(na * La / ar["dec_ms"] / 1e6, 3),
            encode_ms=round(ar["enc_ms"], 3), decode_ms=round(ar["dec_ms"], 3),
            bytes_per_symbol=round(ar["code_bytes"] / (na * La), 5),
            bit_exact_round_trip=ar["ok"])
        # the same model over a 128-symbol alphabet: its decoder's 127-node tree (16 KiB of
        # LDS per wave instead of 32) lets twice the waves share a CU
        a = Leg(torch, rc, synth, ctx, "adaptive128", na, La, lo * (L // La), bufs=bufs)
        ar8 = run_leg(torch, dist, a, max(2, args.steps // 2), 1, world)
        extras["adaptive_c4_128"] = dict(
            workload=f"configs[3] with a 128-symbol alphabet: {na} x 16 KiB chunks per GPU, "
                     f"Zipf(1.2) data over 128 symbols",
            encode_gsym_s=round(na * La / ar8["enc_ms"] / 1e6, 3),
            decode_gsym_s=round(na * La / ar8["dec_ms"] / 1e6, 3),
            decode_vs_256=round(ar["dec_ms"] / ar8["dec_ms"], 3),
            bytes_per_symbol=round(ar8["code_bytes"] / (na * La), 5),
            bit_exact_round_trip=ar8["ok"])

    cpu_b = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        if extras:
            # restore the headline inputs and code for the CPU baseline sample
            synth.fill(ctx, leg.seed, leg.inv, leg.syms, L, n)
            leg.encode()
            torch.cuda.synchronize()
        cpu_b = cpu_baseline(torch, leg, args.cpu_seconds, args.cpu_threads)

    def extra_ok(e):  # every correctness flag a leg reports (host_stream nests two)
        flags = [e.get("bit_exact_round_trip", True), e.get("decode_from_container_ok", True)]
        flags += [v.get("round_trip_ok", True) for v in e.values() if isinstance(v, dict)]
        return all(flags)

    ok_all = res["ok"] and all(extra_ok(e) for e in extras.values() if isinstance(e, dict))
    if rank == 0:
        line = {
            "metric": "Gsymbols/s encode+decode, 256-sym static model, 64KiB chunks, 1/2/4/8 GPU",
            "value": round(value, 3),
            "unit": "Gsymbols/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(res["t"] / args.steps * 1e3, 3),
            "higher_is_better": True,
            "scaling": P["scaling"],
            "vs_baseline": None,
            "dtype": "u64",
            "data": "synthetic",
            "config": {"workload": P["workload"],
                       "chunks_per_gpu": n, "chunks_total": n_all, "chunk_symbols": L,
                       "alphabet": 256,
                       "total_freq": int(leg.total), "parallelism": f"chunk-shard x{world}"},
            "roofline": roofline,
            "cpu_baseline": cpu_b,
            "encode_gsym_s": round(kern["encode"]["gsym_s"], 3),
            "decode_gsym_s": round(kern["decode"]["gsym_s"], 3),
            "encode_ms": round(res["enc_ms"], 3),
            "decode_ms": round(res["dec_ms"], 3),
            "roofline_frac_encode": round(kern["encode"]["frac"], 4),
            "bytes_per_symbol": round(res["code_bytes"] / (n * L), 5),
            "bit_exact_round_trip": res["ok"],
            "extras": extras,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    if not ok_all:
        sys.exit(3)


if __name__ == "__main__":
    main()
