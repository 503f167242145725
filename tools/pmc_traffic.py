"""Turn a tools/profile.sh run into the committed profile evidence.

    python tools/pmc_traffic.py gpurun_out/prof_r02 --tag r02

Writes, under profiles/<tag>/:
  kernel_stats.csv  the rocprofv3 --stats summary of the default bench command
  bench.json        the bench line of that same run
  pmc.json          per-launch counters of the encode / decode kernels, and their byte sums
  pmc_calib.json    the same counters over tools/pmc_calib's known byte counts, per shape
and merges the headline key into profiles/traffic.json, which bench.py reads for
roofline.traffic.

Byte sums (all per launch):
  guide   2 x FETCH_SIZE + WRITE_SIZE (KiB): MI355X_MICROARCH.md's prescription for wide streaming
          reads; FETCH_SIZE's gfx950 expression tallies a 128-B read request as 64 B
  req     TCC->EA requests by size: 32 RDREQ_32B + 64 RDREQ_64B + 128 RDREQ_128B reads,
          32 (WRREQ - WRREQ_64B) + 64 WRREQ_64B writes (= WRITE_SIZE)
  dram    the DRAM-bound 32-B units: 32 RDREQ_DRAM_32B + 32 WRREQ_WRITE_DRAM_32B
Infinity Cache hits are fabric requests too: none of these separates them from HBM.
"""
import argparse
import csv
import glob
import json
import os
import re
import shutil

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KERNELS = {"encode": "k_encode_static", "decode": "k_decode_static"}
CAL_BYTES = (1 << 18) * 65536


def rows(d):
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            yield from csv.DictReader(f)


def per_kernel(dirs, match):
    """{key: {counter: mean per dispatch}} with key = match(kernel name) (None: skip)."""
    acc = {}
    for d in dirs:
        for r in rows(d):
            key = match(r["Kernel_Name"])
            if key is None:
                continue
            a = acc.setdefault(key, {}).setdefault(r["Counter_Name"], {})
            a[r["Dispatch_Id"]] = a.get(r["Dispatch_Id"], 0.0) + float(r["Counter_Value"])
    return {k: {c: sum(v.values()) / len(v) for c, v in cs.items()} for k, cs in acc.items()}


def coder_key(name):
    for dom, kn in KERNELS.items():
        if kn in name:
            return dom
    return None


def calib_key(name):
    m = re.search(r"k_calib<(\d+), (true|false)>", name)
    if m:
        return f"{'write' if m.group(2) == 'true' else 'read'} {16 * int(m.group(1))} B/lane"
    m = re.search(r"k_calib_coal<(true|false)>", name)
    if m:
        return f"{'write' if m.group(1) == 'true' else 'read'} coalesced"
    return None


def sums(cs):
    """byte sums of one kernel's counters (keys absent when a pass is missing)"""
    g = lambda n: cs.get(n, cs.get(n + "_sum"))
    out = {}
    if g("FETCH_SIZE") is not None and g("WRITE_SIZE") is not None:
        out["guide_read"] = 2 * g("FETCH_SIZE") * 1024
        out["guide_write"] = g("WRITE_SIZE") * 1024
    if None not in (g("TCC_EA0_RDREQ_32B"), g("TCC_EA0_RDREQ_64B"), g("TCC_EA0_RDREQ_128B")):
        out["req_read"] = (32 * g("TCC_EA0_RDREQ_32B") + 64 * g("TCC_EA0_RDREQ_64B") +
                           128 * g("TCC_EA0_RDREQ_128B"))
    if None not in (g("TCC_EA0_WRREQ"), g("TCC_EA0_WRREQ_64B")):
        out["req_write"] = 32 * (g("TCC_EA0_WRREQ") - g("TCC_EA0_WRREQ_64B")) + \
            64 * g("TCC_EA0_WRREQ_64B")
    if g("TCC_EA0_RDREQ_DRAM_32B") is not None:
        out["dram_read"] = 32 * g("TCC_EA0_RDREQ_DRAM_32B")
    if g("TCC_EA0_WRREQ_WRITE_DRAM_32B") is not None:
        out["dram_write"] = 32 * g("TCC_EA0_WRREQ_WRITE_DRAM_32B")
    return out


def main():
    p = argparse.ArgumentParser()
    p.add_argument("run", help="gpurun_out/prof_<tag> directory")
    p.add_argument("--tag", required=True)
    p.add_argument("--config", default="zipf")
    p.add_argument("--chunks", type=int, default=1 << 20)
    p.add_argument("--chunk-bytes", type=int, default=65536)
    a = p.parse_args()
    out = os.path.join(ROOT, "profiles", a.tag)
    os.makedirs(out, exist_ok=True)
    stats = glob.glob(os.path.join(a.run, "trace", "**", "*kernel_stats.csv"), recursive=True)
    bench = None
    if stats:  # (profile.sh's trace pass; SKIP_TRACE runs have none)
        shutil.copy(stats[0], os.path.join(out, "kernel_stats.csv"))
        with open(os.path.join(a.run, "bench.json")) as f:
            line = [l for l in f if l.startswith("{")][-1]
        with open(os.path.join(out, "bench.json"), "w") as f:
            f.write(line)
        bench = json.loads(line)

    pmc_dirs = sorted(glob.glob(os.path.join(a.run, "pmc*"))) + [os.path.join(a.run, "sq")]
    cal_dirs = sorted(glob.glob(os.path.join(a.run, "cal*")))
    pmc = per_kernel([d for d in pmc_dirs if os.path.isdir(d)], coder_key)
    cal = per_kernel(cal_dirs, calib_key)

    calib = {}
    for shape, cs in sorted(cal.items()):
        kind = shape.split()[0]
        e = {"counters": cs, "bytes": sums(cs)}
        e["true_over_counted"] = {k: round(CAL_BYTES / v, 4) for k, v in e["bytes"].items()
                                  if k.endswith(kind) and v > 0}
        calib[shape] = e
    with open(os.path.join(out, f"pmc_calib_{a.config}.json"), "w") as f:
        json.dump({"bytes_per_launch": CAL_BYTES, "shapes": calib}, f, indent=1, sort_keys=True)

    # the library the counters ran on (profile.sh records its sha256 on the box); bench.py
    # reports roofline.traffic only for that build
    with open(os.path.join(a.run, "lib.sha256")) as f:
        lib_sha = f.read().split()[0]
    n_sym = a.chunks * a.chunk_bytes
    # algorithmic bytes of the counted workload (profile.sh's plain kbench.py run of it)
    with open(os.path.join(a.run, "kbench.json")) as f:
        kb = json.loads([l for l in f if l.startswith("{")][-1])
    assert kb["config"] == a.config and kb["chunks"] == a.chunks, (kb, a.config, a.chunks)
    alg = kb["alg_bytes"]
    tpath = os.path.join(ROOT, "profiles", "traffic.json")
    traffic = json.load(open(tpath)) if os.path.exists(tpath) else {}
    for dom, cs in pmc.items():
        b = sums(cs)
        cs["bytes"] = b
        hbm = b["req_read"] + b["req_write"]
        cs["hbm_bytes_per_launch"] = hbm
        cs["hbm_bytes_per_symbol"] = hbm / n_sym
        cs["traffic_over_algorithmic"] = hbm / alg
        if "SQ_INSTS_VALU" in cs:
            cs["valu_per_wave_symbol"] = cs["SQ_INSTS_VALU"] / (n_sym / 64)
        # HBM-side estimate: the counted reads include Infinity-Cache hits of
        # the half-line refetch, which no counter on this stack separates; every stream byte is
        # first touched once, so HBM reads ~ the algorithmic read side (symbols for encode,
        # code for decode) and writes are the counted writes
        alg_read = n_sym if dom == "encode" else alg - n_sym
        est = alg_read + b["req_write"]
        cs["hbm_estimate_per_launch"] = est
        traffic[f"{a.config}:{a.chunks}:{a.chunk_bytes}:{dom}"] = {
            "hbm_bytes_per_launch": int(hbm), "round": a.tag, "lib_sha256": lib_sha,
            "counted_over_algorithmic": round(hbm / alg, 4),
            "hbm_estimate_per_launch": int(est),
            "estimate_over_algorithmic": round(est / alg, 4),
            "estimate": "algorithmic read bytes (first touches) + counted writes; the counted "
                        "reads beyond them are half-line refetches that the Infinity Cache "
                        "serves (DESIGN.md §6.2)",
            "bytes": {k: int(v) for k, v in b.items()},
            "correction": "TCC->EA read requests by size (32/64/128 B) + write requests by size "
                          "(= WRITE_SIZE); FETCH_SIZE alone tallies 128-B reads at 64 B"}
    with open(os.path.join(out, f"pmc_{a.config}.json"), "w") as f:
        json.dump(pmc, f, indent=1, sort_keys=True)
    with open(tpath, "w") as f:
        json.dump(traffic, f, indent=1, sort_keys=True)
    for shape, e in calib.items():
        print(f"calib {shape:22s} true/counted {e['true_over_counted']}")
    for dom, cs in pmc.items():
        print(f"{dom}: {cs['hbm_bytes_per_symbol']:.3f} B/sym, {cs['traffic_over_algorithmic']:.3f} "
              f"x algorithmic; bytes {json.dumps({k: round(v / 1e9, 2) for k, v in cs['bytes'].items()})} GB")
    if bench:
        print("bench:", bench["value"], bench["unit"], "roofline", bench["roofline"])


if __name__ == "__main__":
    main()
