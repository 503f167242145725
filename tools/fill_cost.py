"""In-context issue cost of VALU instruction classes in the static coders.

    python tools/fill_cost.py build            # CPU: variants/librc_amd_fill<op>.so
    python tools/fill_cost.py run OUT          # GPU: bench legs per variant, ROUNDS interleaved
    python tools/fill_cost.py report OUT/fill_cost.json [profiles/r04/fill_cost.json]

Each variant adds RC_FILL = 2 fillers of one instruction class (RC_FILL_OP, rc_common.h) to
every symbol step of k_encode_static and k_decode_static; the fillers depend only on each other.
The kernels are bound by VALU issue at 2^20 chunks, so the added time per
wave-symbol, divided by 2, is what one such instruction costs the SIMD inside the real loop:
    cycles = (t_variant - t_base) * f_clk * SIMDs / (2 * wave-symbols)
with wave-symbols = 2^36 / 64 over 1024 SIMDs, and f_clk from profiles/r03/pmc_bound.json.
"""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
OPS = {0: "v_add_u32", 1: "v_lshrrev_b32", 2: "v_lshlrev_b64", 3: "v_mad_u64_u32",
       4: "v_mad_u32_u24", 5: "v_cmp_gt_u64_e64", 6: "v_alignbit_b32", 7: "v_perm_b32",
       8: "v_lshl_add_u64", 9: "v_cvt_f32_u32", 11: "v_lshl_add_u32", 12: "v_ffbh_u32",
       13: "v_lshlrev_b32", 16: "v_lshrrev_b64",
       # round 5: the non-VALU classes (rc_common.h): scalar ALU, a compare + conditional branch,
       # the compare alone, and one LDS read whose result a VALU add waits for
       20: "s_add_u32", 21: "s_cmp+s_cbranch", 22: "s_cmp_eq_u32", 23: "ds_read_b32+v_add",
       24: "v_cmp vcc+v_cndmask vcc", 25: "v_cmp+v_cndmask sgpr"}
ONLY = ("rc_decode_pow2.hip", "rc_encode.hip")


def lib(op):
    return os.path.join(ROOT, "variants", f"librc_amd_fill{op}.so")


def build(ops):
    import __graft_entry__ as g
    for op in ops:
        # (FILL_FLAGS: extra defines, to match the build the fillers are priced against)
        g.build_variant(lib(op), ["-DRC_DEV_ONLY", "-DRC_FILL=2", f"-DRC_FILL_OP={op}"] +
                        os.environ.get("FILL_FLAGS", "").split(), only=ONLY)


def run(out, ops, rounds):
    os.makedirs(out, exist_ok=True)
    args = ["--config", os.environ.get("FILL_CONFIG", "uniform"), "--steps", "3", "--warmup", "1"]
    res = {}
    for r in range(rounds):
        for op in ["base"] + list(ops):
            env = dict(os.environ)
            if op != "base":
                env["RC_LIB_PATH"] = lib(op)
            p = subprocess.run([sys.executable, "tools/kbench.py"] + args, cwd=ROOT, env=env,
                               capture_output=True, text=True, timeout=300)
            if p.returncode != 0:
                sys.stderr.write(p.stderr[-2000:])
                raise SystemExit(f"bench failed for {op}")
            d = json.loads(p.stdout.strip().splitlines()[-1])
            e = d
            row = res.setdefault(str(op), {"encode_ms": [], "decode_ms": []})
            row["encode_ms"].append(e["encode_ms"])
            row["decode_ms"].append(e["decode_ms"])
            print(op, OPS.get(op, "-") if op != "base" else "", e["encode_ms"], e["decode_ms"],
                  flush=True)
    with open(os.path.join(out, "fill_cost.json"), "w") as f:
        json.dump(res, f, indent=1)


def report(path, f_enc=1.93e9, f_dec=1.98e9):
    """Cycles per instruction of each class: (t - t_base) x f_clk / (2 fillers x 2^20 wave-symbols
    per SIMD).  Clocks: profiles/r03/pmc_bound.json (GRBM_GUI_ACTIVE over the kernel time)."""
    d = json.load(open(path))
    mean = {k: (sum(v["encode_ms"]) / len(v["encode_ms"]), sum(v["decode_ms"]) / len(v["decode_ms"]))
            for k, v in d.items()}
    be, bd = mean["base"]
    ws = 2 ** 36 / 64 / 1024  # wave-symbols per SIMD at 2^20 x 64 KiB
    out = {"base_ms": {"encode": round(be, 3), "decode": round(bd, 3)},
           "clock_ghz": {"encode": f_enc / 1e9, "decode": f_dec / 1e9}, "cycles": {}}
    for k, (e, dd) in sorted(mean.items(), key=lambda x: x[0]):
        if k == "base":
            continue
        ce = (e - be) * 1e-3 * f_enc / (2 * ws)
        cd = (dd - bd) * 1e-3 * f_dec / (2 * ws)
        out["cycles"][OPS[int(k)]] = {"encode": round(ce, 2), "decode": round(cd, 2)}
        print(f"{OPS[int(k)]:18s} encode {ce:5.2f}  decode {cd:5.2f}")
    return out


if __name__ == "__main__":
    if sys.argv[1] == "report":
        res = report(sys.argv[2])
        if len(sys.argv) > 3:
            with open(sys.argv[3], "w") as f:
                json.dump(res, f, indent=1)
        raise SystemExit(0)
    ops = [int(x) for x in os.environ.get("OPS", ",".join(map(str, OPS))).split(",")]
    if sys.argv[1] == "build":
        build(ops)
    else:
        run(sys.argv[2], ops, int(os.environ.get("ROUNDS", "2")))
