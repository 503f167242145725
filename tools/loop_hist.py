"""Instruction mix of a kernel's hot loop, from the built library (CPU only, no GPU).

Usage: python3 tools/loop_hist.py LIB KERNEL_SUBSTRING [SYMBOLS_PER_TRIP] [--ops]

Disassembles the kernel's code object (llvm-objdump, as tools/isa_check.py extracts it) and
takes the largest loop closed by a conditional backward branch: the decoders' 64-symbol body
loop (their rare paths sit out of line and return with unconditional branches, which are not
counted as loops).  Prints instruction counts by class and, given SYMBOLS_PER_TRIP, per symbol;
--ops adds the per-opcode histogram.
"""
import collections
import os
import re
import subprocess
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import isa_check  # noqa: E402

OBJDUMP = "/opt/rocm/lib/llvm/bin/llvm-objdump"


def kernel_text(lib, sub):
    import tempfile
    for co in isa_check.code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".elf") as f:
            f.write(co)
            f.flush()
            out = subprocess.run([OBJDUMP, "-d", "--mcpu=gfx950", f.name], capture_output=True,
                                 text=True).stdout
        for m in re.finditer(r"\n[0-9a-f]+ <(\S+)>:\n(.*?)(?=\n[0-9a-f]+ <|\Z)", out, re.S):
            if sub in m.group(1):
                return m.group(1), m.group(2)
    raise SystemExit(f"no kernel matching {sub!r} in {lib}")


def parse(text):
    ins = []
    for line in text.splitlines():
        m = re.match(r"\s+(\S.*?)\s*//\s*([0-9A-Fa-f]+):", line)
        if m:
            ins.append((int(m.group(2), 16), m.group(1)))
    return ins


def hot_loop(ins, min_steps=64):
    """The shortest loop closed by a conditional backward branch that holds at least min_steps
    symbol steps (v_ffbh_u32, one per step); else the longest such loop."""
    idx = {a: i for i, (a, _) in enumerate(ins)}
    loops = []
    for i, (a, t) in enumerate(ins):
        m = re.match(r"(s_cbranch_\w+)\s+(-?\d+)", t)
        if not m:
            continue
        v = int(m.group(2))
        v = v - 65536 if v > 32767 else v
        tgt = a + 4 + 4 * v
        if tgt <= a and tgt in idx:
            loops.append((idx[tgt], i))
    steps = [(j, i) for j, i in loops
             if sum(t.startswith("v_ffbh") for _, t in ins[j:i + 1]) >= min_steps]
    j, i = min(steps, key=lambda x: x[1] - x[0]) if steps else max(loops, key=lambda x: x[1] - x[0])
    return ins[j:i + 1]


def klass(op):
    for p, k in (("v_", "valu"), ("s_nop", "s_nop"), ("s_waitcnt", "s_waitcnt"), ("s_", "salu"),
                 ("ds_", "lds"), ("global_", "vmem"), ("buffer_", "vmem")):
        if op.startswith(p):
            return k
    return op


def main():
    lib, sub = sys.argv[1], sys.argv[2]
    per = int(sys.argv[3]) if len(sys.argv) > 3 and sys.argv[3].isdigit() else 0
    name, text = kernel_text(lib, sub)
    loop = hot_loop(parse(text))
    ops = collections.Counter(t.split()[0] for _, t in loop)
    cls = collections.Counter()
    for op, n in ops.items():
        cls[klass(op)] += n
    print(f"{name}: hot loop {len(loop)} instructions")
    for k, n in cls.most_common():
        print(f"  {k:10s} {n:6d}" + (f"  {n / per:7.2f} per symbol" if per else ""))
    if "--ops" in sys.argv:
        for op, n in ops.most_common():
            print(f"    {op:28s} {n:5d}" + (f"  {n / per:6.2f}" if per else ""))


if __name__ == "__main__":
    main()
