"""Register-renamed variants of the round-1 encoder.

Usage: python3 rename.py <isa.s> <out.elf> <next_free_vgpr> [old=new ...]

Renames single VGPRs (e.g. 86=94) inside k_encode_static<DIV_POW2>'s body only, sets that
kernel's .amdhsa_next_free_vgpr / .amdhsa_accum_offset, and assembles + links the file into a
code object.  The instruction stream is otherwise byte-identical, so comparing variants shows
whether WHICH registers the code touches (relative to the top of its allocation) decides the
failure.  Register tuples (v[a:b]) are left alone; the renamed registers must not appear in one.
"""
import re
import subprocess
import sys

LLVM = "/opt/rocm/lib/llvm/bin"
KERNEL = "_Z15k_encode_staticILi0EEv9ModelArgsPKhPKmjPhS4_PmPj"


def main(src, dst, nfree, pairs):
    lines = open(src).read().split("\n")
    ren = {int(a): int(b) for a, b in (p.split("=") for p in pairs)}
    start = next(i for i, l in enumerate(lines) if l.startswith(KERNEL + ":"))
    end = next(i for i in range(start, len(lines)) if lines[i].strip() == "s_endpgm")
    pat = re.compile(r"\bv(\d+)\b")
    for i in range(start, end + 1):
        line = lines[i]
        code = line.split(";")[0]
        for m in re.finditer(r"v\[(\d+):(\d+)\]", code):
            lo, hi = int(m.group(1)), int(m.group(2))
            if any(lo <= r <= hi for r in ren):
                raise SystemExit(f"renamed register inside a tuple: {line.strip()}")
        new = pat.sub(lambda m: "v%d" % ren.get(int(m.group(1)), int(m.group(1))), code)
        lines[i] = new + line[len(code):]
    kd = next(i for i, l in enumerate(lines) if l.strip() == f".amdhsa_kernel {KERNEL}")
    for i in range(kd, kd + 60):
        s = lines[i].strip()
        if s.startswith(".amdhsa_next_free_vgpr"):
            lines[i] = f"\t\t.amdhsa_next_free_vgpr {nfree}"
        elif s.startswith(".amdhsa_accum_offset"):
            lines[i] = f"\t\t.amdhsa_accum_offset {(nfree + 3) // 4 * 4}"
        elif s == ".end_amdhsa_kernel":
            break
    tmp = dst + ".s"
    open(tmp, "w").write("\n".join(lines))
    subprocess.run([f"{LLVM}/clang", "--target=amdgcn-amd-amdhsa", "-mcpu=gfx950", "-c", tmp,
                    "-o", dst + ".o"], check=True)
    subprocess.run([f"{LLVM}/ld.lld", "-shared", dst + ".o", "-o", dst], check=True)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]), sys.argv[4:])
