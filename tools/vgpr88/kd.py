"""Print the raw resource fields of every kernel descriptor (.kd) in gfx950 code objects.

Usage: python3 kd.py co_a.elf [co_b.elf ...]

The amdhsa kernel descriptor (64 B) holds compute_pgm_rsrc3 at byte 44, rsrc1 at 48 and rsrc2
at 52.  rsrc1[5:0] is the VGPR allocation in granules of 8 minus one (gfx90a+, unified register
file); rsrc3[5:0] is accum_offset / 4 - 1.  These are what the hardware allocates from, so they
are the numbers to compare, not the assembler's `.amdhsa_next_free_vgpr` text.
"""
import struct
import subprocess
import sys

READELF = "/opt/rocm/lib/llvm/bin/llvm-readelf"


def descriptors(path):
    out = subprocess.run([READELF, "-S", "-s", "-W", path], capture_output=True, text=True,
                         check=True).stdout
    data = open(path, "rb").read()
    secs = {}
    for line in out.splitlines():
        t = line.strip()
        if t.startswith("[") and "]" in t:
            try:
                idx = int(t[1:t.index("]")])
            except ValueError:
                continue
            parts = t[t.index("]") + 1:].split()
            if len(parts) >= 4:
                secs[idx] = (int(parts[2], 16), int(parts[3], 16))
    res = {}
    for line in out.splitlines():
        p = line.split()
        if len(p) >= 8 and p[7].endswith(".kd") and p[6].isdigit():
            addr, name = int(p[1], 16), p[7][:-3]
            sa, so = secs[int(p[6])]
            res[name] = data[so + addr - sa: so + addr - sa + 64]
    return res


def main(paths):
    for path in paths:
        print(path)
        for name, kd in sorted(descriptors(path).items()):
            rsrc3, rsrc1, rsrc2 = struct.unpack_from("<III", kd, 44)
            lds = struct.unpack_from("<I", kd, 0)[0]
            vg = ((rsrc1 & 63) + 1) * 8
            acc = ((rsrc3 & 63) + 1) * 4
            sg = ((rsrc1 >> 6) & 15)
            print(f"  {name[:48]:48s} rsrc1 {rsrc1:08x} rsrc2 {rsrc2:08x} rsrc3 {rsrc3:08x}"
                  f"  vgpr_alloc {vg:3d} accum_offset {acc:3d} sgpr_gran {sg} lds {lds}")


if __name__ == "__main__":
    main(sys.argv[1:])
