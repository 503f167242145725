"""The Rust FFI block INTEGRATION.md gives maintainers (`src/gpu/ffi.rs`) against the C ABI it
binds (include/range_coder.h).  There is no rustc in this image, so the block is never compiled
here (VERDICT r03 missing #3); this test checks it as text instead: every `extern "C"` function
exists in the header with the same parameter count and C-compatible parameter and return types,
every header entry point is bound, the `#[repr(C)]` structs list the header's fields in its order
and with its widths, and the constants carry the header's values."""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "range_coder.h")
DOC = os.path.join(ROOT, "INTEGRATION.md")


def _strip_c_comments(s):
    s = re.sub(r"/\*.*?\*/", " ", s, flags=re.S)
    return re.sub(r"//[^\n]*", " ", s)


def header_functions():
    src = _strip_c_comments(open(HEADER).read())
    out = {}
    for m in re.finditer(r"(?:^|\n)\s*((?:const\s+)?\w+\s*\*?)\s*(rc_\w+)\s*\(([^)]*)\)\s*;", src):
        ret, name, args = m.group(1).strip(), m.group(2), m.group(3).strip()
        params = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
        out[name] = (ret, params)
    return out


def rust_block():
    """The ```rust block holding the extern "C" declarations (src/gpu/ffi.rs)."""
    text = open(DOC).read()
    blocks = [b for b in re.findall(r"```rust\n(.*?)```", text, re.S) if 'extern "C"' in b]
    assert len(blocks) == 1, "expected one rust block with the extern declarations"
    return blocks[0]


def rust_functions():
    blk = rust_block()
    ext = re.search(r'extern "C" \{(.*?)\n\}', blk, re.S).group(1)
    ext = re.sub(r"//[^\n]*", " ", ext)
    out = {}
    for m in re.finditer(r"pub fn (rc_\w+)\((.*?)\)\s*(?:->\s*([^;]+))?;", ext, re.S):
        name, args, ret = m.group(1), m.group(2), (m.group(3) or "()").strip()
        params = [a.strip() for a in " ".join(args.split()).split(",") if a.strip()]
        out[name] = (ret, [p.split(":", 1)[1].strip() for p in params])
    return out


SCALAR = {"int": "c_int", "rc_status": "c_int", "uint32_t": "u32", "uint64_t": "u64",
          "size_t": "usize", "uint8_t": "u8", "char": "c_char", "void": "c_void", "double": "f64",
          "rc_ctx": "RcCtx", "rc_model": "RcModel", "rc_stream_state": "RcStreamState",
          "rc_container_info": "RcContainerInfo"}


def c_to_rust(ctype):
    """The Rust spelling of a C parameter or return type (without its name)."""
    t = " ".join(ctype.replace("*", " * ").split())
    toks = t.split()
    # strip a trailing parameter name
    if toks and toks[-1] not in ("*", "const") and toks[-1] not in SCALAR and len(toks) > 1:
        toks = toks[:-1]
    # C reads pointer declarators right to left: "const T * const *" = *const *const T
    base_const = toks[0] == "const"
    if base_const:
        toks = toks[1:]
    base = SCALAR[toks[0]]
    rest = toks[1:]
    out = base
    pending_const = base_const
    i = 0
    while i < len(rest):
        assert rest[i] == "*", ctype
        const_ptr = i + 1 < len(rest) and rest[i + 1] == "const"
        out = ("*const " if pending_const else "*mut ") + out
        pending_const = const_ptr
        i += 2 if const_ptr else 1
    return out


def test_every_header_entry_point_is_bound():
    h, r = header_functions(), rust_functions()
    assert len(h) >= 28
    missing = sorted(set(h) - set(r))
    extra = sorted(set(r) - set(h))
    assert not extra, extra
    assert not missing, missing


def test_bound_signatures_match_the_header():
    h, r = header_functions(), rust_functions()
    for name, (rret, rparams) in r.items():
        cret, cparams = h[name]
        assert len(rparams) == len(cparams), (name, rparams, cparams)
        want_ret = c_to_rust(cret)
        assert rret == want_ret, (name, rret, want_ret)
        for rp, cp in zip(rparams, cparams):
            assert rp == c_to_rust(cp), (name, rp, cp, c_to_rust(cp))


def _c_struct(name):
    src = _strip_c_comments(open(HEADER).read())
    body = re.search(r"typedef struct %s \{(.*?)\} %s;" % (name, name), src, re.S).group(1)
    fields = []
    for decl in body.split(";"):
        decl = " ".join(decl.split())
        if not decl:
            continue
        typ, names = decl.split(" ", 1)
        for n in names.split(","):
            fields.append((n.strip(), SCALAR[typ]))
    return fields


def _rust_struct(name):
    blk = re.sub(r"//[^\n]*", " ", rust_block())
    body = re.search(r"pub struct %s \{(.*?)\}" % name, blk, re.S).group(1)
    return [(m.group(1), m.group(2)) for m in re.finditer(r"pub (\w+): (\w+)", body)]


def test_repr_c_structs_match_the_header():
    for c_name, r_name in (("rc_stream_state", "RcStreamState"),
                           ("rc_container_info", "RcContainerInfo")):
        assert _rust_struct(r_name) == _c_struct(c_name), (c_name, _rust_struct(r_name),
                                                           _c_struct(c_name))


def test_rust_constants_match_the_header():
    src = open(HEADER).read()
    consts = {m.group(1): int(m.group(2), 0) for m in
              re.finditer(r"#define (RC_\w+)\s+\(?(-?(?:0x[0-9a-fA-F]+|\d+))u?\b", src)}
    blk = rust_block()
    seen = 0
    for m in re.finditer(r"pub const (RC_\w+): \w+ = (-?\d+);", blk):
        name, v = m.group(1), int(m.group(2))
        if name in consts:
            assert consts[name] == v, (name, v, consts[name])
            seen += 1
    assert seen >= 10
