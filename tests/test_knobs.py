"""Run-time switches are read once per context: no source of the library
reads the environment except rc_knobs_from_env, which rc_ctx_create alone calls; every switch
it reads is documented in include/range_coder.h.  (CPU: source text only.)"""
import os
import re

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "range_coder_rust_amd", "csrc")


def _sources():
    for f in sorted(os.listdir(CSRC)):
        if f.endswith((".hip", ".inc", ".h", ".cpp")):
            with open(os.path.join(CSRC, f)) as fh:
                yield f, fh.read()


def _function_body(text, name):
    i = text.index(name + "(")
    j = text.index("{", i)
    depth, k = 0, j
    while True:
        if text[k] == "{":
            depth += 1
        elif text[k] == "}":
            depth -= 1
            if depth == 0:
                return text[j:k + 1]
        k += 1


def test_getenv_only_in_rc_knobs_from_env():
    calls = []
    for f, text in _sources():
        for m in re.finditer(r"\bgetenv\s*\(", text):
            line = text[:m.start()].count("\n") + 1
            if not text[text.rfind("\n", 0, m.start()) + 1:m.start()].lstrip().startswith("//"):
                calls.append((f, line))
    assert calls and all(f == "rc_kernels.hip" for f, _ in calls), calls
    k = dict(_sources())["rc_kernels.hip"]
    body = _function_body(k, "RcKnobs rc_knobs_from_env")
    assert len(re.findall(r"\bgetenv\s*\(", body)) == len(calls)
    # called from rc_ctx_create and nowhere else
    users = [(f, m.start()) for f, text in _sources()
             for m in re.finditer(r"rc_knobs_from_env\(\)", text)]
    create = _function_body(k, "rc_status rc_ctx_create")
    assert "rc_knobs_from_env()" in create
    assert len(users) == 3, users  # the declaration, the definition, rc_ctx_create's call


def test_every_switch_is_documented_in_the_header():
    body = _function_body(dict(_sources())["rc_kernels.hip"], "RcKnobs rc_knobs_from_env")
    names = set(re.findall(r'str\("(RC_[A-Z_]+)"\)', body))
    assert names == {"RC_PRIO", "RC_DEC_PAIR", "RC_STREAM_SERVICE", "RC_STREAM_DMA",
                     "RC_STREAM_DIRECT", "RC_STREAM_BATCH_BYTES", "RC_HIST_HOT"}
    with open(os.path.join(ROOT, "include", "range_coder.h")) as f:
        h = f.read()
    env = h[h.index("/* Environment."):]
    env = env[:env.index("*/")]
    for n in names:
        assert n in env, n
