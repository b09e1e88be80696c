"""The cross-workgroup hand-offs (attention split merge, attention.h attn_publish/attn_merge; bgemm split-K,
bgemm.h) use relaxed agent-scope atomics plus an explicit `s_waitcnt vmcnt(0)`, not release/acquire.
Their correctness rests on what gfx950 code generation does with them, so this test pins that in the
generated ISA (CPU only: hipcc cross-compiles ops.hip device-only to assembly):

  * every published partial is a write-through store (`global_store_* ... sc1`): it reaches the
    device-coherent level before the arrival add, whatever XCD the last arriver runs on;
  * the arrival add (`global_atomic_add`) is preceded by `s_waitcnt vmcnt(0)` in the same function: the
    storing wave has drained its publishes before one lane signals;
  * every partial the last arriver reads back is an `sc1` buffer load (L1 bypassed, served by the
    coherent level), never a plain cached load.

If a compiler or ROCm upgrade changes any of these, the hand-offs must move to release/acquire
(__ATOMIC_RELEASE on the counter add, an agent-scope acquire fence in the last arriver).
"""
import os
import re
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SRC = os.path.join(ROOT, "simplellminference_amd", "csrc", "ops.hip")


@pytest.fixture(scope="module")
def asm(tmp_path_factory):
    out = tmp_path_factory.mktemp("isa") / "ops.s"
    inc = ["-I" + os.path.join(ROOT, "include", d) for d in ("", "base", "memory", "op", "model", "kernel")]
    cmd = ["hipcc", "-O3", "-std=c++17", "--offload-arch=gfx950", "--cuda-device-only", "-S", *inc, SRC,
           "-o", str(out)]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        pytest.fail(f"device-only compile failed:\n{r.stderr[-2000:]}")
    text = out.read_text()
    funcs = {}
    for m in re.finditer(r"^(_Z\S+):[^\n]*\n(.*?)(?=^\s*\.Lfunc_end)", text, re.S | re.M):
        funcs[m.group(1)] = m.group(2)
    return funcs


def _bodies(funcs, needle):
    found = {k: v for k, v in funcs.items() if needle in k}
    assert found, f"no kernel matching {needle}"
    return found


def _check_handoff(body, name):
    lines = [ln.strip() for ln in body.splitlines()]
    stores_sc1 = [ln for ln in lines if ln.startswith("global_store") and ln.endswith("sc1")]
    assert stores_sc1, f"{name}: no write-through (sc1) publish store"
    adds = [i for i, ln in enumerate(lines) if ln.startswith("global_atomic_add")]
    assert adds, f"{name}: no arrival add"
    for i in adds:
        before = lines[max(0, i - 40):i]
        assert any(ln.startswith("s_waitcnt") and "vmcnt(0)" in ln for ln in before), \
            f"{name}: arrival add without a preceding vmcnt(0) drain"
    loads = [ln for ln in lines if ln.startswith("buffer_load")]
    assert loads, f"{name}: no buffer loads of the partials"
    bad = [ln for ln in loads if "sc1" not in ln]
    assert not bad, f"{name}: partial read back without sc1: {bad[:3]}"


def test_attention_split_merge_handoff_isa(asm):
    bodies = _bodies(asm, "attn_partial_kernelI6__half")
    for name, body in bodies.items():
        _check_handoff(body, name)


def test_bgemm_splitk_handoff_isa(asm):
    bodies = _bodies(asm, "bgemm_kernel")
    for name, body in bodies.items():
        _check_handoff(body, name)
