"""The ctypes mirrors in _lib.py lay out every C-ABI struct exactly as include/diffattn.h
does: gcc compiles a probe that prints sizeof / offsetof of each field, and each ctypes
Structure must agree field by field (an appended ABI field, e.g. ABI 5's rope_freqs /
q_rot, that one side misses would shift everything after it).  CPU only."""
import ctypes
import os
import shutil
import subprocess
import tempfile

import pytest

from differential_transformer_replication_amd import _lib

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

STRUCTS = {
    "dta_tensor": _lib.DtaTensor,
    "dta_attn_fwd_args": _lib.AttnFwdArgs,
    "dta_attn_bwd_args": _lib.AttnBwdArgs,
    "dta_ln_args": _lib.LnArgs,
    "dta_rope_args": _lib.RopeArgs,
    "dta_attn_decode_args": _lib.DecodeArgs,
    "dta_swiglu_args": _lib.SwigluArgs,
}


@pytest.mark.skipif(shutil.which("gcc") is None, reason="no gcc")
def test_ctypes_structs_match_the_header():
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "diffattn.h"', "int main(void) {"]
    for cname, py in STRUCTS.items():
        lines.append(f'  printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f in py._fields_:
            lines.append(f'  printf("{cname} {f[0]} %zu\\n", offsetof({cname}, {f[0]}));')
    lines += ["  return 0;", "}"]
    with tempfile.TemporaryDirectory() as d:
        src = os.path.join(d, "probe.c")
        exe = os.path.join(d, "probe")
        with open(src, "w") as fh:
            fh.write("\n".join(lines))
        subprocess.run(["gcc", "-std=c11", "-I", os.path.join(ROOT, "include"), src, "-o", exe], check=True)
        out = subprocess.run([exe], check=True, capture_output=True, text=True).stdout
    got = {}
    for ln in out.splitlines():
        s, f, v = ln.split()
        got[(s, f)] = int(v)
    bad = []
    for cname, py in STRUCTS.items():
        if got[(cname, "sizeof")] != ctypes.sizeof(py):
            bad.append((cname, "sizeof", got[(cname, "sizeof")], ctypes.sizeof(py)))
        for f in py._fields_:
            off = getattr(py, f[0]).offset
            if got[(cname, f[0])] != off:
                bad.append((cname, f[0], got[(cname, f[0])], off))
    assert not bad, bad
