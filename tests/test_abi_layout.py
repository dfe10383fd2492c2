"""The ctypes mirrors of include/arx.h's structs (audiorenderingv2_amd/_lib.py) have the C layout:
every field's offset and each struct's size, as gcc compiles the header on this host (no GPU, no
libarx needed).  A field added to the header but not to the mirror, or in another order, fails here."""
import ctypes as C
import os
import shutil
import subprocess

import pytest

from audiorenderingv2_amd._lib import ArxAppConfig, ArxConfig, ArxStats

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
MIRRORS = {"arx_config": ArxConfig, "arx_stats": ArxStats, "arx_app_config": ArxAppConfig}


@pytest.mark.skipif(shutil.which("gcc") is None, reason="needs gcc")
def test_ctypes_mirrors_match_the_header(tmp_path):
    lines = ["#include <stdio.h>", "#include <stddef.h>", '#include "arx.h"', "int main(void) {"]
    for cname, py in MIRRORS.items():
        lines.append(f'  printf("{cname} sizeof %zu\\n", sizeof({cname}));')
        for f, _ in py._fields_:
            lines.append(f'  printf("{cname} {f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["  return 0;", "}"]
    src, exe = tmp_path / "layout.c", tmp_path / "layout"
    src.write_text("\n".join(lines) + "\n")
    subprocess.run(["gcc", "-std=c11", "-I", os.path.join(REPO, "include"), str(src), "-o", str(exe)], check=True)
    got = {}
    for ln in subprocess.run([str(exe)], check=True, capture_output=True, text=True).stdout.splitlines():
        cname, field, v = ln.split()
        got[(cname, field)] = int(v)
    for cname, py in MIRRORS.items():
        assert got[(cname, "sizeof")] == C.sizeof(py), cname
        for f, _ in py._fields_:
            assert got[(cname, f)] == getattr(py, f).offset, (cname, f)
