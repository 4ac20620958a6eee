"""The C-ABI library loads and exports exactly what include/mof.h declares
(no compute calls: runs without a GPU)."""
import ctypes
import os
import re

import pytest

import mofhip
from mofhip import _lib as L

HEADER = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include", "mof.h")


def header_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return set(re.findall(r"\b(mof_[a-z_0-9]+)\s*\(", src))


def test_header_matches_binding_table():
    assert header_symbols() == set(L.EXPORTS)


def test_library_exports_every_symbol():
    lib = L.lib()
    for name in L.EXPORTS:
        assert hasattr(lib, name), name


def test_library_is_gfx950_code_object():
    data = open(L.LIB_PATH, "rb").read()
    assert b"gfx950" in data


def test_version_and_error_path():
    assert "gfx950" in mofhip.version()
    h = ctypes.c_void_p()
    # NULL inputs are rejected before any device work
    rc = L.lib().mof_mesh_create(None, None, None, None, 3, 1, 0, 0, ctypes.byref(h))
    assert rc == L.MOF_E_ARG
    assert b"NULL" in L.lib().mof_last_error()
    with pytest.raises(L.MofError):
        L.check(rc)


def test_struct_layouts():
    # mirror of the C structs in include/mof.h (x86-64 SysV layout)
    assert ctypes.sizeof(L.MofOpts) == 56
    assert ctypes.sizeof(L.MofStats) == 136
    assert ctypes.sizeof(L.MofMeshInfo) == 64


def test_struct_offsets_match_header(tmp_path):
    """Compile a probe against include/mof.h and compare every field offset."""
    import subprocess
    import shutil
    if shutil.which("gcc") is None:
        pytest.skip("gcc not available")
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "mof.h"', 'int main(void){']
    for cname, pyt in (("mof_opts", L.MofOpts), ("mof_stats", L.MofStats),
                       ("mof_mesh_info", L.MofMeshInfo)):
        lines.append('printf("%s %%zu\\n", sizeof(%s));' % (cname, cname))
        for f, _ in pyt._fields_:
            lines.append('printf("%s.%s %%zu\\n", offsetof(%s, %s));' % (cname, f, cname, f))
    lines.append("return 0;}")
    src = tmp_path / "probe.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "probe"
    subprocess.check_call(["gcc", "-I", os.path.dirname(HEADER), str(src), "-o", str(exe)])
    out = dict(l.split() for l in subprocess.check_output([str(exe)]).decode().splitlines())
    for cname, pyt in (("mof_opts", L.MofOpts), ("mof_stats", L.MofStats),
                       ("mof_mesh_info", L.MofMeshInfo)):
        assert int(out[cname]) == ctypes.sizeof(pyt)
        for f, _ in pyt._fields_:
            assert int(out["%s.%s" % (cname, f)]) == getattr(pyt, f).offset, (cname, f)
