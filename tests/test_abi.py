"""CPU-side checks of the drop-in boundary: libskv.so builds for gfx950, exports every symbol
include/skv.h declares, and refuses to run without a GPU (no silent CPU fallback)."""
import ctypes as C
import os
import re

import pytest

from skv import _abi
from skv import api

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_header_declares_exactly_the_bound_symbols():
    hdr = open(os.path.join(ROOT, "include", "skv.h")).read()
    declared = sorted(set(re.findall(r"\b(skv_[a-z_]+)\s*\(", hdr)))
    assert declared == sorted(_abi.EXPORTED_SYMBOLS)


def test_library_exports_every_symbol():
    api.build()
    assert api.exported_symbols_present() == _abi.EXPORTED_SYMBOLS
    assert api.load().skv_abi_version() == 9


def test_struct_layouts_match_header():
    assert C.sizeof(_abi.SkvRunDesc) == 80
    assert C.sizeof(_abi.SkvStream) == 32
    assert C.sizeof(_abi.SkvResult) == 64


def test_timings_layout_matches_header(tmp_path):
    """skv_timings as the C compiler lays it out (include/skv.h) == the ctypes mirror (_abi.py)."""
    import subprocess

    src = tmp_path / "t.c"
    src.write_text('#include <stdio.h>\n#include <stddef.h>\n#include "skv.h"\n'
                   'int main(void) { printf("%zu %zu %zu\\n", sizeof(skv_timings), '
                   'offsetof(skv_timings, span_parse), offsetof(skv_timings, wal_stage)); return 0; }\n')
    exe = tmp_path / "t"
    inc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "include")
    subprocess.check_call(["gcc", "-I", inc, str(src), "-o", str(exe)])
    size, off_span, off_wal = map(int, subprocess.check_output([str(exe)]).split())
    assert C.sizeof(_abi.SkvTimings) == size
    assert _abi.SkvTimings.span_parse.offset == off_span
    assert _abi.SkvTimings.wal_stage.offset == off_wal


def test_code_object_targets_gfx950():
    api.build()
    data = open(api.LIB_PATH, "rb").read()
    assert b"gfx950" in data


@pytest.mark.skipif(os.path.exists("/dev/kfd") and os.access("/dev/kfd", os.R_OK), reason="GPU present")
def test_no_gpu_means_loud_failure():
    with pytest.raises(_abi.RunError) as ei:
        api.Compactor(0)
    assert ei.value.code in (_abi.SKV_E_DEVICE, _abi.SKV_E_INVALID_ARG)
