"""The C-ABI library loads and exports every symbol include/gmagg.h declares.

CPU only: no compute calls (there is no GPU here); calls that need a device must
fail cleanly with a status code and a message, never crash.
"""
import ctypes as C
import os
import re
import subprocess

import pytest

from conftest import ROOT
from byzantine_aircomp_amd import _lib

HEADER = os.path.join(ROOT, "include", "gmagg.h")


def declared_functions():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\s*\*?\s*(gm_\w+)\s*\(", text, flags=re.M)))


def test_header_declares_the_boundary():
    names = declared_functions()
    for must in ("gm_weiszfeld_f32", "gm_oma_philox_f32", "gm_oma_apply_f32", "gm_ctx_create",
                 "gm_ctx_destroy", "gm_last_error"):
        assert must in names


def test_library_exports_every_declared_symbol():
    lib = _lib.load()
    for name in declared_functions():
        assert hasattr(lib, name), name
    bound = {n for n, _, _ in _lib.SIGNATURES}
    assert set(declared_functions()) == bound


def test_exports_are_c_linkage():
    out = subprocess.run(["nm", "-D", "--defined-only", _lib.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    syms = {line.split()[-1] for line in out.splitlines() if line.strip()}
    for name in declared_functions():
        assert name in syms, f"{name} not exported with C linkage"


def test_library_is_gfx950_code_object():
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", _lib.LIB_PATH],
                         capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("llvm-objdump --offloading unavailable")
    assert "gfx950" in out.stdout + out.stderr


def test_struct_layouts_match_header(tmp_path):
    """ctypes' view of gm_opts / gm_result == the C compiler's (gcc on the header)."""
    fields = [f for f, _ in _lib.GmOpts._fields_]
    rfields = [f for f, _ in _lib.GmResult._fields_]
    src = ["#include <stdio.h>", "#include <stddef.h>", '#include "gmagg.h"', "int main(void){",
           'printf("%zu\\n", sizeof(gm_opts));', 'printf("%zu\\n", sizeof(gm_result));']
    src += [f'printf("%zu\\n", offsetof(gm_opts, {f}));' for f in fields]
    src += [f'printf("%zu\\n", offsetof(gm_result, {f}));' for f in rfields]
    src += ["return 0;}"]
    (tmp_path / "layout.c").write_text("\n".join(src))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-I", os.path.join(ROOT, "include"), str(tmp_path / "layout.c"),
                    "-o", str(exe)], check=True)
    got = [int(x) for x in subprocess.run([str(exe)], capture_output=True, text=True,
                                          check=True).stdout.split()]
    want = [C.sizeof(_lib.GmOpts), C.sizeof(_lib.GmResult)]
    want += [getattr(_lib.GmOpts, f).offset for f in fields]
    want += [getattr(_lib.GmResult, f).offset for f in rfields]
    assert got == want


def test_errors_are_reported_not_raised():
    lib = _lib.load()
    assert lib.gm_abi_version() == _lib.ABI_VERSION
    rc = lib.gm_weiszfeld_f32(None, None, 0, 0, 0, None, None, None, None, None)
    assert rc == -1
    assert b"NULL" in lib.gm_last_error()
    rc = lib.gm_ctx_set_shard(None, 10, 0)
    assert rc == -1


def test_panel_width_table():
    """gm_panel_width is the streaming tile's chunk width (no GPU needed)."""
    lib = _lib.load()
    assert lib.gm_panel_width(0) == 0
    assert lib.gm_panel_width(1000) == 32
    assert lib.gm_panel_width(50) in (64, 128, 256)
    assert lib.gm_panel_width(4096) == 0
    for K in (1, 16, 17, 100, 256, 257, 600, 1024, 2048):
        W = lib.gm_panel_width(K)
        assert W > 0 and 256 % W == 0          # shard boundaries (256-aligned) stay on panels


def _disassemble_bundle(tmp_path, src_index):
    """The gfx950 code object of the library's `src_index`-th source (Makefile SRCS order),
    disassembled."""
    import glob
    import shutil
    lib = tmp_path / "lib.so"
    shutil.copy(_lib.LIB_PATH, lib)
    subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                   capture_output=True, text=True, cwd=tmp_path)
    co = sorted(glob.glob(str(tmp_path / f"lib.so.{src_index}.hipv4-amdgcn-amd-amdhsa--gfx950")))
    if not co:
        pytest.skip("llvm-objdump --offloading unavailable")
    out = subprocess.run(["/opt/rocm/lib/llvm/bin/llvm-objdump", "-d", "--mcpu=gfx950", co[0]],
                         capture_output=True, text=True, check=True).stdout
    return out


def test_resident_granule_store_flavours(tmp_path):
    """The single-problem resident kernel's exchange contract (resident.hip put_value /
    gather_value), pinned in the ISA it was measured on: granules are published with ONE
    8-byte vector store — `sc0` (workgroup scope: the line stays in the XCD's L2; gfx950's
    vector L1 is write-through, so the store reaches that L2) when the check-in confirmed
    one XCD, `sc1` (agent scope) otherwise — and polled with `sc1` vector loads, which miss
    the L1 and are served by the L2 the writers share.  A compiler that lowered the scoped
    stores differently would change the measured exchange (and its correctness argument):
    this fails first, on the CPU."""
    import re
    dis = _disassemble_bundle(tmp_path, 2)          # resident.hip (Makefile SRCS order)
    funcs = re.split(r"\n(?=[0-9a-f]+ <)", dis)
    res = [f for f in funcs if "weiszfeld_resident" in f.split("\n", 1)[0]]
    assert res, "no weiszfeld_resident kernel in the resident.hip code object"
    for f in res:
        name = f.split("\n", 1)[0]
        stores = re.findall(r"global_store_dwordx2 [^\n]*", f)
        assert any(re.search(r"\bsc0\b", s) and not re.search(r"\bsc1\b", s) for s in stores), name
        assert any(re.search(r"\bsc1\b", s) for s in stores), name
        polls = re.findall(r"global_load_dwordx2 [^\n]*", f)
        assert polls and all(re.search(r"\bsc1\b", p) for p in polls), name
