"""The C-ABI library loads and exports every symbol include/ccg.h declares
(no compute: this runs without a GPU)."""
import ctypes
import os
import shutil
import subprocess

import pytest

from consensusclustr_amd import _lib


def test_header_declares_expected_entry_points():
    syms = _lib.header_symbols()
    for s in ("ccg_open", "ccg_knn_boot", "ccg_knn_rows_dev", "ccg_snn", "ccg_snn_dev", "ccg_silhouette",
              "ccg_select_mapback_dev", "ccg_cocluster", "ccg_cocluster_dev", "ccg_consensus_knn",
              "ccg_consensus_knn_assign", "ccg_consensus_knn_assign_dev", "ccg_check_errors", "ccg_timing_read",
              "ccg_group_open", "ccg_group_open_rank", "ccg_group_unique_id", "ccg_allgather_columns",
              "ccg_cocluster_sharded_dev", "ccg_consensus_knn_sharded_dev", "ccg_row_slabs", "ccg_boot_shard"):
        assert s in syms


def test_library_exports_every_header_symbol():
    lib = _lib.load()
    missing = [s for s in _lib.header_symbols() if not hasattr(lib, s)]
    assert not missing
    assert set(_lib.header_symbols()) <= set(_lib.SIGNATURES)


def test_nm_exports_are_extern_c():
    out = subprocess.check_output(["nm", "-D", "--defined-only", _lib.LIB_PATH]).decode()
    names = {line.split()[-1] for line in out.splitlines() if " T " in line}
    for s in _lib.header_symbols():
        assert s in names, f"{s} not exported unmangled"


def test_abi_version_and_error_path():
    lib = _lib.load()
    assert lib.ccg_abi_version() == 7
    # NULL out-pointer: rejected before any device work, message set
    assert lib.ccg_open(None, None) == _lib.CCG_EINVAL
    assert b"NULL" in lib.ccg_last_error()


def test_library_is_gfx950_code_object(tmp_path):
    # (--offloading extracts the bundled code objects next to its input: run it on a copy)
    lib = tmp_path / "libccg.so"
    shutil.copyfile(_lib.LIB_PATH, lib)
    out = subprocess.check_output(["/opt/rocm/lib/llvm/bin/llvm-objdump", "--offloading", str(lib)],
                                  stderr=subprocess.STDOUT, cwd=tmp_path).decode(errors="replace")
    assert "gfx950" in out


def test_no_cpu_fallback_when_library_missing(tmp_path, monkeypatch):
    monkeypatch.setattr(_lib, "LIB_PATH", str(tmp_path / "libccg.so"))
    monkeypatch.setattr(_lib, "_LIB", None)
    with pytest.raises(ImportError):
        _lib.load()


def test_consts_match_header():
    text = open(_lib.HEADER_PATH).read()
    for name in ("CCG_EINVAL", "CCG_ECAP", "CCG_ENAN", "CCG_SNN_RANK", "CCG_MODE_GRANULAR"):
        assert name in text
    assert f"CCG_COCLUSTER_ROW_ALIGN {_lib.COCLUSTER_ROW_ALIGN}" in text


def test_library_links_rccl():
    out = subprocess.check_output(["readelf", "-d", _lib.LIB_PATH]).decode()
    assert "librccl.so" in out  # the device group's collectives are RCCL, inside the library


def _header_prototypes():
    """name -> list of parameter type strings, from include/ccg.h."""
    import re
    text = open(_lib.HEADER_PATH).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    out = {}
    for m in re.finditer(r"^\s*(?:int|int64_t|const char\*|void\*)\s+(ccg_\w+)\s*\(([^)]*)\)\s*;", text, re.M | re.S):
        args = " ".join(m.group(2).split())
        out[m.group(1)] = [] if args in ("", "void") else [a.strip() for a in args.split(",")]
    return out


def test_ctypes_signatures_match_header_prototypes():
    """Every SIGNATURES entry has the header's parameter count, and each
    integer parameter has the header's width (pointers are opaque)."""
    protos = _header_prototypes()
    for name, (_, args) in _lib.SIGNATURES.items():
        params = protos[name]
        assert len(args) == len(params), (name, len(args), len(params))
        for a, p in zip(args, params):
            if "*" in p:
                assert a is ctypes.c_void_p, (name, p)
            elif p.startswith(("int64_t", "const int64_t")):
                assert a is ctypes.c_int64, (name, p)
            elif p.startswith("int "):
                assert a is ctypes.c_int, (name, p)
