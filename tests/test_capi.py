"""The C-ABI library builds, loads and exports every symbol include/pyrope_ann.h declares.

CPU-only: no compute call reaches a GPU here.  Where no device exists the product
path must fail loudly (PYR_E_DEVICE), never fall back to the CPU.
"""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "pyrope_ann.h")


def _declared():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(pyr_[a-z0-9_]+)\s*\(", text)))


def test_header_declares_the_boundary():
    names = _declared()
    for must in ["pyr_index_create", "pyr_index_add", "pyr_index_upsert", "pyr_index_remove", "pyr_index_build",
                 "pyr_index_search", "pyr_index_search_device", "pyr_index_stats", "pyr_index_get_centroids",
                 "pyr_merge_topk_device", "pyr_last_error"]:
        assert must in names


def test_library_exports_every_declared_symbol(hiplib):
    for name in _declared():
        assert hasattr(hiplib, name), name


def test_binding_covers_every_declared_symbol():
    from pyrope_amd import _lib
    assert set(_declared()) == set(_lib.SIGNATURES), set(_declared()) ^ set(_lib.SIGNATURES)


def test_version(hiplib):
    assert b"gfx950" in hiplib.pyr_version()


def test_generate_synthetic_matches_oracle(hiplib, oracle):
    from pyrope_amd import generate_synthetic
    np.testing.assert_array_equal(generate_synthetic(100, 16, 42), oracle.generate_vectors(100, 16, 42))
    np.testing.assert_array_equal(generate_synthetic(3, 5, 1337), oracle.generate_vectors(3, 5, 1337))


def test_generate_synthetic_blocked_matches_oracle(hiplib, oracle):
    """Row-blocked generator: block b = the Random(seed + b) sequence; any row
    range, including ranges that start or end inside a block, equals the per-block oracle rows."""
    from pyrope_amd import generate_synthetic, generate_synthetic_blocked
    B, D = 37, 6
    full = np.concatenate([oracle.generate_vectors(B, D, 42 + b) for b in range(5)])
    for r0, n in [(0, 5 * B), (0, 10), (13, 60), (B, B), (2 * B + 5, 2 * B - 5), (4 * B + 36, 1)]:
        np.testing.assert_array_equal(generate_synthetic_blocked(r0, n, D, 42, B), full[r0:r0 + n])
    # within one block it is the plain generator
    np.testing.assert_array_equal(generate_synthetic_blocked(0, 50, 16, 42), generate_synthetic(50, 16, 42))


def _has_gpu():
    try:
        import torch
        return torch.cuda.device_count() > 0
    except Exception:
        return False


@pytest.mark.skipif(_has_gpu(), reason="checks the no-device failure path")
def test_no_device_fails_loudly(hiplib):
    from pyrope_amd import BruteForceVectorIndex, DeviceError, VectorMetric, kmeans_train
    with pytest.raises(DeviceError):
        BruteForceVectorIndex(4, VectorMetric.L2)
    with pytest.raises(DeviceError):
        kmeans_train(np.zeros((4, 4), np.float32), 2, VectorMetric.L2)


def test_null_arguments_are_rejected(hiplib):
    from pyrope_amd import _lib
    assert hiplib.pyr_index_create(None, None) == _lib.PYR_E_ARG
    assert b"null" in hiplib.pyr_last_error()
    assert hiplib.pyr_index_search(None, None, 0, 10, None, None, None, None) == _lib.PYR_E_ARG
    assert hiplib.pyr_merge_topk_device(None, None, 1, 0, 10, None, None, None) == _lib.PYR_E_ARG
    assert hiplib.pyr_generate_synthetic(-1, 4, 1, None) == _lib.PYR_E_ARG
    hiplib.pyr_index_destroy(None)  # no-op


def test_status_mapping():
    from pyrope_amd import _lib
    for st, exc in [(_lib.PYR_E_DIM, _lib.ArgumentException), (_lib.PYR_E_DUPLICATE, _lib.InvalidOperationException),
                    (_lib.PYR_E_STATE, _lib.InvalidOperationException), (_lib.PYR_E_DEVICE, _lib.DeviceError)]:
        with pytest.raises(exc):
            _lib.check(st)
    _lib.check(_lib.PYR_OK)


def _image(path, sections):
    """a hand-written image (persist.h layout): header, then (tag, payload) sections padded to 8 bytes"""
    import struct
    with open(path, "wb") as f:
        f.write(b"PYRIDX01" + struct.pack("<iiiiI", 1, 0, 4, 0, len(sections)))
        for tag, payload in sections:
            f.write(struct.pack("<IIQ", tag, 0, len(payload)) + payload + b"\0" * (-len(payload) % 8))


def test_image_nonce_reads_the_nonce_section(hiplib, tmp_path):
    """pyr_image_nonce (host only, no device): the T_NONCE section's 16 bytes; zeros for an image
    written without one; PYR_E_NOT_FOUND / PYR_E_FORMAT like pyr_index_load."""
    from pyrope_amd import _lib
    out = (C.c_uint8 * 16)()
    nonce = bytes(range(7, 23))
    p = str(tmp_path / "a")
    _image(p, [(8, b"\1" * 8), (13, nonce)])
    assert hiplib.pyr_image_nonce(p.encode(), out) == _lib.PYR_OK
    assert bytes(out) == nonce
    _image(p, [(8, b"\1" * 8)])
    assert hiplib.pyr_image_nonce(p.encode(), out) == _lib.PYR_OK
    assert bytes(out) == b"\0" * 16
    assert hiplib.pyr_image_nonce(str(tmp_path / "missing").encode(), out) == _lib.PYR_E_NOT_FOUND
    open(p, "wb").write(b"not an image")
    assert hiplib.pyr_image_nonce(p.encode(), out) == _lib.PYR_E_FORMAT


def test_struct_layouts_match_the_header(tmp_path):
    """pyr_index_desc / pyr_search_params as a C compiler lays them out (the C# shim's StructLayout.Sequential
    mirrors them) equal the ctypes binding's: size and every field offset."""
    import subprocess

    from pyrope_amd import _lib
    fields = {"pyr_index_desc": _lib.IndexDesc, "pyr_search_params": _lib.SearchParams}
    body = []
    for cname, ct in fields.items():
        body.append(f'printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in ct._fields_:
            body.append(f'printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    src = tmp_path / "layout.c"
    src.write_text('#include <stddef.h>\n#include <stdio.h>\n#include "pyrope_ann.h"\nint main(void) {\n' +
                   "\n".join(body) + "\nreturn 0;\n}\n")
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-I", os.path.join(ROOT, "include"), str(src), "-o", str(exe)], check=True)
    got = dict(line.split() for line in subprocess.run([str(exe)], check=True, capture_output=True,
                                                       text=True).stdout.splitlines())
    for cname, ct in fields.items():
        assert int(got[cname]) == C.sizeof(ct), cname
        for f, _ in ct._fields_:
            assert int(got[f"{cname}.{f}"]) == getattr(ct, f).offset, (cname, f)
