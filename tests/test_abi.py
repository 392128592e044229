"""The C-ABI library loads and exports every entry point include/gaphuff.h
declares; without a GPU the decoder fails loudly (no CPU fallback)."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared():
    src = open(os.path.join(ROOT, "include", "gaphuff.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gh_[a-z0-9_]+)\s*\(", src)))


def test_header_lists_expected_entry_points(gh):
    assert set(declared()) == set(gh.EXPORTED)


def test_library_exports_all(gh):
    lib = ctypes.CDLL(gh.LIB_PATH)
    for name in declared():
        assert hasattr(lib, name), name


def test_version_and_error_strings(gh):
    assert b"gfx950" in gh.lib().gh_version()
    assert isinstance(gh.lib().gh_last_error(), bytes)


def test_no_gpu_fails_loudly(gh):
    if gh.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(gh.GapHuffError) as e:
        gh.Decoder(0)
    assert e.value.code == -5
    img = gh.encode(gh.generate(1, 0.5, 1000))
    with pytest.raises(gh.GapHuffError):
        gh.decode(img)


def test_no_gpu_encoder_fails_loudly(gh):
    if gh.device_count() > 0:
        pytest.skip("a GPU is visible")
    with pytest.raises(gh.GapHuffError) as e:
        gh.Encoder(0)
    assert e.value.code == -5
    with pytest.raises(gh.GapHuffError):
        gh.encode_gpu(gh.generate(1, 0.5, 1000))
