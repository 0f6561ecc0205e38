"""CPU-side checks of the C ABI library: it loads, exports every entry point
include/pokec_fas.h declares, and refuses to run without a GPU (no CPU fallback)."""
import ctypes
import os
import re

import numpy as np
import pytest

import pokec_testlib as tl


def header_functions(name="pokec_fas.h"):
    """Entry points a header declares (its static inline helpers are compiled into the caller)."""
    with open(os.path.join(tl.ROOT, "include", name)) as f:
        src = f.read()
    inline = set(re.findall(r"static inline [^(]*\b(pf_[a-z_]+)\s*\(", src))
    return sorted(set(re.findall(r"\b(pf_[a-z_]+)\s*\(", src)) - inline)


def test_library_exports_every_declared_symbol():
    pf = tl.product()
    L = pf.lib()
    names = header_functions()
    assert len(names) >= 15
    for n in names:
        assert hasattr(L, n), n
    assert sorted(pf.EXPORTS) == names
    io = [n for n in header_functions("pokec_io.h") if n not in names]  # minus pokec_fas.h names it cites
    for n in io:
        assert hasattr(L, n), n
    assert sorted(pf.IO_EXPORTS) == io
    assert L.pf_abi_version() == 2


def _key(score, uid):
    b = int(np.float32(score).view(np.uint32))
    if b & 0x7FFFFFFF == 0:
        b = 0
    ordv = (~b & 0xFFFFFFFF) if b & 0x80000000 else (b | 0x80000000)
    return ((~ordv & 0xFFFFFFFF) << 32) | ((uid & 0xFFFFFFFF) ^ 0x80000000)


def test_key_order_matches_reference_comparator():
    pf = tl.product()
    items = [(0.5, 7), (0.5, 3), (0.75, 9), (0.0, 1), (0.25, -4), (0.25, 2)]
    keys = np.array(sorted(_key(s, u) for s, u in items) + [2**64 - 1], np.uint64)
    uids, scores = pf.decode_keys(keys)
    ref = sorted(items, key=lambda x: (-x[0], x[1]))
    assert list(uids) == [u for _, u in ref]
    assert list(scores) == [np.float32(s) for s, _ in ref]


def test_open_without_gpu_fails_loudly():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    pf = tl.product()
    c = tl.golden_corpus("B")
    with pytest.raises(pf.FasError):
        pf.FasEngine(c.desc_ptr(), 0)
